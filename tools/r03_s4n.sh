# usage (GPU box): bash tools/r03_s4n.sh <tag> — in-launch split sums for the narrow lanes now also
# in the classifier forward: classifier / conv / deferral tests, then K2 / KT interleaved x3:
# default, FH_SPLIT_TICKETS_FILL=0 (separate reduction launches), FH_FUSE_POOL2_BWD=1
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_classifier_gpu.py tests/test_conv_gpu.py tests/test_defer_wgrad_gpu.py tests/test_lanes_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
CONFIGS="K2 KT" REPS=3 bash tools/r03_ab.sh $T FH_NOOP=1 FH_SPLIT_TICKETS_FILL=0 FH_FUSE_POOL2_BWD=1
