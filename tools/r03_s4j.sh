# usage (GPU box): bash tools/r03_s4j.sh <tag> — narrow-lane knobs: deferral tests, then K2 / KT
# interleaved A/B (in-launch split sums for the 1-client / narrow lanes, min stages per split,
# classifier-forward chunking)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_defer_wgrad_gpu.py tests/test_fuse_pool1_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
CONFIGS="K2 KT" REPS=2 bash tools/r03_ab.sh $T FH_NOOP=1 FH_SPLIT_TICKETS_FILL=0.25 FH_SPLIT_TICKETS_FILL=0.5 FH_DCONV_MINSTAGES=2 FH_LF_MINKB=2
