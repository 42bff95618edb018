# usage (GPU box): bash tools/r03_s4e.sh <tag> — in-launch split sums (write-through partials):
# conv tests, then KT interleaved A/B: in-launch sum (cap 4 / 8), cap 4 with the epilogue
# launch, and the r03 epilogue launch (FH_DCONV_INK=0)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_fuse_bn_gpu.py tests/test_lanes_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
CONFIGS="KT" REPS=2 bash tools/r03_ab.sh $T FH_DCONV_INK=4 "FH_DCONV_INK=4 FH_SPLIT_TICKETS=0" FH_DCONV_INK=8 FH_DCONV_INK=0
