# usage (GPU box): bash tools/r03_s4d.sh <tag> — in-launch split sums: conv tests, the GPU
# suite, then KT / K2 interleaved A/B against the splitk_epilogue launch (FH_DCONV_INK=0)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/conv_tests.log 2>&1
tail -1 $O/conv_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
CONFIGS="KT K2" REPS=2 bash tools/r03_ab.sh $T FH_DCONV_INK=4 FH_DCONV_INK=0
