# usage (GPU box): bash tools/r03_batch1.sh <tag> — one call, several steps (the pool is busy):
# all GPU tests; K2 A/B of pool2's backward folded into fc1 (interleaved x2); a KT line; the
# DP-SGD line + kernel trace and the SQ-counter pass of tools/r03_evidence.sh
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
CONFIG=K2 bash tools/r02_iter.sh ${T}_k2ab NONE FH_FUSE_POOL2_BWD=1 FH_FUSE_POOL2_BWD=0 FH_FUSE_POOL2_BWD=1 FH_FUSE_POOL2_BWD=0
bash tools/r02_iter.sh ${T}_kt NONE FH_NOOP=1
bash tools/r03_evidence.sh ${T}_ev
