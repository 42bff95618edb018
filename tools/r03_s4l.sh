# usage (GPU box): bash tools/r03_s4l.sh <tag> — BM=32 direct-conv tiles with CK=4 (34 KB of LDS,
# ~124 registers: four workgroups per CU instead of three): full-width step traces with CK=8 / 4,
# then KT / K3 interleaved A/B
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -1 $O/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
for ck in 8 4; do
  FH_DCONV_CK32=$ck timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fs_ck$ck -o run -- python3 $GRAFT_REPO_ROOT/tools/fullstep.py cifar10_cnn 23 12 > $O/fs_ck$ck.log 2>&1
  python3 $GRAFT_REPO_ROOT/tools/fullstep.py --breakdown $O/fs_ck$ck > $O/fs_ck${ck}_breakdown.txt 2>&1
  head -16 $O/fs_ck${ck}_breakdown.txt
done
cd $GRAFT_REPO_ROOT
CONFIGS="KT K3" REPS=2 bash tools/r03_ab.sh $T FH_DCONV_CK32=8 FH_DCONV_CK32=4
