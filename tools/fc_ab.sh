# usage (GPU box): bash tools/fc_ab.sh <tag> — linear-layer parity tests, fc_bench skinny vs
# implicit GEMM, KT bench A/B
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
for v in 1 0; do
  FH_LINEAR_SKINNY=$v timeout -k 10 200 python -u tools/fc_bench.py > $OUT/fc_$v.txt 2>&1
  echo "== skinny $v"; grep "^C=" $OUT/fc_$v.txt
done
bash tools/ab_bench.sh $1/ab skinny=FH_X=0 igemm=FH_LINEAR_SKINNY=0
