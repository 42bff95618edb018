# usage (GPU box): bash tools/tpb_sweep.sh <tag> — dconv tiles-per-workgroup sweep + parity
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
FH_DCONV_TPB=3 timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_fuse_bn_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_tpb3.log 2>&1
tail -1 $OUT/tests_tpb3.log
for t in 1 2 3 4; do
  FH_DCONV_TPB=$t FH_BENCH_CLIENTS=32,23,8 timeout -k 10 200 python -u tools/conv_bench.py > $OUT/tpb$t.txt 2>&1
  echo "== tpb $t"; grep "^C=" $OUT/tpb$t.txt | cut -c1-80
done
