# usage (GPU box): bash tools/r03_lf.sh <tag> — skinny linear FORWARD: tests, fc_bench A/B
# (FH_LINEAR_SKINNY=3 = the implicit GEMM forward) and split-plan sweep, then K2 / KT bench A/B
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_classifier_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "linear" > $O/tests.log 2>&1
tail -1 $O/tests.log
L="3136x128,2048x512,512x256"
for v in "FH_LINEAR_SKINNY=3" "FH_LF_DEPTH=2" "FH_LF_DEPTH=3" "FH_LF_DEPTH=1" "FH_LF_TARGET=256" "FH_LF_TARGET=1024" "FH_LF_MINKB=2" "FH_LF_MINKB=8"; do
  echo "== $v" >> $O/fc.txt
  env $v FH_BENCH_LAYERS=$L FH_BENCH_CLIENTS=32,23,8,2,1 timeout -k 10 120 python tools/fc_bench.py >> $O/fc.txt 2>/dev/null
done
for i in 1 2; do
  for v in "FH_LINEAR_SKINNY=3" "FH_NOOP=1"; do
    for C in K2 KT; do
      env $v timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 --no-instances --no-k2 > $O/b_${C}_${v}_$i.json 2>/dev/null
      python -c "import json,sys; d=json.loads(open('$O/b_${C}_${v}_$i.json').read().strip().splitlines()[-1]); print('$C $v $i', d['value'], d['ms_per_step'])" >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
