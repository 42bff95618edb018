# usage (GPU box): bash tools/r02_iter.sh <tag> "<pytest -k expr|ALL|NONE>" [ENV=VAL ...]
# one development iteration: GPU tests (a -k subset, all, or none), then the KT bench line
# (no baselines, no rounds-to-target) once per env setting given (default: one plain run)
set -e
TAG=$1; K=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ "$K" = "ALL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
elif [ "$K" != "NONE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/gpu_tests.log 2>&1
fi
[ $# -eq 0 ] && set -- "FH_NOOP=1"
i=0
for E in "$@"; do
  env $E timeout -k 10 300 python bench.py --config ${CONFIG:-KT} --no-cpu-baseline --rounds-target 0 --no-instances --no-k2 --steps ${STEPS:-5} --warmup 1 > $OUT/bench_$i.json 2> $OUT/bench_$i.err
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$E', d['value'], d['ms_per_step'], d['round_frac'])" | tee -a $OUT/summary.txt
  i=$((i+1))
done
