# usage (GPU box): bash tools/r02_iterK.sh <tag> <config> "<pytest -k expr|NONE>" [ENV=VAL ...]
# r02_iter.sh for another BASELINE config's bench line
set -e
TAG=$1; CFG=$2; K=$3; shift 3
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ "$K" != "NONE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/gpu_tests.log 2>&1
fi
[ $# -eq 0 ] && set -- "FH_NOOP=1"
i=0
for E in "$@"; do
  env $E timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --rounds-target 0 --no-instances --steps ${STEPS:-5} --warmup 1 > $OUT/bench_$i.json 2> $OUT/bench_$i.err
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$CFG $E', d['value'], d['ms_per_step'], d['round_frac'])" | tee -a $OUT/summary.txt
  i=$((i+1))
done
