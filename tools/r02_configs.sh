# usage (GPU box): bash tools/r02_configs.sh <tag> [configs...] — bench lines (with the
# per-launch-shape instances) of the given BASELINE configs (default K2..K5), 3 timed rounds
set -e
TAG=$1; shift
[ $# -eq 0 ] && set -- K2 K3 K4 K5
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for C in "$@"; do
  timeout -k 10 500 python bench.py --config $C --rounds-target 0 --steps 3 --warmup 1 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  python -c "import json; d=json.load(open('$OUT/bench_$C.json')); print('$C', d['value'], d['ms_per_step'], d['round_frac'], d['roofline']['kernel'], d['roofline']['frac'])" | tee -a $OUT/summary.txt
done
