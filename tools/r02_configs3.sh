# usage (GPU box): bash tools/r02_configs3.sh <tag>
# full GPU tests, then one bench line per BASELINE config (K2..K5 slices, no baselines)
set -e
TAG=${1:-cfg}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
for C in K2 K3 K4 K5; do
  timeout -k 10 400 python bench.py --config $C --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  python -c "import json; d=json.load(open('$OUT/bench_$C.json')); print('$C', d['value'], d['ms_per_step'], d['round_frac'], d['roofline']['kernel'], d['roofline']['frac'])" | tee -a $OUT/summary.txt
done
