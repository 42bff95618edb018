# usage (GPU box): REPS=2 STEPS=10 bash tools/ab_env.sh <tag> "<configs>" "<env assignments>"...
# — bench lines of each environment variant ("-" = none), interleaved REPS times per config
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
CONFIGS=$2; shift 2
for C in $CONFIGS; do
  for rep in $(seq 1 ${REPS:-2}); do
    i=0
    for v in "$@"; do
      i=$((i+1)); E=""; [ "$v" != "-" ] && E="$v"
      env $E timeout -k 10 300 python bench.py --config $C --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --rounds-target 0 --no-instances --no-k2 --no-dpsgd --detail-out '' > $O/${C}_v${i}_${rep}.json 2>> $O/ab.err || exit 1
      python -c "import json; d=json.loads(open('$O/${C}_v${i}_${rep}.json').read().strip().splitlines()[-1]); print('$C', '[$v]', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
    done
  done
done
