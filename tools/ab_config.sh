# usage (GPU box): bash tools/ab_config.sh <tag> <config> NAME=ENV[+ENV..] ... — bench A/B of
# one BASELINE config (KT, K2..K5), each variant three times, interleaved (--steps 3, no CPU
# baseline / rounds-to-target / instances)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
CFG=$2
shift 2
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//+/ } timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline --rounds-target 0 --no-instances --steps ${STEPS:-3} --warmup 1 > $OUT/$CFG.$name.$rep.json 2> $OUT/$CFG.$name.$rep.err || { echo "$name FAILED"; tail -3 $OUT/$CFG.$name.$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$CFG.$name.$rep.json')); print('$CFG $name', d['value'], d['ms_per_step'], d['round_frac'])" | tee -a $OUT/summary.txt
  done
done
