# usage (GPU box): bash tools/ab_bench.sh <tag> NAME=ENV[+ENV..] ... — KT bench A/B, each
# variant twice, interleaved (bench.py --steps 5, no CPU baseline / rounds-to-target)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//+/ } timeout -k 10 120 python bench.py --no-cpu-baseline --rounds-target 0 --steps 5 > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "$name FAILED"; tail -3 $OUT/$name.$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$name.$rep.json')); print('$name', d['value'], d['ms_per_step'])"
  done
done
