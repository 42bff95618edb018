# usage (GPU box): bash tools/ab_tree.sh <tag> <config> <other-tree> [rounds] — interleaved
# bench of this tree and another checkout (regression hunting)
set -e
TAG=$1; CFG=$2; OTHER=$3; R=${4:-2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $R); do
  for T in . $OTHER; do
    (cd $GRAFT_REPO_ROOT/$T && timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --rounds-target 0 --no-instances --steps ${STEPS:-5} --warmup 1 > $OUT/b_${i}_$(basename $T).json 2> $OUT/b_${i}_$(basename $T).err)
    python -c "import json; d=json.load(open('$OUT/b_${i}_$(basename $T).json')); print('$CFG $T', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
