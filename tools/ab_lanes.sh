# usage (GPU box): bash tools/ab_lanes.sh <tag> <config> "<lane counts>" [reps] — interleaved
# bench lines of the same tree at different --lanes caps (the lane planner's maximum)
set -e
TAG=$1; CFG=$2; LANES=$3; R=${4:-2}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in $(seq 1 $R); do
  for L in $LANES; do
    timeout -k 10 300 python bench.py --config $CFG --lanes $L --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --rounds-target 0 --no-instances --no-k2 --detail-out '' > $O/${CFG}_L${L}_$i.json 2>> $O/lanes.err
    python -c "import json; d=json.loads(open('$O/${CFG}_L${L}_$i.json').read().strip().splitlines()[-1]); print('$CFG lanes<=$L', d['value'], d['ms_per_step'], d['config']['lanes'])" | tee -a $O/lanes.txt
  done
done
