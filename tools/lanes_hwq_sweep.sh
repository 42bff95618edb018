# usage (GPU box): bash tools/lanes_hwq_sweep.sh <tag> — KT bench (program launch mode) over
# lane counts and HIP hardware-queue counts
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --rounds-target 0 --steps 5 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name FAILED"; tail -3 $OUT/$name.err; return 0; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['config'].get('lanes'))"
}
run l3q4 FH_LANES=3
run l3q8 FH_LANES=3 GPU_MAX_HW_QUEUES=8
run l4q8 FH_LANES=4 GPU_MAX_HW_QUEUES=8
run l5q8 FH_LANES=5 GPU_MAX_HW_QUEUES=8
run l6q8 FH_LANES=6 GPU_MAX_HW_QUEUES=8
run l8q12 FH_LANES=8 GPU_MAX_HW_QUEUES=12
run l4q8p FH_LANES=4 GPU_MAX_HW_QUEUES=8 FH_LANE_PRIO=-1,0,0,0
