# usage (GPU box): bash tools/stream_sweep.sh <tag> — KT bench under lane-stream dispatch
# variants: default streams, lane-0 priority, CU masks reserving CUs for lane 0
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --rounds-target 0 --steps 5 > $OUT/$name.json 2> $OUT/$name.err
  python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
run base FH_X=0
run prio FH_LANE_PRIO=-1,0,0
run prio2 FH_LANE_PRIO=-1,0,1
run cu32s FH_LANE_CU=32
run cu64s FH_LANE_CU=64
run cu32b FH_LANE_CU=32 FH_LANE_CU_LAYOUT=block
run cu16s FH_LANE_CU=16
