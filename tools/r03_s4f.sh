# usage (GPU box): bash tools/r03_s4f.sh <tag> — the default bench line (KT + K2 block, host legs
# last), then a KT lane fill / cut re-sweep on the r03 s4 kernels (interleaved x2)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('KT', d['value'], d['round_frac'], 'K2', d['k2']['value'], d['k2']['round_frac'])"
CONFIGS="KT" REPS=2 bash tools/r03_ab.sh $T FH_NOOP=1 FH_LANE_FILL=0.5,0.5,0.75 FH_LANE_FILL=0.25,0.5,1.0 FH_LANE_FILL=0.25,0.75,0.75 FH_LANE_CUT=0,1,6,32 FH_LANE_CUT=0,1,12,32 FH_LANE_CUT=0,2,9,32
