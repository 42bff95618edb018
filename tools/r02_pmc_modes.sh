# usage (GPU box): bash tools/r02_pmc_modes.sh <tag>
# FETCH_SIZE passes of the default bench (lanes on) under different launch settings, to
# locate the program-mode crash under rocprofv3 --pmc: (1) lanes replaying HIP graphs,
# (2) step programs with every lane at the default stream priority
set -e
TAG=${1:-pmcmodes}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT/graph $OUT/prog_noprio
cd /tmp && export TMPDIR=/tmp
FH_LAUNCH=graph timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/graph -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $OUT/graph/bench.json 2> $OUT/graph/log.txt
FH_LANE_PRIO=0,0,0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prog_noprio -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $OUT/prog_noprio/bench.json 2> $OUT/prog_noprio/log.txt
