# usage (GPU box): bash tools/r02_pmc_bisect2.sh <tag>
# rocprofv3 --pmc FETCH_SIZE of bench.py on pre-normalised fp32 shards (no uint8 gather):
# (1) one lane, eager steps; (2) default lanes + step programs
set -e
TAG=${1:-pmcbis2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT/fp32_eager $OUT/fp32_lanes
cd /tmp && export TMPDIR=/tmp
FH_LAUNCH=eager timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fp32_eager -o run -- python3 $GRAFT_REPO_ROOT/bench.py --fp32-data --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --lanes 1 > $OUT/fp32_eager/bench.json 2> $OUT/fp32_eager/log.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fp32_lanes -o run -- python3 $GRAFT_REPO_ROOT/bench.py --fp32-data --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $OUT/fp32_lanes/bench.json 2> $OUT/fp32_lanes/log.txt
