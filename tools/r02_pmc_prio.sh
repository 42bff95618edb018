# usage (GPU box): bash tools/r02_pmc_prio.sh <tag>
# rocprofv3 --pmc of the default bench (lanes + step programs) with every lane stream at
# priority 0 (FH_LANE_PRIO=0): FETCH_SIZE, then WRITE_SIZE (separate runs)
set -e
TAG=${1:-pmcprio}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for CTR in FETCH_SIZE WRITE_SIZE; do
  D=$OUT/$(echo $CTR | tr A-Z a-z)
  mkdir -p $D
  FH_LANE_PRIO=0 timeout -s KILL 240 rocprofv3 --pmc $CTR --output-format csv -d $D -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $D/bench.json 2> $D/log.txt
done
