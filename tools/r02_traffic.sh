# usage (GPU box): bash tools/r02_traffic.sh <tag>
# HBM traffic of the conv launch shapes: FETCH_SIZE and WRITE_SIZE PMC passes (separate
# runs) of the default KT bench with ONE lane, steps issued eagerly (FH_LAUNCH=eager; 2nd arg).
# With concurrent lanes every rocprofv3 --pmc run of this image segfaulted inside the
# profiler's dispatch path whatever issued the launch (step program, HIP graph replay,
# torch's device copy: profiles/r02_s2b/pmc_lanes_crash.txt); the last pass retries lanes
# on with counters restricted to the dominant kernels.
set -e
TAG=${1:-traffic}; MODE=${2:-eager}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for CTR in FETCH_SIZE WRITE_SIZE; do
  D=$OUT/lane1_$(echo $CTR | tr A-Z a-z)
  mkdir -p $D
  FH_LAUNCH=$MODE timeout -s KILL 240 rocprofv3 --pmc $CTR --output-format csv -d $D -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --lanes 1 > $D/bench.json 2> $D/log.txt
done
D=$OUT/lanes_fetch_regex
mkdir -p $D
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dconv_wgrad_kernel" --output-format csv -d $D -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $D/bench.json 2> $D/log.txt
