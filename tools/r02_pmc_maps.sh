# usage (GPU box): bash tools/r02_pmc_maps.sh <tag>
# one rocprofv3 --pmc FETCH_SIZE run of the bench that crashes, with the process's memory
# map written just before the first round (to place the faulting PC and address)
TAG=${1:-pmcmaps}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
FH_DUMP_MAPS=$OUT/maps.txt timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $OUT/bench.json 2> $OUT/log.txt
echo "rc=$?"
exit 0
