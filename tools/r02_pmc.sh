# usage (GPU box): bash tools/r02_pmc.sh <tag> <COUNTER> [bench args]
# one rocprofv3 --pmc pass (one counter) of the default bench: lanes and step programs on
TAG=$1; CTR=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/$(echo $CTR | tr A-Z a-z)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc $CTR --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 "$@" > $OUT/log.txt 2>&1
rc=$?
ls -la $OUT
exit $rc
