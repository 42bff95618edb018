# usage (GPU box): bash tools/r02_pmc2.sh <tag> <COUNTER> <clients,...>
TAG=$1; CTR=$2; CL=$3
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/$(echo $CTR | tr A-Z a-z)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc $CTR --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/tools/traffic_probe.py $CL 3 > $OUT/log.txt 2>&1
rc=$?
ls -la $OUT
exit $rc
