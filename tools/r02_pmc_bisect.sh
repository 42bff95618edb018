# usage (GPU box): bash tools/r02_pmc_bisect.sh <tag>
# rocprofv3 --pmc FETCH_SIZE over libfedhip launches in isolation (tools/pmc_bisect.py)
set -e
TAG=${1:-pmcbis}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for W in fedavg conv; do
  mkdir -p $OUT/$W
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$W -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_bisect.py $W > $OUT/$W/out.txt 2> $OUT/$W/log.txt
done
