# usage (GPU box): bash tools/r02_pmc_stream.sh <tag>
# rocprofv3 --pmc FETCH_SIZE of a pure-torch workload on a non-default stream (no libfedhip)
set -e
TAG=${1:-pmcstream}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for M in stream stream_prio; do
  mkdir -p $OUT/$M
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$M -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_control.py $M > $OUT/$M/out.txt 2> $OUT/$M/log.txt
done
