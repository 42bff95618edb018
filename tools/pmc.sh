# usage (GPU box): bash tools/pmc.sh <tag> "<counters>" <script.py relative to repo> [args...]
set -e
TAG=$1; shift
CTRS=$1; shift
SCRIPT=$GRAFT_REPO_ROOT/$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc $CTRS --output-format csv -d $OUT -o run -- python3 $SCRIPT "$@" > $OUT/log.txt 2>&1
