# usage (GPU box): bash tools/r02_check.sh <tag> [pytest -k expr]
set -e
TAG=${1:-chk}; K=${2:-}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $OUT/gputests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputests.log 2>&1
fi
timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline --rounds-target 0 > $OUT/bench.json 2> $OUT/bench.err
