# usage (GPU box): bash tools/gpu_round.sh <tag>
# GPU tests, smoke, default bench line, and a rocprofv3 kernel-trace --stats pass of the
# same bench command; every GPU step under its own time limit, chained so a failure stops it.
set -e
TAG=${1:-round}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err
python3 $GRAFT_REPO_ROOT/tools/probe_agree.py $OUT/prof/run_kernel_trace.csv $OUT/prof_bench.json > $OUT/probe_agree.txt 2>&1 || true
echo done
