# usage (GPU box): bash tools/r02_round.sh <tag>
# the round's evidence in one call: GPU tests, smoke, the full KT bench line, a rocprofv3
# kernel trace of the same bench, then FETCH_SIZE and WRITE_SIZE PMC passes (separate runs)
# of the bench with lanes and step programs on (the default product launch path)
set -e
TAG=${1:-r02}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
for CTR in FETCH_SIZE WRITE_SIZE; do
  D=$OUT/pmc_$(echo $CTR | tr A-Z a-z)
  mkdir -p $D
  timeout -s KILL 300 rocprofv3 --pmc $CTR --output-format csv -d $D -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 > $D/bench.json 2> $D/log.txt
done
