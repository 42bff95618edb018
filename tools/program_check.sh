# usage (GPU box): bash tools/program_check.sh <tag> — lane parity tests, then the KT bench
# with lanes launched as step programs vs HIP graphs, and a kernel trace of the former
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_lanes_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/lanes_tests.log 2>&1
tail -1 $OUT/lanes_tests.log
for m in program graph; do
  FH_LAUNCH=$m timeout -k 10 150 python bench.py --no-cpu-baseline --rounds-target 0 --steps 5 > $OUT/$m.json 2> $OUT/$m.err
  python -c "import json; d=json.load(open('$OUT/$m.json')); print('$m', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 2 > $OUT/prof.json 2> $OUT/prof.err
