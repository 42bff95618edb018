# usage (GPU box): bash tools/r03_s4z.sh <tag> A|B — round-3 session-4 evidence of the final tree.
# A: GPU tests, smoke, the default bench line (KT + K2 block, CPU baselines, rounds to target),
#    a rocprofv3 kernel trace + stats of the same bench (no host legs).
# B: the K3 / K4 / K5 / K2-dpsgd lines, then separate rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE
#    passes of the KT bench for roofline.traffic (tools/bench_traffic.py).
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$2" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
  timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
  python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('KT', d['value'], d['round_frac'], d['roofline']['kernel'], d['roofline']['frac'], 'K2', d['k2']['value'], d['k2']['round_frac'])"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 > $O/prof_bench.json 2> $O/prof_bench.err
  python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/prof > $O/trace_summary.txt 2>&1 || true
  head -5 $O/trace_summary.txt
else
  for C in K3 K4 K5 K2-dpsgd; do
    timeout -k 10 500 python bench.py --config $C --rounds-target 0 --steps 3 --warmup 1 > $O/bench_$C.json 2> $O/bench_$C.err
    python -c "import json; d=json.loads(open('$O/bench_$C.json').read().strip().splitlines()[-1]); print('$C', d['value'], d['round_frac'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --no-k2 > $O/pmc_fetch.json 2> $O/pmc_fetch.log
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --no-k2 > $O/pmc_write.json 2> $O/pmc_write.log
  python3 $GRAFT_REPO_ROOT/tools/bench_traffic.py $O/pmc_fetch $O/pmc_write $O/bench_traffic.json > $O/bench_traffic.log 2>&1 || true
  tail -5 $O/bench_traffic.log
fi
