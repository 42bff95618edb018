# usage (GPU box): bash tools/evidence.sh <tag> [stages]
# The round's evidence, written to gpurun_out/<tag>/:
#   t  GPU tests (pytest -m gpu)
#   s  smoke()
#   b  the default bench line (KT + its K2 block, CPU baselines, rounds to target) + detail file
#   p  a rocprofv3 kernel trace + stats of the same bench (no host legs) + trace summary
#   q  the same trace of KT with each layer's WGRAD and DGRAD as separate launches
#      (--separate-conv-bwd): per-kernel averages of the dual-role launch's two roles
#   k  the K3 / K4 / K5 / K2-dpsgd lines (+ their detail files)
#   m  separate rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes of the KT bench -> the
#      per-launch-shape HBM traffic of the timed launches as they run, dual-role WGRAD + DGRAD
#      grids included (tools/bench_traffic.py)
#   n  the same two passes of the K2 config (its conv2 forward and dual-role backward)
# default stages "tsb".  Every GPU step has its own time limit and the chain stops at the
# first failure (set -e).
set -e
T=${1:-evidence}
ST=${2:-tsb}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
summ() {  # one-line summary of a bench line
  python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; k=d.get('k2') or {}; print('$2', d['value'], d.get('round_frac'), r['kernel'], r['frac'], 'K2', k.get('value'), k.get('round_frac'), 'bytes', len(open('$1').read().strip().splitlines()[-1]))"
}
if [[ $ST == *t* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
fi
if [[ $ST == *s* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
fi
if [[ $ST == *b* ]]; then
  timeout -k 10 900 python bench.py --steps 20 --warmup 5 --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err
  summ $O/bench.json KT
fi
if [[ $ST == *k* ]]; then
  for C in K3 K4 K5 K2-dpsgd; do
    timeout -k 10 500 python bench.py --config $C --rounds-target 0 --steps 3 --warmup 1 --detail-out $O/detail_$C.json > $O/bench_$C.json 2> $O/bench_$C.err
    summ $O/bench_$C.json $C
  done
fi
if [[ $ST == *p* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --rounds-target 0 --detail-out $O/prof_detail.json > $O/prof_bench.json 2> $O/prof_bench.err
  python3 $R/tools/trace_summary.py $O/prof > $O/trace_summary.txt 2>&1 || true
  head -5 $O/trace_summary.txt
  python3 $R/tools/roofline_check.py $O/prof $O/prof_detail.json > $O/roofline_check.json 2>&1 || true
  cat $O/roofline_check.json
  cd $R
fi
if [[ $ST == *q* ]]; then  # the same kernel trace with WGRAD / DGRAD as separate launches
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sep -o run -- python3 $R/bench.py --no-cpu-baseline --rounds-target 0 --no-k2 --separate-conv-bwd --detail-out '' > $O/prof_sep_bench.json 2> $O/prof_sep_bench.err
  python3 $R/tools/trace_summary.py $O/prof_sep > $O/trace_summary_sep.txt 2>&1 || true
  head -5 $O/trace_summary_sep.txt
  cd $R
fi
if [[ $ST == *m* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --no-k2 --detail-out '' > $O/pmc_fetch.json 2> $O/pmc_fetch.log
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --no-k2 --detail-out '' > $O/pmc_write.json 2> $O/pmc_write.log
  python3 $R/tools/bench_traffic.py $O/pmc_fetch $O/pmc_write $O/bench_traffic.json > $O/bench_traffic.log 2>&1 || true
  tail -5 $O/bench_traffic.log
  cd $R
fi
if [[ $ST == *n* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_k2_fetch -o run -- python3 $R/bench.py --config K2 --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --detail-out '' > $O/pmc_k2_fetch.json 2> $O/pmc_k2_fetch.log
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_k2_write -o run -- python3 $R/bench.py --config K2 --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --detail-out '' > $O/pmc_k2_write.json 2> $O/pmc_k2_write.log
  mkdir -p $O/k2
  python3 $R/tools/bench_traffic.py $O/pmc_k2_fetch $O/pmc_k2_write $O/k2/bench_traffic.json K2 > $O/bench_traffic_k2.log 2>&1 || true
  tail -5 $O/bench_traffic_k2.log
  cd $R
fi
