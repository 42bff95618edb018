# usage (GPU box): bash tools/dpsgd_check.sh <tag> — DP-SGD tests, the K2-dpsgd bench line and
# its rocprofv3 kernel trace + summary
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dpsgd_gpu.py -x -v --timeout 120 --timeout-method thread > $O/dpsgd_tests.log 2>&1 || { tail -40 $O/dpsgd_tests.log; exit 1; }
tail -1 $O/dpsgd_tests.log
timeout -k 10 300 python bench.py --config K2-dpsgd --steps 5 --warmup 1 --detail-out $O/detail_K2-dpsgd.json > $O/bench_K2-dpsgd.json 2> $O/bench_K2-dpsgd.err
python -c "import json; d=json.loads(open('$O/bench_K2-dpsgd.json').read().strip().splitlines()[-1]); print('K2-dpsgd', d['value'], d['round_frac'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config K2-dpsgd --steps 3 --warmup 1 --no-cpu-baseline --detail-out '' > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof_bench.err
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $GRAFT_REPO_ROOT/$O/prof > $GRAFT_REPO_ROOT/$O/trace_summary_dpsgd.txt
head -16 $GRAFT_REPO_ROOT/$O/trace_summary_dpsgd.txt
