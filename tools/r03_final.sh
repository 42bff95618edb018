# usage (GPU box): bash tools/r03_final.sh <tag> [stages]
# the round's evidence: GPU tests, smoke, the default bench line (KT + its K2 block, CPU
# baselines, rounds to target), a rocprofv3 kernel trace + stats of the same bench, the
# K3..K5 and K2-dpsgd lines.  stages: any of t (tests) s (smoke) b (bench) p (profile)
# k (K3..K5, K2-dpsgd lines); default "tsbpk".
set -e
TAG=${1:-final}
ST=${2:-tsbpk}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [[ $ST == *t* ]]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
fi
if [[ $ST == *s* ]]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
fi
if [[ $ST == *b* ]]; then
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
fi
if [[ $ST == *p* ]]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $OUT/prof > $OUT/trace_summary.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
fi
if [[ $ST == *k* ]]; then
for C in K3 K4 K5 K2-dpsgd; do
  timeout -k 10 500 python bench.py --config $C --rounds-target 0 --steps 3 --warmup 1 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
done
fi
