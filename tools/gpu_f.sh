# GPU box: f-row tests (eval/compression), lanes test, bench with rounds-to-target
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/f
timeout -k 10 300 python -u -m pytest tests/test_eval_compress_gpu.py tests/test_lanes_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/f/tests.log 2>&1
for S in 0.15 0.1 0.12; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --proxy-signal $S > gpurun_out/f/bench_$S.json 2> gpurun_out/f/bench_$S.err
done
