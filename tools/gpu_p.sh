# GPU box: pipeline tests + full gpu suite + bench (uint8 pipeline vs fp32)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/p/bench_u8.json 2> gpurun_out/p/bench_u8.err
timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-data --rounds-target 0 > gpurun_out/p/bench_f32.json 2> gpurun_out/p/bench_f32.err
