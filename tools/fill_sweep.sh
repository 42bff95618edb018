# GPU box: split-K fill-fraction sweep of the laned KT bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fill
timeout -k 10 300 python -u -m pytest tests/test_lanes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fill/tests.log 2>&1
for F in "$@"; do
  FH_LANE_FILL=$F timeout -k 10 200 python bench.py --no-cpu-baseline --rounds-target 0 > gpurun_out/fill/F$F.json 2>gpurun_out/fill/F$F.err
done
