# GPU box: lane-cut sweep of the KT bench (tools/lanes_sweep.sh [cuts...])
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lanes
timeout -k 10 300 python -u -m pytest tests/test_lanes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lanes/tests.log 2>&1
for C in "$@"; do
  FH_LANE_CUT=$C timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/lanes/C$C.json 2>gpurun_out/lanes/C$C.err
done
