set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w
timeout -k 10 300 python -u -m pytest tests/test_wire_gpu.py tests/test_accuracy_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w/tests.log 2>&1
bash tools/profile.sh r01_v8_prof --rounds-target 0
