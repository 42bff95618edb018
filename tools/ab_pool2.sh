set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_pool2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fuse_pool2_gpu.py tests/test_fuse_pool1_gpu.py tests/test_dpsgd_gpu.py tests/test_configs_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python tools/ab_attr.py fuse_pool2=$v -- --config K2 --steps 20 --warmup 5 --no-cpu-baseline --rounds-target 0 --no-instances --detail-out '' > $O/k2_${v}_${i}.json 2>$O/k2.err
    python -c "import json; d=json.loads(open('$O/k2_${v}_${i}.json').read().strip().splitlines()[-1]); print('fuse_pool2=$v', d['value'], d['ms_per_step'])"
  done
done
