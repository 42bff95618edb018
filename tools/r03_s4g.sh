# usage (GPU box): bash tools/r03_s4g.sh <tag> — BN glue kernels (two quads per thread in the BN
# backward apply, 8 windows per thread in the pooled BN finalize): BN / layer tests, a full-width
# step trace, KT lines, one KT round with the lanes' GPU step-end timeline (FH_HOST_TIMING)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py tests/test_fuse_bn_gpu.py tests/test_graph_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fullstep -o run -- python3 $GRAFT_REPO_ROOT/tools/fullstep.py cifar10_cnn 32 12 > $O/fullstep.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/fullstep.py --breakdown $O/fullstep > $O/fullstep_breakdown.txt 2>&1
head -20 $O/fullstep_breakdown.txt
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py --config KT --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 --no-instances --no-k2 > $O/b_KT_$i.json 2>/dev/null
  python -c "import json; d=json.loads(open('$O/b_KT_$i.json').read().strip().splitlines()[-1]); print('KT', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
done
FH_HOST_TIMING=1 timeout -k 10 300 python bench.py --config KT --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --no-k2 > $O/timing.json 2> $O/timing.err
grep -E "lane|host issue" $O/timing.err | tail -12
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('default line: KT', d['value'], d['round_frac'], 'K2 block', d['k2']['value'], d['k2']['round_frac'])"
