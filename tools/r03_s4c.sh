# usage (GPU box): bash tools/r03_s4c.sh <tag> — conv tests, a full-width step trace, KT / K2 lines
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_fuse_bn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fullstep -o run -- python3 $GRAFT_REPO_ROOT/tools/fullstep.py cifar10_cnn 32 12 > $O/fullstep.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/fullstep.py --breakdown $O/fullstep > $O/fullstep_breakdown.txt 2>&1
head -14 $O/fullstep_breakdown.txt
cd $GRAFT_REPO_ROOT
for C in KT K2 KT K2; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 --no-instances --no-k2 > $O/b_$C.json 2>/dev/null
  python -c "import json; d=json.loads(open('$O/b_$C.json').read().strip().splitlines()[-1]); print('$C', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
done
