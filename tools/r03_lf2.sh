# usage (GPU box): bash tools/r03_lf2.sh <tag> — skinny linear FORWARD variants timed from a
# rocprofv3 kernel trace of fc_bench (forward only)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_classifier_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "linear" > $O/tests.log 2>&1
tail -1 $O/tests.log
L="3136x128,2048x512,512x256"
CL="32,23,8,2,1"
cd /tmp && export TMPDIR=/tmp
i=0
V=("FH_LINEAR_SKINNY=3" "FH_LF_OT=4" "FH_LF_OT=1" "FH_LF_OT=2" "FH_LF_OT=1 FH_LF_DEPTH=3"
   "FH_LF_OT=1 FH_LF_TARGET=256" "FH_LF_OT=1 FH_LF_MINKB=2" "FH_LF_OT=1 FH_LF_DEPTH=1"
   "FH_LF_OT=2 FH_LF_DEPTH=3" "FH_LF_OT=1 FH_LF_TARGET=1024")
for v in "${V[@]}"; do
  i=$((i+1))
  export FH_BENCH_LAYERS=$L FH_BENCH_CLIENTS=$CL FH_BENCH_FWD_ONLY=1
  for kv in $v; do export $kv; done
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/fc_bench.py > /dev/null 2>&1
  for kv in $v; do unset ${kv%%=*}; done
  echo "== $v" >> $O/lf.txt
  python3 $GRAFT_REPO_ROOT/tools/lf_trace.py $O/p$i/run_kernel_trace.csv $CL $L >> $O/lf.txt
  rm -rf $O/p$i
done
cat $O/lf.txt
