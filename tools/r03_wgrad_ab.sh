# usage (GPU box): bash tools/r03_wgrad_ab.sh <tag> ["ENV=.. ENV=.." ...] — conv parity tests,
# then WGRAD per-launch timing (tools/conv_micro.py) under each environment given (default:
# the quadrant-wave kernel as built vs FH_DWGRAD_Q=0, the r02 kernel)
set -o pipefail
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_fuse_bn_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
S=${SHAPES:-"wgrad:32:32:32:3:1 wgrad:128:8:128:3:1 wgrad:64:16:64:3:1 wgrad:64:32:64:3:1 wgrad:256:8:256:3:1"}
[ $# -eq 0 ] && set -- "FH_DWGRAD_Q=1" "FH_DWGRAD_Q=0"
i=0; files=""
for v in "$@"; do
  env $v timeout -k 10 300 python -u tools/conv_micro.py $S --clients ${CLIENTS:-32,8,4,2,1} > $O/micro_$i.txt 2>&1 || exit 2
  echo "[$i] $v"; files="$files $O/micro_$i.txt"; i=$((i+1))
done
paste $files | awk '{l=$1" "$3; for(i=9;i<=NF;i+=9) l=l" "$i; print l}'
