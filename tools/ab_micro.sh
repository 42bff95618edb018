# usage (GPU box): bash tools/ab_micro.sh <tag> "<conv_micro args>" — conv_micro with the
# baseline library (ab_lib/base/libfedhip.so) and the tree's library, interleaved twice
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in base new; do
    L=""; [ $v = base ] && L="--lib $GRAFT_REPO_ROOT/ab_lib/base/libfedhip.so"
    echo "== $v $rep" | tee -a $O/ab.txt
    timeout -k 10 200 python tools/conv_micro.py $2 $L 2>/dev/null | tee -a $O/ab.txt
  done
done
