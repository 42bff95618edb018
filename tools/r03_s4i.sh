# usage (GPU box): bash tools/r03_s4i.sh <tag> — narrow-lane step anatomy: kernel traces of
# one-lane CIFAR10CNN steps at 1 and 8 clients (every client at every step)
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fs$n -o run -- python3 $GRAFT_REPO_ROOT/tools/fullstep.py cifar10_cnn $n 24 > $O/fs$n.log 2>&1
  python3 $GRAFT_REPO_ROOT/tools/fullstep.py --breakdown $O/fs$n > $O/fs${n}_breakdown.txt 2>&1
  grep "round 2" $O/fs$n.log
  head -45 $O/fs${n}_breakdown.txt
done
cd $GRAFT_REPO_ROOT
for n in 1 8; do timeout -k 10 120 python tools/fullstep.py cifar10_cnn $n 24 2>&1 | grep round; done
