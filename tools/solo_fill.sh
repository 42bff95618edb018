# usage (GPU box): bash tools/solo_fill.sh <tag> "<fills>" [model] — one-client training steps alone
# on the chip (tools/fullstep.py) at each split-K fill fraction: ms per step (plain run) and the
# per-step kernel table of a kernel trace
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O; M=${3:-cifar10_cnn}
cd /tmp && export TMPDIR=/tmp
for F in $2; do
  echo "fill $F" >> $O/solo.txt
  timeout -k 10 120 python $GRAFT_REPO_ROOT/tools/fullstep.py --u8 --fill $F $M 1 60 >> $O/solo.txt 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$F -o run -- python3 $GRAFT_REPO_ROOT/tools/fullstep.py --u8 --fill $F $M 1 24 > /dev/null 2>&1 || exit 1
  python3 $GRAFT_REPO_ROOT/tools/fullstep.py --breakdown $O/prof_$F > $O/steps_$F.txt
done
