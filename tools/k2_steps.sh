# usage (GPU box): bash tools/k2_steps.sh <tag> "<libs>" "<clients>" [model] [--dpsgd] — per-step kernel
# table (tools/fullstep.py --breakdown) of one packed lane of SimpleCNN on uint8 images, for each
# library ("-" = the tree's) and client count; the lane's split-K fill as the bench's lanes
# (1 client 0.25, else 0.5)
set -e
T=$1; LIBS=$2; CS=$3; M=${4:-simple_cnn}; X=${5:-}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in $CS; do
  F=0.5; [ "$C" = "1" ] && F=0.25
  i=0
  for L in $LIBS; do
    i=$((i+1)); A=""; [ "$L" != "-" ] && A="--lib $R/$L"
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/prof_${C}_$i -o run -- python3 $R/tools/fullstep.py --u8 $X $A --fill $F $M $C 24 > $O/run_${C}_$i.txt 2> $O/run_${C}_$i.err
    python3 $R/tools/fullstep.py --breakdown $O/prof_${C}_$i > $O/steps_${C}_$i.txt
    echo "== $C clients, lib $L"; head -16 $O/steps_${C}_$i.txt
  done
done
