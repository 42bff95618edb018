# usage (GPU box): bash tools/r03_s4b.sh <tag> — deferred-WGRAD A/B (K2, KT interleaved x2) and
# a kernel trace of full-width CIFAR10CNN steps (tools/fullstep.py) for the per-step breakdown
set -e
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
CONFIGS="K2 KT" REPS=2 bash tools/r03_ab.sh $T FH_DEFER_WGRAD=1 FH_DEFER_WGRAD=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fullstep -o run -- python3 $GRAFT_REPO_ROOT/tools/fullstep.py cifar10_cnn 32 12 > $O/fullstep.log 2>&1
python3 $GRAFT_REPO_ROOT/tools/fullstep.py --breakdown $O/fullstep > $O/fullstep_breakdown.txt 2>&1
