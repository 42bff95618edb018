# usage (GPU box): bash tools/r02_fullstep.sh <tag> [ENV=VAL ...] — kernel trace of full-width
# CIFAR10CNN steps (32 clients x 32 images, eager, one stream) per env variant:
# where a 32-client step's time goes (analyse with tools/step_breakdown.py)
set -e
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ $# -eq 0 ] && set -- "FH_NOOP=1"
i=0
for E in "$@"; do
  export $E
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$i -o run -- python3 $GRAFT_REPO_ROOT/tools/traffic_probe.py ${CLIENTS:-32} 20 > $OUT/probe_$i.log 2>&1
  unset ${E%%=*}
  echo "$i $E" >> $OUT/variants.txt
  i=$((i+1))
done
