# usage (GPU box): bash tools/fc_sweep.sh <tag> — classifier split-K planner sweep
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for cfg in "192 768" "512 768" "1024 1536" "1024 3072" "2048 3072"; do
  set -- $cfg
  FH_MN_SPLIT_BELOW=$1 FH_MN_TARGET=$2 timeout -k 10 200 python -u tools/fc_bench.py > $OUT/fc_$1_$2.txt 2>&1
  echo "== below $1 target $2"; cat $OUT/fc_$1_$2.txt | grep "^C="
done
