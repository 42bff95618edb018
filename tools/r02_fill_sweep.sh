# usage (GPU box): bash tools/r02_fill_sweep.sh <tag> <fill>...   (per-lane split-K fill fractions)
TAG=$1; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for F in "$@"; do
  FH_LANE_FILL=$F timeout -k 10 200 python bench.py --no-cpu-baseline --rounds-target 0 --no-instances --steps 4 --warmup 1 > $OUT/b_$F.json 2> $OUT/b_$F.err || exit 1
  echo "$F $(python3 -c "import json;d=json.load(open('$OUT/b_$F.json'));print(d['value'],d['ms_per_step'])")" | tee -a $OUT/sweep.txt
done
