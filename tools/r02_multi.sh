# usage (GPU box): bash tools/r02_multi.sh <tag> <config>...  bench lines (no baselines)
TAG=$1; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for C in "$@"; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --rounds-target 0 --no-instances --steps 3 --warmup 1 > $OUT/b_$C.json 2> $OUT/b_$C.err || exit 1
  echo "$C $(python3 -c "import json;d=json.load(open('$OUT/b_$C.json'));print(d['value'],d['ms_per_step'],d['round_frac'],d['config']['lanes'])")" >> $OUT/sum.txt
done
