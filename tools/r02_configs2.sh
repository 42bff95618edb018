# usage (GPU box): bash tools/r02_configs2.sh <tag> <configs...>
# one full bench line per BASELINE config slice (roofline over all launches, instances,
# cpu_baseline), no rounds-to-target (the KT line carries it)
set -e
TAG=${1:-r02}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for C in "$@"; do
  timeout -k 10 500 python bench.py --config $C --rounds-target 0 --steps 3 --warmup 1 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
done
