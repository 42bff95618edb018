# usage (GPU box): bash tools/r02_configs.sh <tag> <configs...>
# bench line + rocprofv3 kernel stats for each BASELINE config slice
set -e
TAG=${1:-r02}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for C in "$@"; do
  timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$C -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --no-cpu-baseline --rounds-target 0 --steps 2 --warmup 1 > $OUT/profbench_$C.log 2>&1)
done
