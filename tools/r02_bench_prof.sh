# usage (GPU box): bash tools/r02_bench_prof.sh <tag> [bench args...]
# 1) the bench line; 2) rocprofv3 kernel trace + stats of the same bench (no baselines)
set -e
TAG=$1; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 "$@" > $OUT/prof_bench.json 2> $OUT/prof_bench.err
