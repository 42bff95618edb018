# usage (GPU box): bash tools/prof_env.sh <tag> [bench args] — kernel trace of the KT bench
# under the caller's environment (e.g. FH_LANE_CU=32)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 "$@" > $OUT/bench.json 2> $OUT/bench.err
