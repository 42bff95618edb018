# usage (GPU box): bash tools/prof_tail.sh <tag>   — kernel trace of tools/tail_graph_bench.py
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
FH_BENCH_CLIENTS=${FH_BENCH_CLIENTS:-1} FH_FILLS=${FH_FILLS:-1,0.25} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/tools/tail_graph_bench.py > $OUT/log.txt 2>&1
