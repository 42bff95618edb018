# usage (GPU box): bash tools/split_sweep.sh <tag> — graph-mode conv costs per forced split count
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
for s in 0 1 2 4 8 16; do
  FH_DCONV_SPLITS=$s FH_DWGRAD_SPLITS=$s FH_FILLS=1 FH_BENCH_CLIENTS=1,2,3,4,6,8,12,16,23,32 \
    timeout -k 10 240 python -u tools/tail_graph_bench.py > $OUT/split_$s.txt 2>&1
done
