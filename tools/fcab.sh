# usage (GPU box): bash tools/fcab.sh <tag> — classifier launch costs (tools/fc_bench.py) of
# ab_lib/base vs the tree's library at the lanes' fill fractions, interleaved twice
O=gpurun_out/$1; mkdir -p $O
for rep in 1 2; do
  for L in base tree; do
    A=""; [ $L = base ] && A="--lib ab_lib/base/libfedhip.so"
    for F in "0.75 23" "0.5 8" "0.25 1"; do set -- $F
      echo "== $L rep $rep fill $1" >> $O/fc.txt
      FH_BENCH_FILL=$1 FH_BENCH_CLIENTS=$2 timeout -k 10 120 python tools/fc_bench.py $A >> $O/fc.txt 2>&1 || exit 1
    done
    for F in "0.75 21" "0.5 10" "0.25 1"; do set -- $F
      echo "== $L rep $rep fill $1 simple" >> $O/fc.txt
      FH_BENCH_FILL=$1 FH_BENCH_CLIENTS=$2 FH_BENCH_LAYERS=3136x128 timeout -k 10 120 python tools/fc_bench.py $A >> $O/fc.txt 2>&1 || exit 1
    done
  done
done
