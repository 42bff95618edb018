# usage (GPU box): bash tools/k2prof.sh <tag> [configs]
# A rocprofv3 kernel trace of `bench.py --config C` (no instrumented round, no host legs) per
# config, with the per-round kernel families and the conv launches by grid (trace_rounds.py).
set -e
T=${1:-k2prof}
CS=${2:-K2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in $CS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$C -o run -- python3 $R/bench.py --config $C --steps 4 --warmup 1 --no-cpu-baseline --rounds-target 0 --no-instances --no-k2 --detail-out '' > $O/bench_$C.json 2> $O/bench_$C.err
  python3 $R/tools/trace_rounds.py $O/prof_$C 5 fh::dconv_kernel fh::dconv_wgrad_dual_kernel > $O/trace_rounds_$C.txt 2>&1
  head -24 $O/trace_rounds_$C.txt
done
