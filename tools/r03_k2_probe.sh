# usage (GPU box): bash tools/r03_k2_probe.sh <tag> — K2 (SimpleCNN) per-kernel evidence: conv1
# (single input channel) FWD / WGRAD and the classifier layers per client count, then a
# rocprofv3 kernel trace + stats of the K2 bench line
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/conv_micro.py wgrad:1:28:32:3:1 fwd:1:28:32:3:1 wgrad:32:16:64:3:1 fwd:32:16:64:3:1 dgrad:32:16:64:3:1 --clients 32,8,1 > $O/micro.txt 2>&1 || exit 1
FH_BENCH_LAYERS=3136x128,128x10 FH_BENCH_CLIENTS=32,8,1 timeout -k 10 200 python -u tools/fc_bench.py > $O/fc.txt 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config K2 --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 > $O/bench_K2.json 2> $O/bench_K2.err || exit 3
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/prof > $O/trace_summary.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profKT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --no-k2 --steps 3 --warmup 1 > $O/bench_KT.json 2> $O/bench_KT.err || exit 4
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/profKT > $O/trace_summary_KT.txt 2>&1 || true
