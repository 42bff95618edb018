# usage (GPU box): bash tools/r03_batch2.sh <tag> — K2 A/B of the pool2 fold (10 rounds x 3 pairs),
# a KT sweep of the direct-conv split-K thresholds, a kernel trace of KT, then ONE rocprofv3 --pmc
# pass of bench.py with /proc/self/maps snapshots (last: it may crash the profiler)
set -e
T=$1
cd $GRAFT_REPO_ROOT
STEPS=10 CONFIG=K2 bash tools/r02_iter.sh ${T}_k2ab NONE FH_FUSE_POOL2_BWD=1 FH_FUSE_POOL2_BWD=0 FH_FUSE_POOL2_BWD=1 FH_FUSE_POOL2_BWD=0 FH_FUSE_POOL2_BWD=1 FH_FUSE_POOL2_BWD=0
bash tools/r02_iter.sh ${T}_split NONE FH_NOOP=1 "FH_DCONV_SPLIT_BELOW=256 FH_DCONV_SPLIT_TARGET=512" "FH_DCONV_SPLIT_BELOW=1024 FH_DCONV_SPLIT_TARGET=2048" FH_NOOP=1 "FH_DCONV_SPLIT_BELOW=256 FH_DCONV_SPLIT_TARGET=512" "FH_DCONV_SPLIT_BELOW=1024 FH_DCONV_SPLIT_TARGET=2048"
O=$GRAFT_REPO_ROOT/gpurun_out/${T}_kt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --no-k2 --steps 3 --warmup 1 > $O/bench_KT.json 2> $O/bench_KT.err
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/prof > $O/trace_summary_KT.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
set +e
bash tools/r03_pmc_crash.sh ${T}_pmc
