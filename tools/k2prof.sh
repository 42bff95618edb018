set -e
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r04_k2prof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config K2 --steps 4 --warmup 1 --no-cpu-baseline --rounds-target 0 --no-instances --detail-out '' > $O/bench.json 2> $O/bench.err
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/prof > $O/trace_summary.txt 2>&1
head -24 $O/trace_summary.txt
