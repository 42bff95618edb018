# usage (GPU box): bash tools/r03_r02pmc.sh <tag> — the r02 tree (worktree under _old/r02tree, built
# here) under ONE rocprofv3 --pmc FETCH_SIZE pass of its own bench.py, to tell whether the r02
# profiler segfault follows the code or the box/profiler.  Runs last in its call.
T=$1
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
R=$GRAFT_REPO_ROOT/_old/r02tree
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o run -- python3 $R/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances > $O/bench.json 2> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
grep -a -m3 "SIGSEGV\|PC:" $O/log.txt
exit 0
