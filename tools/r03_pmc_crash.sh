# usage (GPU box): [PMC_COUNTER=WRITE_SIZE] bash tools/r03_pmc_crash.sh <tag> [bench args...] — ONE
# rocprofv3 --pmc FETCH_SIZE (or $PMC_COUNTER) pass of bench.py with /proc/self/maps snapshotted every 0.1 s (FH_DUMP_MAPS), so
# a profiler SIGSEGV can be placed against what was mapped just before it.  One pass per call:
# a segfault ends the call.
T=$1; shift
CTR=${PMC_COUNTER:-FETCH_SIZE}
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
FH_DUMP_MAPS=$O/maps.txt timeout -s KILL 150 rocprofv3 --pmc $CTR --output-format csv -d $O/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --no-k2 "$@" > $O/bench.json 2> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
grep -a -m3 "SIGSEGV\|PC:" $O/log.txt
exit 0
