# usage (GPU box): bash tools/gpu_traffic_pass.sh <tag> <COUNTER>
# One rocprofv3 --pmc pass of a short one-lane, graph-replay bench (one counter per call).
# Under --pmc the process aborts in the CUDA-graph destructor at exit after the counter
# file is written, and then hangs in the profiler's signal handler: the pass is bounded
# by its own time limit and the call ends there; tools/traffic.py merges two calls' files.
TAG=$1; CTR=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG/$(echo $CTR | tr A-Z a-z)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
FH_LAUNCH=graph FH_LANES=1 timeout -s KILL 100 rocprofv3 --pmc $CTR --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $OUT/log.txt 2>&1
rc=$?
ls -la $OUT
exit $rc
