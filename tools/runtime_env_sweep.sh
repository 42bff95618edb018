# usage (GPU box): bash tools/runtime_env_sweep.sh <tag> — KT bench under HIP runtime knobs
# (cross-lane serialisation of graph launches: signal pool, AQL queue size, batching)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --rounds-target 0 --steps 5 > $OUT/$name.json 2> $OUT/$name.err || { echo "$name FAILED"; tail -3 $OUT/$name.err; return 0; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'])"
}
run base FH_X=0
run sigpool4k ROC_SIGNAL_POOL_SIZE=4096
run aql64k ROC_AQL_QUEUE_SIZE=65536
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run batch1k DEBUG_CLR_MAX_BATCH_SIZE=1024
run cpusync DEBUG_CLR_BATCH_CPU_SYNC_SIZE=100000
run cpuwait0 ROC_CPU_WAIT_FOR_SIGNAL=0
run dynq DEBUG_HIP_DYNAMIC_QUEUES=1
run graphq DEBUG_HIP_FORCE_GRAPH_QUEUES=1
run kacopy0 DEBUG_HIP_KERNARG_COPY_OPT=0
