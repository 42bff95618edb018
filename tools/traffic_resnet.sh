# usage (GPU box): bash tools/traffic_resnet.sh <tag> — two rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE; one counter each) of the eager ResNet-8 probe at 8 and 2 clients
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT/fetch $OUT/write
cd /tmp && export TMPDIR=/tmp
export PROBE_MODEL=federated_resnet PROBE_KW='{"num_blocks": [1, 1, 1]}'
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/traffic_probe.py 8,2 3 > $OUT/fetch/log.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $GRAFT_REPO_ROOT/tools/traffic_probe.py 8,2 3 > $OUT/write/log.txt 2>&1
