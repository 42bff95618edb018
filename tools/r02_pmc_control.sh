# usage (GPU box): bash tools/r02_pmc_control.sh <tag>
# (1) control: a pure-torch process (no libfedhip) issuing ~40k small dispatches under
#     rocprofv3 --pmc FETCH_SIZE; (2) the one-lane KT bench under --pmc FETCH_SIZE with HIP's
#     kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0)
set -e
TAG=${1:-pmcctl}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT/torch $OUT/hostkernarg
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/torch -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_control.py > $OUT/torch/out.txt 2> $OUT/torch/log.txt
HIP_FORCE_DEV_KERNARG=0 FH_LAUNCH=program timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/hostkernarg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rounds-target 0 --steps 1 --warmup 1 --no-instances --lanes 1 > $OUT/hostkernarg/bench.json 2> $OUT/hostkernarg/log.txt
