# usage (GPU box): bash tools/r02_ablate2.sh <tag>
# finer timing ablations of the KT round (results wrong by construction): the classifier's
# small layers vs fc1, the BN finalize, cross-entropy, max-pool
set -e
TAG=${1:-ablate2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --rounds-target 0 --no-instances --steps 5 --warmup 1 > $OUT/$1.json 2> $OUT/$1.err
  python -c "import json,sys; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
}
run base FH_NOOP=1
run fc23 FH_ABLATE_LINEAR=512,256
run fc1 FH_ABLATE_LINEAR=2048
run finalize FH_ABLATE=fh_bn_finalize_tiles
run ce FH_ABLATE=fh_ce_fwd_bwd
run dropout FH_ABLATE=fh_dropout_fwd,fh_dropout_bwd
run copy FH_ABLATE=fh_copy_bytes
run base2 FH_NOOP=1
