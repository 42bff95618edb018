# usage (GPU box): bash tools/r02_ablate.sh <tag>
# KT client-images/s with kernel families removed (FH_ABLATE: the entry points are not
# called; results wrong by construction) -- what each family costs the concurrent round
set -e
TAG=${1:-ablate}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
run() {
  FH_ABLATE=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --rounds-target 0 --no-instances --steps 3 --warmup 1 > $OUT/$1.json 2> $OUT/$1.err
  python -c "import json,sys; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
}
run base ""
run bnfwd fh_bn_fwd_stats
run bnbwd fh_bn_bwd,fh_bn_bwd_pool
run linear fh_linear_fwd,fh_linear_dgrad,fh_linear_wgrad
run wgrad fh_conv2d_wgrad,fh_conv2d_wgrad_bnrelu
run fwd fh_conv2d_fwd,fh_conv2d_fwd_bnrelu
run dgrad fh_conv2d_dgrad
run pool fh_maxpool2_fwd,fh_maxpool2_fwd_bnrelu
run dropout fh_dropout_fwd,fh_dropout_bwd
run sgd fh_sgd_step
run gather fh_gather_u8,fh_ce_fwd_bwd
run base2 ""
