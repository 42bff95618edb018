# usage (GPU box): bash tools/ab_libs.sh <tag> NAME=path/to/libfedhip.so ... — A/B of built
# library variants: each is copied over lib/libfedhip.so, then the conv microbench and the
# KT bench (--steps 5, no CPU baseline / rounds-to-target) run; two interleaved repetitions.
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
shift
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
LIB=federated-learning-for-privacy-preserving-image-classification_amd/lib/libfedhip.so
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; so=${spec#*=}
    cp $so $LIB
    if [ $rep = 1 ]; then
      FH_BENCH_CLIENTS=32 timeout -k 10 120 python tools/conv_bench.py > $OUT/$name.conv.txt 2>&1 || { echo "$name conv FAILED"; tail -3 $OUT/$name.conv.txt; exit 1; }
    fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --rounds-target 0 --steps 5 > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || { echo "$name FAILED"; tail -3 $OUT/$name.$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$name.$rep.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
