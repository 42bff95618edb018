# usage (GPU box): [REPS=2] [STEPS=20] bash tools/ab_variants.sh <tag> "<configs>" "<tests>"
# "<variant>"... — bench lines of each variant (tools/ab_attr.py arguments, e.g.
# "lib=ab_lib/base/libfedhip.so" or "fuse_pool2=0"; "-" = the tree as is), interleaved REPS
# times per config, STEPS timed rounds each; the named GPU tests first
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
CONFIGS=$2; TESTS=$3; shift 3
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for C in $CONFIGS; do
  for rep in $(seq 1 ${REPS:-2}); do
    i=0
    for v in "$@"; do
      i=$((i+1)); A=$v; [ "$v" = "-" ] && A=""
      timeout -k 10 300 python tools/ab_attr.py $A -- --config $C --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --rounds-target 0 --no-instances --no-k2 --detail-out '' > $O/${C}_v${i}_${rep}.json 2>> $O/ab.err
      python -c "import json; d=json.loads(open('$O/${C}_v${i}_${rep}.json').read().strip().splitlines()[-1]); print('$C', '[$v]', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
    done
  done
done
