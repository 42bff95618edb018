# usage (GPU box): bash tools/ab_lib.sh <tag> "<configs>" [tests] — bench lines of the baseline
# library (ab_lib/base/libfedhip.so, tools/build_base_lib.sh) and the tree's library,
# interleaved twice per config; the named GPU tests first
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
if [ -n "$3" ]; then
  timeout -k 10 400 python -u -m pytest $3 -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for C in $2; do
  for rep in 1 2; do
    for v in base new; do
      L=""; [ $v = base ] && L="lib=$GRAFT_REPO_ROOT/ab_lib/base/libfedhip.so"
      timeout -k 10 300 python tools/ab_attr.py $L -- --config $C --steps 20 --warmup 5 --no-cpu-baseline --rounds-target 0 --no-instances --no-k2 --detail-out '' > $O/${C}_${v}_${rep}.json 2>> $O/ab.err
      python -c "import json; d=json.loads(open('$O/${C}_${v}_${rep}.json').read().strip().splitlines()[-1]); print('$C $v', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
    done
  done
done
