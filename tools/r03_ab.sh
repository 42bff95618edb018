# usage (GPU box): [TESTS=1] [CONFIGS="K2 KT"] [REPS=2] bash tools/r03_ab.sh <tag> "<env A>" "<env B>" ...
# optional full GPU test suite first, then interleaved bench A/B of the given env settings
set -e
T=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T; mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
fi
for i in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    for C in ${CONFIGS:-K2 KT}; do
      n=$(echo "$v" | tr ' =' '_-')
      env $v timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --rounds-target 0 --steps 3 --warmup 1 --no-instances --no-k2 > $O/b_${C}_${n}_$i.json 2>/dev/null
      python -c "import json; d=json.loads(open('$O/b_${C}_${n}_$i.json').read().strip().splitlines()[-1]); print('$C', '$v', $i, d['value'], d['ms_per_step'])" >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
