# usage (GPU box): bash tools/ab_stamps.sh <tag> — the default KT + K2 line with and without the
# roofline shape's launch stamps in the timed rounds, interleaved twice
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
for rep in 1 2; do
  for v in stamps nostamps; do
    A=""; [ $v = nostamps ] && A="--no-stamps"
    timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --rounds-target 0 --no-dpsgd $A --detail-out '' > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python -c "import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', $rep, 'KT', d['value'], 'K2', d['k2']['value'], 'roof', d['roofline']['frac'], d['k2']['roofline']['frac'])" | tee -a $O/ab.txt
  done
done
