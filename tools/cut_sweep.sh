O=gpurun_out/r06_cut; mkdir -p $O
for rep in 1 2; do
for C in default 0,1,8,32 0,1,10,32 0,1,7,32 0,1,11,32 0,2,10,32; do
  if [ $C = default ]; then E=""; else E="FH_LANE_CUT=$C"; fi
  env $E timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-k2 --no-dpsgd --no-cpu-baseline --rounds-target 0 --no-instances --detail-out "" > $O/kt_${C}_$rep.json 2> $O/kt_${C}_$rep.err || exit 1
  python -c "import json,sys; d=json.loads(open('$O/kt_${C}_$rep.json').read().strip().splitlines()[-1]); print('$C', $rep, d['value'], d['ms_per_step'], d['config']['lanes'])" >> $O/summary.txt
done; done
