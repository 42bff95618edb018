O=gpurun_out/r06_h; mkdir -p $O
for K in KT K5 K3; do
  timeout -k 10 300 python bench.py --config $K --predict-strong 1,2,4,8 --steps 3 --warmup 1 > $O/predict_strong_$K.json 2> $O/predict_strong_$K.err || exit 1
done
REPS=2 STEPS=10 bash tools/ab_variants.sh r06_h/ab "KT" "" "lib=ab_lib/base/libfedhip.so" "-"
