set -e
O=gpurun_out/r02_ds2b; mkdir -p $O
for cfg in "512 32" "256 32" "512 64" "1024 16" "256 64"; do
  set -- $cfg
  echo "### FILL=$1 MINCH=$2" >> $O/sweep.txt
  FH_DS2_FILL=$1 FH_DS2_MINCH=$2 timeout -k 10 120 python tools/conv_micro.py dgrad:64:32:128:3:2 dgrad:128:16:256:3:2 --clients 8,4,2,1 >> $O/sweep.txt 2>&1
done
