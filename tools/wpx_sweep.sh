# usage (GPU box): bash tools/wpx_sweep.sh <tag> — direct WGRAD pixel-wave count (FH_DWGRAD_WPX)
# on the ResNet / CIFAR10CNN wgrad shapes at several client counts (tools/conv_micro.py)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
for wpx in 4 2 1; do
  echo "### WPX=$wpx" >> $O/sweep.txt
  FH_DWGRAD_WPX=$wpx timeout -k 10 120 python tools/conv_micro.py wgrad:64:32:64:3:1 wgrad:128:16:128:3:1 wgrad:256:8:256:3:1 wgrad:64:16:64:3:1 wgrad:128:8:128:3:1 --clients 16,4,1 2>&1 | grep -v amdgpu >> $O/sweep.txt
done
