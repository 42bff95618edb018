cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/diag
timeout -k 10 200 python tools/diag_layers.py 1,1,1 > gpurun_out/diag/layers111.txt 2>&1
