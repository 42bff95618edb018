O=$GRAFT_REPO_ROOT/gpurun_out/r06_i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_inlaunch_split_gpu.py tests/test_conv_gpu.py > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -2 $O/t1.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 1200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
REPS=2 STEPS=10 bash tools/ab_env.sh r06_i/ab "KT K2" "FH_SPLIT_TICKETS=0" "-"
bash tools/solo_fill.sh r06_i/solo "0.25"
