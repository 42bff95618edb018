set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r03_a; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/conv_micro.py wgrad:32:32:32:3:1 wgrad:128:8:128:3:1 wgrad:64:16:64:3:1 wgrad:64:32:64:3:1 fwd:32:32:32:3:1 dgrad:32:32:32:3:1 fwd:128:8:128:3:1 --clients 32,16,8,4,2,1 > $O/micro.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 --clients 32,4,1 --reps 5 > $O/kt_log.txt 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 --clients 32,4,1 --reps 5 > $O/pmc1_log.txt 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 --clients 32,4,1 --reps 5 > $O/pmc2_log.txt 2>&1 || exit 4
ls -R $O | head -50
