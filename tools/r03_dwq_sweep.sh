# usage (GPU box): bash tools/r03_dwq_sweep.sh <tag> — quadrant-wave WGRAD: split target sweep
# (FH_DWQ_BLOCKS) per shape and client count, then one PMC pass of the default at 32 / 1 clients
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
cd $GRAFT_REPO_ROOT
S="wgrad:32:32:32:3:1 wgrad:128:8:128:3:1 wgrad:64:16:64:3:1 wgrad:64:32:64:3:1"
for b in 256 512 768 1024; do
  FH_DWQ_BLOCKS=$b timeout -k 10 300 python -u tools/conv_micro.py $S --clients 32,8,2,1 > $O/micro_b$b.txt 2>&1 || exit 2
done
paste $O/micro_b256.txt $O/micro_b512.txt $O/micro_b768.txt $O/micro_b1024.txt | awk '{print $1, $3, $9, $18, $27, $36}'
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 --clients 32,1 --reps 3 > $O/pmc1_log.txt 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 --clients 32,1 --reps 3 > $O/pmc2_log.txt 2>&1 || exit 4
