# usage (GPU box): bash tools/pmc_conv.sh <tag> <shapes...> — SQ counters of conv_micro launches
# (one rocprofv3 --pmc pass, 32 clients), summarised per kernel instance by tools/pmc_summary.py
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $O/pmc -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py "$@" --clients 32 --reps 5 > $O/micro.txt 2> $O/pmc.log
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt
cat $O/pmc_summary.txt
