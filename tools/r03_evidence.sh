# usage (GPU box): bash tools/r03_evidence.sh <tag> — round-3 evidence that is not the bench line:
# (1) the DP-SGD workload (bench.py --config K2-dpsgd) and its rocprofv3 kernel trace + stats;
# (2) one --pmc pass of SQ counters (MFMA busy, wave / busy cycles, LDS) over tools/conv_micro.py
#     for the round's MFMA kernels (quadrant-wave WGRAD, conv1 WGRAD, direct FWD / DGRAD)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --config K2-dpsgd --steps 3 --warmup 1 > $O/bench_K2dpsgd.json 2> $O/bench_K2dpsgd.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dpsgd -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config K2-dpsgd --steps 2 --warmup 1 > $O/prof_dpsgd.json 2> $O/prof_dpsgd.err || exit 2
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/prof_dpsgd > $O/trace_summary_dpsgd.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sq -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 wgrad:128:8:128:3:1 wgrad:1:28:32:3:1 fwd:32:32:32:3:1 dgrad:32:32:32:3:1 --clients 32,8,1 --reps 3 > $O/pmc_sq.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_grbm -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py wgrad:32:32:32:3:1 wgrad:128:8:128:3:1 wgrad:1:28:32:3:1 fwd:32:32:32:3:1 dgrad:32:32:32:3:1 --clients 32,8,1 --reps 3 > $O/pmc_grbm.log 2>&1 || exit 4
