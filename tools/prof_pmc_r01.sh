set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o p -- python3 tools/prof_kernels.py --reps 1 > gpurun_out/pmc1.log 2>&1
$P --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 -d gpurun_out/pmc2 -o p -- python3 tools/prof_kernels.py --reps 1 > gpurun_out/pmc2.log 2>&1
