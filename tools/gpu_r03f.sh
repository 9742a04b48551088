set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
N=300 timeout -k 10 300 python tools/bvh_stress.py > $O/bvh_stress.log 2>&1
SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu > $O/c5.log
GROUP=3/8 SPP=64 REPS=5 timeout -k 10 120 python tools/c5_time.py 2>&1 | grep -v amdgpu >> $O/c5.log
SPP=64 SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE;SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_BRANCH;FETCH_SIZE;WRITE_SIZE" bash tools/pmc_c5.sh > $O/pmc_c5.log 2>&1
cp -r gpurun_out/pmc_c5 $O/
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o c5 -- python3 tools/c5_time.py > $O/stats.log 2>&1
