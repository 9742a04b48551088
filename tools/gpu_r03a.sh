set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
LIBS=gs0,gs1 REPS=5 SPP=64 bash tools/ab_c5.sh > $O/ab.log 2>&1
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=1 K=0 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n1.log 2>&1
RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/trace/librt_hip.so N=8 K=0,1,2,3,4,5,6,7 timeout -k 10 200 python tools/c5_phase.py > $O/phase_n8.log 2>&1
LIBS=gs0,gs1 bash tools/pmc_c5_writes.sh > $O/pmcw.log 2>&1
