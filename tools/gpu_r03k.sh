set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m; mkdir -p $O
for sp in 0 1 2; do
  for h in 1024 2048; do
  for g in "" 3/8 0/8; do
    echo "split=$sp heavy=$h group=$g" >> $O/heavy.log
    SPP=64 RT_SPT_SPLIT=$sp RT_WIDE_HEAVY=$h GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/heavy.log 2>&1
  done
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
RT_SPT_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread -k "configs4 or adaptive or bvh" > $O/t_smallpt_split1.log 2>&1
RT_SPT_WIDE=0 LIBS=gs0,gs1 bash tools/pmc_c5_writes.sh > $O/pmcw.log 2>&1
