# Whitted: two-level back-accumulation (RT_WHITTED_BACKACC=2, default) vs a
# launch per level (=1): exactness, frame times, PMC traffic per frame
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_whitted.py tests/test_gpu_shims.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted.log 2>&1
RT_WHITTED_BACKACC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_whitted.py -x -q --timeout 120 --timeout-method thread -k "bit_exact or counts" > $O/t_whitted_b1.log 2>&1
for r in 1 2 3; do
  for b in 1 2; do
    KERNEL=whitted VARIANT=ba$b RT_WHITTED_BACKACC=$b REPS=20 WARM=3 timeout -k 10 120 python -u tools/ab.py child 2>&1 | grep whitted >> $O/ab.log
    WH=640x480 KERNEL=whitted VARIANT=ba$b RT_WHITTED_BACKACC=$b REPS=20 WARM=3 timeout -k 10 120 python -u tools/ab.py child 2>&1 | grep whitted >> $O/ab.log
  done
done
for b in 1 2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    KERNEL=whitted RT_WHITTED_BACKACC=$b REPS=1 WARM=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
        --pmc $c -d $O/pmc_ba$b/$c -o p -- python3 tools/ab.py child > $O/pmc_ba$b.$c.log 2>&1
  done
  SLABS=2 python3 tools/pmc_frame_sum.py $O/pmc_ba$b > $O/traffic_ba$b.txt
done
