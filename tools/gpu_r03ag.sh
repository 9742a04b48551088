# Whitted: per-tree records in tile-linear pixel order (tile) vs row-major (prev = a7d8613):
# exactness, frame times, PMC traffic per frame
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_whitted.py tests/test_gpu_shims.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted.log 2>&1
LIBS=prev,tile KERNEL=whitted ROUNDS=4 REPS=20 WARM=3 timeout -k 10 300 python -u tools/ab.py > $O/ab.log 2>&1
WH=640x480 LIBS=prev,tile KERNEL=whitted ROUNDS=4 REPS=20 WARM=3 timeout -k 10 300 python -u tools/ab.py >> $O/ab.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  KERNEL=whitted REPS=1 WARM=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
      --pmc $c -d $O/pmc_tile/$c -o p -- python3 tools/ab.py child > $O/pmc_tile.$c.log 2>&1
done
SLABS=2 python3 tools/pmc_frame_sum.py $O/pmc_tile > $O/traffic_tile.txt
