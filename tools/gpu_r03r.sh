set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03r; mkdir -p $O
RT_WHITTED_STREAMS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_whitted.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted_2s.log 2>&1
for r in 1 2 3; do
  for v in "RT_WHITTED_STREAMS=1" "RT_WHITTED_STREAMS=2" "RT_WHITTED_SLABS=2"; do
    echo "$v" >> $O/streams.log
    env $v KERNEL=whitted LIBS=cur ROUNDS=1 REPS=10 timeout -k 10 120 python -u tools/ab.py >> $O/streams.log 2>&1
  done
done
