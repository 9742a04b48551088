set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s; mkdir -p $O
RT_QUEUE_STREAMS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q --timeout 120 --timeout-method thread > $O/t_queue_2s.log 2>&1
for r in 1 2 3; do
  for v in 1 2; do
    echo "streams=$v" >> $O/qstreams.log
    RT_QUEUE_STREAMS=$v timeout -k 10 120 python -u tools/queue_time.py 20 >> $O/qstreams.log 2>&1
  done
done
