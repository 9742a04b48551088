set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_shims.py -x -q --timeout 120 --timeout-method thread > $O/t_queue.log 2>&1
timeout -k 10 200 python -u tools/queue_time.py 20 > $O/queue.log 2>&1
