# drop-in: pinned pixel buffer (rt_host_alloc); shim tests and the drop-in bench
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_shims.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/t_shims.log 2>&1
for r in 1 2; do
  timeout -k 10 60 tests/native/smallpt_dropin_bench 1920 1080 3.0 >> $O/dropin.log 2>&1
  RT_SPT_SHIM_BATCH=1 timeout -k 10 60 tests/native/smallpt_dropin_bench 1920 1080 3.0 >> $O/dropin.log 2>&1
done
