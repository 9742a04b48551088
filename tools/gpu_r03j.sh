set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_whitted.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted.log 2>&1
VARS="- RT_WHITTED_BACKACC=1 -" bash tools/wf_env.sh > $O/whitted_kernels.log 2>&1
