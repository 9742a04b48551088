set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h; mkdir -p $O
for cfg in "12000000 0.9" "12000000 0.75" "6000000 0.75" "4000000 0.75" "3000000 0.75"; do
  set -- $cfg
  echo "== slab $1 frac0 $2" >> $O/queue.log
  RT_QUEUE_SLAB_TREES=$1 RT_QUEUE_POOL_FRAC0=$2 timeout -k 10 120 python tools/queue_time.py 20 2>&1 | grep -v amdgpu >> $O/queue.log
done
VARS="-" bash tools/wf_env.sh > $O/whitted_kernels.log 2>&1
