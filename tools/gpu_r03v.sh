set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03v; mkdir -p $O
for r in 1 2 3; do
  for v in 2 3 4 6; do
    echo "whitted slabs=$v" >> $O/wslabs.log
    RT_WHITTED_SLABS=$v KERNEL=whitted LIBS=cur ROUNDS=1 REPS=10 timeout -k 10 120 python -u tools/ab.py >> $O/wslabs.log 2>&1
  done
done
