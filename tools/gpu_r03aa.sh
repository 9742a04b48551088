set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03aa; mkdir -p $O
for r in 1 2 3; do
  for v in 1 2 3; do
    echo "grid_div=$v" >> $O/gd.log
    RT_WHITTED_GRID_DIV=$v KERNEL=whitted LIBS=cur ROUNDS=1 REPS=10 timeout -k 10 120 python -u tools/ab.py >> $O/gd.log 2>&1
  done
done
