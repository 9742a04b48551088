set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03t; mkdir -p $O
for r in 1 2; do
  for cfg in "1 12000000" "2 12000000" "2 6000000" "2 4500000" "2 3000000"; do
    set -- $cfg
    echo "streams=$1 slab=$2" >> $O/qsweep.log
    RT_QUEUE_STREAMS=$1 RT_QUEUE_SLAB_TREES=$2 timeout -k 10 120 python -u tools/queue_time.py 20 >> $O/qsweep.log 2>&1
  done
done
for r in 1 2; do
  for wh in 1920x1080 800x600 640x480; do
    for v in 1 2; do
      echo "whitted $wh streams=$v" >> $O/wstreams.log
      WH=$wh RT_WHITTED_STREAMS=$v KERNEL=whitted LIBS=cur ROUNDS=1 REPS=10 timeout -k 10 120 python -u tools/ab.py >> $O/wstreams.log 2>&1
    done
  done
done
