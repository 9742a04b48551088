set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ab; mkdir -p $O
for r in 1 2; do
for ps in default 0,0,0 32,64,128; do
  for g in "" 3/8 0/8; do
    echo "prio=$ps group=$g" >> $O/prio.log
    if [ "$ps" = default ]; then
      SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/prio.log 2>&1
    else
      RT_SPT_PRIO_SCHED=$ps SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/prio.log 2>&1
    fi
  done
done
done
