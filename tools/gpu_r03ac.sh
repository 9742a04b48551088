set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03ac; mkdir -p $O
for r in 1 2; do
for hv in 64 0 256 1024; do
  for g in "" 3/8 0/8; do
    echo "heavyprio=$hv group=$g" >> $O/hp.log
    RT_SPT_HEAVY=$hv SPP=64 GROUP=$g REPS=5 timeout -k 10 120 python -u tools/c5_time.py >> $O/hp.log 2>&1
  done
done
done
