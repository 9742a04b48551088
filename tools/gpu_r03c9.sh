# counted configs[4] frame: is it chain-bound? cooperative tiles on the counted full frame
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c9; mkdir -p $O
run() { echo "$1" >> $O/ab.log; shift; env "$@" SPP=64 REPS=5 timeout -k 10 120 python -u tools/c5_time.py 2>&1 | grep c5 >> $O/ab.log; }
for rnd in 1 2; do
  run "counted full default" COUNTED=1
  run "counted full coop256 hw4" COUNTED=1 RT_WIDE_COOP=256 RT_WIDE_HEAVY_WAVES=4
  run "counted full coop256 hw8" COUNTED=1 RT_WIDE_COOP=256 RT_WIDE_HEAVY_WAVES=8
  run "counted full coop512 hw8" COUNTED=1 RT_WIDE_COOP=512 RT_WIDE_HEAVY_WAVES=8
  run "counted full coop512 hw16" COUNTED=1 RT_WIDE_COOP=512 RT_WIDE_HEAVY_WAVES=16
  run "counted full coop1024 hw16" COUNTED=1 RT_WIDE_COOP=1024 RT_WIDE_HEAVY_WAVES=16
  run "counted g=0/8 default" COUNTED=1 GROUP=0/8
  run "counted g=0/2 default" COUNTED=1 GROUP=0/2
  run "counted g=0/2 coop256 hw8" COUNTED=1 GROUP=0/2 RT_WIDE_COOP=256 RT_WIDE_HEAVY_WAVES=8
done
