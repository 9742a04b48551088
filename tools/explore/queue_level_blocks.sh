# Queue level_kernel grid sweep (profiles/r04/queue_level_grid_ab.log). The RT_QUEUE_LEVEL_BLOCKS hook it sets was a temporary A/B build and is not in queue.hip.
cd $GRAFT_REPO_ROOT
for b in 0 1024 1536 2560 3072 4096; do
  echo "--- blocks=$b"; RT_QUEUE_LEVEL_BLOCKS=$b timeout -k 10 100 python -u tools/queue_time.py 20 2>&1 | grep ms
done
