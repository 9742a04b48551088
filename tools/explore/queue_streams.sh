# 800x600 / 1080p queue frame under the slab / stream A/B hooks (no rebuild).
cd "$GRAFT_REPO_ROOT"
for cfg in "" "RT_QUEUE_STREAMS=2" "RT_QUEUE_STREAMS=2 RT_QUEUE_SLABS=3" "RT_QUEUE_STREAMS=2 RT_QUEUE_SLABS=4" "RT_QUEUE_SLAB_TREES=3000000" "RT_QUEUE_SLAB_TREES=9000000"; do
  for r in 1 2; do
    echo "--- [$cfg] round=$r"; env $cfg timeout -k 10 100 python -u tools/queue_time.py 20 2>&1 | grep ms
  done
done
