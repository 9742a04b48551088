# N = 2 rehearsal of bench.py's multi-GPU path on a one-GPU box: two ranks on
# device 0 over gloo (RT_BENCH_SHARE_GPU / RT_BENCH_BACKEND: never set by the
# driver).  Output: gpurun_out/${TAG:-rehearse}/n2.log.
O=gpurun_out/${TAG:-rehearse}; mkdir -p $O
RT_BENCH_BACKEND=gloo RT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > $O/n2.log 2>&1 || exit 1
grep "^{" $O/n2.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('frame_check'), d.get('configs3',{}).get('ms_per_frame'), json.dumps(d.get('configs4_tiled')))"
