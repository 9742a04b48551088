RT_BENCH_BACKEND=gloo RT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/n2.log 2>&1 || exit 1
grep "^{" gpurun_out/n2.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('frame_check'), d.get('configs3',{}).get('ms_per_frame'), d.get('configs4_tiled'))"
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/n1.log 2>&1 || exit 1
grep "^{" gpurun_out/n1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('configs3',{}).get('ms_per_frame'), d.get('configs4_tiled'), d['configs4']['ms_per_frame'])"
