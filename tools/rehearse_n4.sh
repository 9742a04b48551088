# Four ranks sharing the one GPU over gloo (RT_BENCH_SHARE_GPU): the N = 4
# bench path end to end (bands, gather, frame_check, per-rank fields).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RT_BENCH_BACKEND=gloo RT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/n4.log 2>&1
grep "^{" gpurun_out/n4.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('frame_check'), d.get('ranks'), d.get('configs4_tiled'))"
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/n1.log 2>&1
grep "^{" gpurun_out/n1.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('configs4_tiled'), d['configs4'])"
