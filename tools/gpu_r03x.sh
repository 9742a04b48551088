set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_smallpt.py -x -q --timeout 120 --timeout-method thread > $O/t_smallpt.log 2>&1
KERNEL=smallpt LIBS=pk0,pk1,pk1o6,pk1o5 ROUNDS=3 REPS=5 timeout -k 10 400 python -u tools/ab.py > $O/pk_full.log 2>&1
BAND=3/8 KERNEL=smallpt LIBS=pk0,pk1,pk1o6,pk1o5 ROUNDS=2 REPS=5 timeout -k 10 300 python -u tools/ab.py > $O/pk_band8.log 2>&1
