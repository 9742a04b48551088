set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_whitted.py -x -q --timeout 120 --timeout-method thread > $O/t_whitted.log 2>&1
KERNEL=whitted LIBS=tf0,tf1 ROUNDS=3 REPS=10 timeout -k 10 300 python -u tools/ab.py > $O/tf.log 2>&1
WH=640x480 KERNEL=whitted LIBS=tf0,tf1 ROUNDS=2 REPS=10 timeout -k 10 300 python -u tools/ab.py >> $O/tf.log 2>&1
KERNEL=whitted REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/wt -o w -- python3 tools/ab.py child > $O/wt.log 2>&1
python3 tools/wf_timeline.py $O/wt > $O/timeline.txt 2>&1
