set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03y; mkdir -p $O
KERNEL=whitted REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/wt -o w -- python3 tools/ab.py child > $O/wt.log 2>&1
python3 tools/wf_timeline.py $O/wt > $O/timeline.txt 2>&1
