#!/bin/bash
# One parametrised GPU-box job (replaces round 3's one-off gpu_r03*.sh):
#
#   gpurun -- bash tools/gpu_job.sh TAG STEP [STEP ...]
#
# Output under gpurun_out/TAG/.  Each step runs under its own time limit and
# the job stops at the first failing step (set -e), so a fault or a hang ends
# the job instead of starting more GPU work.  Steps:
#   tests               the whole -m gpu suite
#   tests:FILE[:K]      one test file (optionally -k K)
#   smoke               __graft_entry__.smoke()
#   bench               python bench.py (default line)         -> bench.json
#   prof                tools/prof_round.sh TAG (bench + rocprofv3 stats + PMC passes)
#   c4part              tools/c4_partition.py (configs[4] N=4/8 per-rank proxy)
#   c4time[:GROUP]      tools/c5_time.py, 64 spp, 5 reps (GROUP=k/N: an interleaved share)
#   stress              tools/bvh_stress.py REPEAT=2 N=60
#   ab:KERNEL:LIBS      tools/ab.py A/B of build_ab/<lib> variants (KERNEL=smallpt|whitted|queue|c4)
#   py:SCRIPT[:ARGS]    any tools/ script, e.g. py:queue_time.py:20
# Environment passes through (e.g. RT_HIP_LIB=..., REPS=...).
set -e
TAG=${1:?tag}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p "$O"
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for step in "$@"; do
  echo "== $step ($(date +%T))" | tee -a "$O/job.log"
  case "$step" in
    tests) timeout -k 10 1100 $PYT tests -m gpu > "$O/gputests.log" 2>&1 ;;
    tests:*) IFS=: read -r _ f k <<< "$step"
             timeout -k 10 600 $PYT "tests/$f" ${k:+-k "$k"} > "$O/t_$(basename "$f" .py).log" 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 ;;
    bench) timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" ;;
    prof) bash tools/prof_round.sh "$TAG" ;;
    c4part) timeout -k 10 400 python -u tools/c4_partition.py > "$O/c4_partition.log" 2>&1 ;;
    c4time*) g=${step#c4time}; g=${g#:}
             SPP=64 REPS=5 GROUP=$g timeout -k 10 200 python -u tools/c5_time.py >> "$O/c4time.log" 2>&1 ;;
    stress) REPEAT=2 N=60 SEED=11 timeout -k 10 500 python -u tools/bvh_stress.py > "$O/bvh_stress.log" 2>&1 ;;
    ab:*) IFS=: read -r _ kern libs <<< "$step"
          KERNEL=$kern LIBS=$libs timeout -k 10 500 python -u tools/ab.py >> "$O/ab_$kern.log" 2>&1 ;;
    py:*) IFS=: read -r _ script args <<< "$step"
          timeout -k 10 500 python -u "tools/$script" $args >> "$O/$(basename "$script" .py).log" 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "job done ($(date +%T))" | tee -a "$O/job.log"
