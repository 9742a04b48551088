# Whitted 1080p frame under RT_WHITTED_SPLIT=p,q (the first of two streams takes p of every p+q row groups).
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for sp in default 1,1 3,2 5,4 4,3 2,1 7,5; do
    if [ $sp = default ]; then unset RT_WHITTED_SPLIT; else export RT_WHITTED_SPLIT=$sp; fi
    echo "--- split=$sp round=$r"
    KERNEL=whitted LIBS=main ROUNDS=1 REPS=20 WARM=3 timeout -k 10 100 python -u tools/ab.py 2>&1 | grep whitted
  done
done
