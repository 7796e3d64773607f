#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06o; mkdir -p $OUT; cd $R
for a in none sync mark zeros fbread; do
  timeout -k 10 150 python -u tools/check_lds_replay.py $a > $OUT/$a.log 2>&1 || { tail -5 $OUT/$a.log; exit 1; }
  grep -E "replay [3-7]:|vs gather" $OUT/$a.log
done
