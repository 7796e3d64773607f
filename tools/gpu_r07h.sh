R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r07h; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_skip_fold.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_skip_from_go.py > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log | tail -3; exit $rc
