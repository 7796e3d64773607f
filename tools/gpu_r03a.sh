R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03a; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_distributed.py -m gpu > $OUT/dist.log 2>&1; rc=$?; tail -12 $OUT/dist.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; cat $OUT/bench.json | head -c 3000; exit $rc
