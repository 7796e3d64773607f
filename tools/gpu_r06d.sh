set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/r06d; mkdir -p $OUT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_api.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --mode train --graphs 2 --no-cpu-baseline > $OUT/ppi2_train.json 2> $OUT/ppi2_train.err || exit 1
timeout -k 10 300 python bench.py --mode train --graphs 2 --hipgraph off --no-cpu-baseline > $OUT/ppi2_train_eager.json 2> $OUT/ppi2_train_eager.err || exit 1
python -c "
import json
for f in ('ppi2_train','ppi2_train_eager'):
    d=json.load(open('$OUT/'+f+'.json')); print(f, d['ms_per_step'], d['config']['launch'])"
bash tools/gpu_ab.sh r06c 3 "" "-" "--tune edge_chunk=2245" "--tune edge_chunk=1122" || exit 1
cd tools/edge_lab && timeout -k 10 120 ./edge_lab > $OUT/edge_lab.txt 2>&1; rc=$?; cat $OUT/edge_lab.txt; exit $rc
