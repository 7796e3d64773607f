mkdir -p gpurun_out/rcab
GATX_LIB=$PWD/tools/gemm_lab/libgatx_rc2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_layer.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "wgrad or backward" > gpurun_out/rcab/tests.log 2>&1 && tail -1 gpurun_out/rcab/tests.log &&
for r in a b; do
  timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > gpurun_out/rcab/base_$r.json 2>/dev/null &&
  GATX_LIB=$PWD/tools/gemm_lab/libgatx_rc2.so timeout -k 10 300 python bench.py --mode train --no-cpu-baseline > gpurun_out/rcab/rc2_$r.json 2>/dev/null || exit 1
done &&
python -c "
import json
for r in 'ab':
    for v in ('base','rc2'):
        d=json.load(open(f'gpurun_out/rcab/{v}_{r}.json'))
        print(v, r, d['ms_per_step'], round(d['kernels']['bwd_gemm_gw']['avg_ms']*1e3,1))
"
