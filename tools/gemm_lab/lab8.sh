set -o pipefail
mkdir -p gpurun_out/lab8
LAB_ONLY="lib f16p,v6,v7,v8" timeout -k 10 300 python -u tools/gemm_lab/run_lab.py > gpurun_out/lab8/lab.txt 2>&1
