#!/bin/bash
# round 6: resid piece loaded ahead in the concat walk's last pair step (RES): tests, then an
# interleaved library A/B against the previous build (tools/ab/libgatx_base.so) and a trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r09d; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_lds.py tests/test_gpu_headline.py tests/test_gpu_capture.py tests/test_gpu_skip.py tests/test_gpu_dropout.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/gpu_lib_ab.sh r09d_ab 3 "" gat-pytorch_amd/gatx/libgatx.so tools/ab/libgatx_base.so || exit 1
bash tools/gpu_args_trace.sh r09d_tr "" "-"
# probes (timing only, wrong results by design; bench.py's replay check may fail on them): the
# LDS walks without their walk / without their staging
cd /tmp && export TMPDIR=/tmp
for v in NOSTAGE NOWALK; do
  GATX_LIB=$R/tools/ab/libgatx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/probe_$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-train-leg > "$OUT/probe_$v.log" 2>&1
  rc=$?; echo "probe $v rc=$rc"; [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && exit 1
  python3 "$R/tools/trace_window.py" "$OUT/probe_$v" "$OUT/probe_$v.txt" | grep -E "edge_lds|edge_records|steps in"
done
