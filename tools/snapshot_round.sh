#!/bin/bash
# Copy what tools/gpu_round.sh TAG left under gpurun_out/TAG into profiles/TAG (tracked): the
# bench lines, the GPU test log, rocprofv3 kernel stats + the windowed per-step breakdowns
# (tools/trace_window.py) and the windowed PMC summaries; also refresh profiles/pmc_latest.json
# and profiles/pmc_rmat.json, which bench.py reads.
#   bash tools/snapshot_round.sh TAG
set -e
T=$1
S=gpurun_out/$T
D=profiles/$T
mkdir -p "$D"
cp "$S"/bench.json "$S"/bench_train.json "$S"/bench_rmat.json "$S"/bench_pattern_train.json "$S"/bench_ppi2_train.json "$S"/gpu_tests.log "$D"/
for p in fwd train rmat pattern; do
  cp "$S/prof_$p/run_kernel_stats.csv" "$D/${p}_kernel_stats.csv"
  python tools/trace_window.py "$S/prof_$p" "$D/${p}_breakdown.txt" > /dev/null
done
PMC_SOURCE="bench.py --steps 3 --warmup 1" \
  python tools/pmc_summary.py "$S/pmc" profiles/pmc_latest.json > "$D/fwd_pmc_summary.txt"
PMC_SOURCE="bench.py --mode train --steps 3 --warmup 1" \
  python tools/pmc_summary.py "$S/pmct" profiles/pmc_train.json > "$D/train_pmc_summary.txt"
PMC_SOURCE="bench.py --workload rmat --steps 1 --warmup 2" \
  python tools/pmc_summary.py "$S/pmcr" profiles/pmc_rmat.json > "$D/rmat_pmc_summary.txt"
echo "snapshot in $D"
