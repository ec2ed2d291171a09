#!/bin/bash
# Copy one tools/profile.sh run (gpurun_out/*_$TAG, merged back by gpurun) into
# profiles/$TAG and summarise it (tools/summarize_profile.py).
set -euo pipefail
TAG=$1
cd "$(dirname "$0")/.."
G=gpurun_out
D=profiles/$TAG
mkdir -p "$D"
cp "$G/prof_$TAG/run_kernel_stats.csv" "$D/kernel_stats.csv"
cp "$G/prof_$TAG.bench.json" "$D/bench_under_rocprof.json"
cp "$G/pmc_fetch_$TAG/run_counter_collection.csv" "$D/pmc_fetch_size.csv"
cp "$G/pmc_write_$TAG/run_counter_collection.csv" "$D/pmc_write_size.csv"
cp "$G/pmc_sq_$TAG/run_counter_collection.csv" "$D/pmc_sq.csv"
if [ -f "$G/pmc_wait_$TAG/run_counter_collection.csv" ]; then
  cp "$G/pmc_wait_$TAG/run_counter_collection.csv" "$D/pmc_wait.csv"
fi
python3 tools/summarize_profile.py "$TAG" ${PMC_HEADERS:+--pmc-headers $PMC_HEADERS} > /dev/null
echo "profiles/$TAG: $(ls "$D" | tr '\n' ' ')"
