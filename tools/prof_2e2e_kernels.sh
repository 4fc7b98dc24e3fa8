#!/bin/bash
# Kernel trace of the 2e2e brain cycle (rocprofv3 --kernel-trace --stats only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof2e2e
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2e2e -o run -- \
  python3 benchmarks/bench_configs.py --config 2e2e --steps 10 --warmup 2 > gpurun_out/prof2e2e.log 2>&1 || exit 1
f=$(find gpurun_out/prof2e2e -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py "$f" > gpurun_out/prof2e2e_summary.txt 2>&1 || exit 1
head -30 gpurun_out/prof2e2e_summary.txt
