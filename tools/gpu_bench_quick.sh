#!/bin/bash
# Headline bench.py + config 2 (Holt-Winters grid) one line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 python -u benchmarks/bench_configs.py --config 2 --steps 20 --warmup 3 > gpurun_out/c2.log 2>&1 || exit 1
grep '^{' gpurun_out/c2.log | cut -c1-600
