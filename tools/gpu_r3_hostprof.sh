#!/bin/bash
# Round 3: host profiles (cProfile over the timed cycles) of configs 2e2e and 4e2e on the GPU box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python tools/profile_3e2e.py --config 2e2e --steps 10 --warmup 2 > gpurun_out/host_c2e2e.txt 2>&1 || { tail -20 gpurun_out/host_c2e2e.txt; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"span_ms_median_rank0": {[^}]*}' gpurun_out/host_c2e2e.txt
timeout -k 10 600 python tools/profile_3e2e.py --config 4e2e --steps 8 --warmup 2 --hpa-log-interval 300 > gpurun_out/host_c4e2e.txt 2>&1 || { tail -20 gpurun_out/host_c4e2e.txt; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"span_ms_median_rank0": {[^}]*}' gpurun_out/host_c4e2e.txt
