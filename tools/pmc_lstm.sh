#!/bin/bash
# PMC counters for the config-4 LSTM kernel and the canary tick kernels
# (kernel-trace + counters only; no sys/runtime traces).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
rocprofv3 --list-avail > "$R/gpurun_out/pmc_avail.txt" 2>&1 || true
set -e
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU \
  -d "$R/gpurun_out/pmc_c4a" -o c4a -- python3 "$R/benchmarks/bench_configs.py" --config 4 --steps 2 --warmup 1 \
  > "$R/gpurun_out/pmc_c4a.log" 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  -d "$R/gpurun_out/pmc_c4b" -o c4b -- python3 "$R/benchmarks/bench_configs.py" --config 4 --steps 2 --warmup 1 \
  > "$R/gpurun_out/pmc_c4b.log" 2>&1
echo done
