#!/bin/bash
# PMC counters of the FFT period-detection kernel (config 2 --detect-period),
# one pass of <= 8 SQ counters, kernel-trace + counters only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
set -e
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$R/gpurun_out/pmc_fft_a" -o a -- python3 "$R/benchmarks/bench_configs.py" --config 2 --detect-period \
  --steps 1 --warmup 1 > "$R/gpurun_out/pmc_fft_a.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM \
  SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA \
  -d "$R/gpurun_out/pmc_fft_b" -o b -- python3 "$R/benchmarks/bench_configs.py" --config 2 --detect-period \
  --steps 1 --warmup 1 > "$R/gpurun_out/pmc_fft_b.log" 2>&1
# keep only the per-kernel summaries (the databases exceed what gpurun copies back)
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_fft_a" "$R/gpurun_out/pmc_fft_b" --kernel fft_ > "$R/gpurun_out/pmc_fft.txt"
rm -rf "$R/gpurun_out/pmc_fft_a" "$R/gpurun_out/pmc_fft_b"
echo done
