#!/bin/bash
# PMC counters of the FFT period-detection kernel (tools/fft_bench.py, 40k x
# 10,080), one pass per counter group, kernel-trace + counters only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
set -e
B="python3 $R/tools/fft_bench.py --lengths 10080 --iters 2"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
  SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$R/gpurun_out/pmc_fft_a" -o a -- $B > "$R/gpurun_out/pmc_fft_a.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM \
  SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_FMA_F32 \
  -d "$R/gpurun_out/pmc_fft_b" -o b -- $B > "$R/gpurun_out/pmc_fft_b.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 \
  -d "$R/gpurun_out/pmc_fft_c" -o c -- $B > "$R/gpurun_out/pmc_fft_c.log" 2>&1
# keep only the per-kernel summaries (the databases exceed what gpurun copies back)
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_fft_a" "$R/gpurun_out/pmc_fft_b" "$R/gpurun_out/pmc_fft_c" \
  --kernel fft_ > "$R/gpurun_out/pmc_fft.txt"
rm -rf "$R/gpurun_out/pmc_fft_a" "$R/gpurun_out/pmc_fft_b" "$R/gpurun_out/pmc_fft_c"
echo done
