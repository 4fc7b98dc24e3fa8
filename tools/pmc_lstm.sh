#!/bin/bash
# PMC counters of the LSTM kernel variants (tools/lstm_ab.py: column tiling x
# cell form), two passes of <= 8 SQ counters each, kernel-trace + counters
# only (no sys/runtime traces).  Summarise with tools/pmc_summary.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
set -e
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 \
  SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES \
  -d "$R/gpurun_out/pmc_lstm_a" -o a -- python3 "$R/tools/lstm_ab.py" > "$R/gpurun_out/pmc_lstm_a.log" 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_CYCLES SQ_ACTIVE_INST_MISC \
  -d "$R/gpurun_out/pmc_lstm_b" -o b -- python3 "$R/tools/lstm_ab.py" > "$R/gpurun_out/pmc_lstm_b.log" 2>&1
echo done
