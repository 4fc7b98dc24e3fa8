#!/bin/bash
# PMC counters of the H = 256 x 2 stacked-LSTM variants (tools/lstm_stack_ab.py:
# 4:1p layer-pipelined, 4:2p row-streamed BT = 64 (the two-layer default)), two
# passes of <= 8 SQ counters, kernel-trace + counters only.  Summarise with
# tools/pmc_summary.py --kernel lstm_stack.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
set -e
T="--tilings ${PMC_TILINGS:-4:1p,4:2p}"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 \
  SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES \
  -d "$R/gpurun_out/pmc_lstm_stack_a" -o a -- python3 "$R/tools/lstm_stack_ab.py" $T > "$R/gpurun_out/pmc_lstm_stack_a.log" 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/pmc_lstm_stack_b" -o b -- python3 "$R/tools/lstm_stack_ab.py" $T > "$R/gpurun_out/pmc_lstm_stack_b.log" 2>&1
cd "$R" && python3 tools/pmc_summary.py gpurun_out/pmc_lstm_stack_a gpurun_out/pmc_lstm_stack_b --kernel lstm_stack > gpurun_out/pmc_lstm_stack.txt
echo done
