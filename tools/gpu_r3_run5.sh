#!/bin/bash
# Round 3: e2e configs 2/4 after the hpalog batch + memo work, then PMC of the stacked LSTM variants
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_r3_e2e.sh && bash tools/pmc_lstm_stack.sh
