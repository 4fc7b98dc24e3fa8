#!/bin/bash
# Round 3: e2e configs 2/4 after the hpalog batch + memo work, PMC of the stacked LSTM variants, config 2 timing + traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_r3_e2e.sh && bash tools/pmc_lstm_stack.sh &&
timeout -k 10 300 python benchmarks/bench_configs.py --config 2 > gpurun_out/c2_r3.jsonl 2> gpurun_out/c2_r3.err &&
tail -1 gpurun_out/c2_r3.jsonl && bash tools/pmc_c2.sh
