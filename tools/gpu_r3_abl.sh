#!/bin/bash
# Round 3: ablations of the pipelined LSTM kernel (no cell math / L2-hot weights / both), then the e2e configs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/lstm_stack_ab.py --tilings 4:1p,4:211,4:212,4:213,4:1p > gpurun_out/lstm_abl.jsonl 2> gpurun_out/lstm_abl.err || { tail -20 gpurun_out/lstm_abl.err; exit 1; }
tail -1 gpurun_out/lstm_abl.jsonl
bash tools/gpu_r3_e2e2.sh
