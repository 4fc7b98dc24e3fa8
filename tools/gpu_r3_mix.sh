#!/bin/bash
# Round 3: stacked-LSTM numerics + tiling A/B (incl. the layer-pipelined kernel), then the e2e benches of configs 2 and 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "lstm_stack" > gpurun_out/lstm_r3_tests.log 2>&1 || { tail -30 gpurun_out/lstm_r3_tests.log; exit 1; }
tail -2 gpurun_out/lstm_r3_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py > gpurun_out/lstm_r3_ab2.jsonl 2> gpurun_out/lstm_r3_ab2.err || { tail -20 gpurun_out/lstm_r3_ab2.err; exit 1; }
tail -1 gpurun_out/lstm_r3_ab2.jsonl
bash tools/gpu_r3_e2e.sh
