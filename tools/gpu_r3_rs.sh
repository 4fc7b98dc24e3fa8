#!/bin/bash
# Round 3: the row-streamed BT = 64 two-layer LSTM kernel (4:2p) vs the layer-pipelined one (4:1p)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_model_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "stack" > gpurun_out/rs_tests.log 2>&1 || { tail -40 gpurun_out/rs_tests.log; exit 1; }
tail -1 gpurun_out/rs_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py --tilings 4:1p,4:2p,4:1p,4:2p > gpurun_out/rs_10k.jsonl 2> gpurun_out/rs_10k.err || { tail -20 gpurun_out/rs_10k.err; exit 1; }
tail -1 gpurun_out/rs_10k.jsonl
timeout -k 10 200 python -u tools/lstm_stack_ab.py --batch 80000 --tilings 4:1p,4:2p > gpurun_out/rs_80k.jsonl 2> gpurun_out/rs_80k.err || { tail -20 gpurun_out/rs_80k.err; exit 1; }
tail -1 gpurun_out/rs_80k.jsonl
echo done
