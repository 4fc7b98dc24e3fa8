#!/bin/bash
# 16x16-tile two-layer LSTM (FM_LSTM_STACK_TILING=8:216): numerics against the
# bf16-emulating reference / fp32 torch.nn.LSTM, then the A/B against the
# row-streamed 32x32 kernel (4:2p) at 10k x 240, H = 256 x 2.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_model_ops.py \
  -k "lstm_stack" > gpurun_out/l16_tests.log 2>&1 || { echo lstm tests failed; tail -40 gpurun_out/l16_tests.log; exit 1; }
tail -1 gpurun_out/l16_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py --tilings 4:2p,8:216,4:2p,8:216 > gpurun_out/lstm16_ab.jsonl 2> gpurun_out/l16_ab.err || { echo ab failed; tail -5 gpurun_out/l16_ab.err; exit 1; }
cat gpurun_out/lstm16_ab.jsonl
