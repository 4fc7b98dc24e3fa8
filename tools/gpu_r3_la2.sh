#!/bin/bash
# Round 3: A-fragment lookahead depth in the pipelined LSTM kernel (4:1p = two k-steps ahead, 4:214 = one)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_model_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stack or lstm" > gpurun_out/la2_tests.log 2>&1 || { tail -30 gpurun_out/la2_tests.log; exit 1; }
tail -1 gpurun_out/la2_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py --tilings 4:214,4:1p,4:214,4:1p > gpurun_out/la2_10k.jsonl 2> gpurun_out/la2_10k.err || { tail -20 gpurun_out/la2_10k.err; exit 1; }
tail -1 gpurun_out/la2_10k.jsonl
timeout -k 10 200 python -u tools/lstm_stack_ab.py --batch 80000 --tilings 4:214,4:1p > gpurun_out/la2_80k.jsonl 2> gpurun_out/la2_80k.err || { tail -20 gpurun_out/la2_80k.err; exit 1; }
tail -1 gpurun_out/la2_80k.jsonl
echo done
