#!/bin/bash
# Round 3: stacked-LSTM numerics, A/B at the config-4 multivariate shape (10k x 240) and the univariate
# fleet shape (80k sequences), then the config-2 request-count traffic check
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "lstm_stack" > gpurun_out/lstm_r3_tests.log 2>&1 || { tail -30 gpurun_out/lstm_r3_tests.log; exit 1; }
tail -2 gpurun_out/lstm_r3_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py --tilings 4:2,4:1p,2:1p,4:1f > gpurun_out/lstm_r3_ab4.jsonl 2> gpurun_out/lstm_r3_ab4.err || { tail -20 gpurun_out/lstm_r3_ab4.err; exit 1; }
tail -1 gpurun_out/lstm_r3_ab4.jsonl
timeout -k 10 300 python -u tools/lstm_stack_ab.py --batch 80000 --tilings 4:2,4:1p,2:1p > gpurun_out/lstm_r3_ab80k.jsonl 2> gpurun_out/lstm_r3_ab80k.err || { tail -20 gpurun_out/lstm_r3_ab80k.err; exit 1; }
tail -1 gpurun_out/lstm_r3_ab80k.jsonl
bash tools/pmc_c2_req.sh
