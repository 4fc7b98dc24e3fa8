#!/bin/bash
# Stacked-LSTM kernel A/B at H = 256 x 2 (register lookahead vs LDS-DMA weight ring) + numerics + config 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "lstm_stack" > gpurun_out/lstm_r3_tests.log 2>&1 || { tail -30 gpurun_out/lstm_r3_tests.log; exit 1; }
tail -2 gpurun_out/lstm_r3_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py > gpurun_out/lstm_r3_ab.jsonl 2> gpurun_out/lstm_r3_ab.err || { tail -20 gpurun_out/lstm_r3_ab.err; exit 1; }
cat gpurun_out/lstm_r3_ab.jsonl
for t in 4:2 4:1 4:1g; do
  FM_LSTM_STACK_TILING=$t timeout -k 10 200 python benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate > gpurun_out/c4_tile_r3.jsonl 2>gpurun_out/c4_tile_r3.err || { tail -20 gpurun_out/c4_tile_r3.err; exit 1; }
  echo "tiling=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4_tile_r3.jsonl)" | tee -a gpurun_out/lstm_r3_c4.txt
done
echo done
