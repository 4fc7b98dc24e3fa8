#!/bin/bash
# H = 256 stacked-LSTM tiling A/B (FM_LSTM_STACK_TILING) on config 4 (2 layers, multivariate) + numerics
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "lstm_stack" > gpurun_out/lstmtile_tests.log 2>&1 || exit 1
for t in 4:1 4:2 4:1 4:2; do
  FM_LSTM_STACK_TILING=$t timeout -k 10 200 python benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate > gpurun_out/c4_tile.jsonl 2>&1 || exit 1
  echo "tiling=$t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c4_tile.jsonl)" >> gpurun_out/lstm_tile_ab.txt
done
echo done
