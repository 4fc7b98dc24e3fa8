#!/bin/bash
# Packed Holt-Winters block pipeline A/B (FM_HW_PIPE 0/1/2) on config 2 + the ES numerics tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "es or hw or holt or smoothing" > gpurun_out/hw_tests.log 2>&1 &&
for p in 0 1 2 0 1 2; do
  FM_HW_PIPE=$p timeout -k 10 200 python benchmarks/bench_configs.py --config 2 > gpurun_out/c2_pipe$p.jsonl 2>&1 || exit 1
  echo "pipe=$p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c2_pipe$p.jsonl)" >> gpurun_out/hw_pipe_ab.txt
done
echo rc=$?
