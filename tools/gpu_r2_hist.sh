#!/bin/bash
# history-role register diet (masked rows re-read, unclamped in-row loads): canary numerics + headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_canary_ops.py tests/test_fastpath.py -m gpu > gpurun_out/hist_tests.log 2>&1 || { tail -30 gpurun_out/hist_tests.log; exit 1; }
tail -2 gpurun_out/hist_tests.log
rm -f gpurun_out/hist_bench.txt
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/hb.jsonl 2>&1 || exit 1
  echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hb.jsonl)" >> gpurun_out/hist_bench.txt
done
timeout -k 10 120 python bench.py --steps 300 --warmup 30 --services 1250 > gpurun_out/hb1250.jsonl 2>&1 || exit 1
echo "1250: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hb1250.jsonl)" >> gpurun_out/hist_bench.txt
cat gpurun_out/hist_bench.txt
