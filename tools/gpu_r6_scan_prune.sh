#!/bin/bash
# Scan-fit pruning: the HW fit GPU tests, the exact vs pruned A/B on the
# config-2 series, and config 2 itself (zoo.decide, pruned by default).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_model_ops.py \
  -k "hw_scan or es_fit or es_update" > gpurun_out/sp_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/sp_tests.log; exit 1; }
tail -1 gpurun_out/sp_tests.log
timeout -k 10 300 python -u tools/hw_scan_prune_ab.py > gpurun_out/scan_prune_ab.jsonl 2> gpurun_out/sp_ab.err || { echo ab failed; tail -5 gpurun_out/sp_ab.err; exit 1; }
cat gpurun_out/scan_prune_ab.jsonl
for pr in 0 1.25; do
  FOREMAST_HW_SCAN_PRUNE=$pr timeout -k 10 300 python -u benchmarks/bench_configs.py --config 2 --steps 10 --warmup 2 > gpurun_out/sp_c2_$pr.log 2>&1 || { echo c2 failed; tail -5 gpurun_out/sp_c2_$pr.log; exit 1; }
  grep '^{' gpurun_out/sp_c2_$pr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config2 prune=$pr', round(d['ms_per_step'],3))"
done
