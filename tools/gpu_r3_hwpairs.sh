#!/bin/bash
# Round 3: Holt-Winters grid fit, two candidates per thread (hw2_fit_kernel) vs two pairs per thread
# (hwp_fit_kernel<2>, FM_HW_PAIRS=2): numerics under FM_HW_PAIRS=2, config 2 at 10k / 7k services
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FM_HW_PAIRS=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "es_fit or es_update" > gpurun_out/hwpairs_tests.log 2>&1 || { tail -30 gpurun_out/hwpairs_tests.log; exit 1; }
tail -2 gpurun_out/hwpairs_tests.log
out=gpurun_out/hwpairs.jsonl; rm -f $out
for s in 10000 7000; do for p in 1 2 1 2; do
  FM_HW_PAIRS=$p timeout -k 10 300 python benchmarks/bench_configs.py --config 2 --services $s > gpurun_out/hwp.json 2> gpurun_out/hwp.err || { tail -20 gpurun_out/hwp.err; exit 1; }
  echo "{\"pairs\": $p, \"services\": $s, \"ms\": $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hwp.json | cut -d' ' -f2)}" | tee -a $out
done; done
