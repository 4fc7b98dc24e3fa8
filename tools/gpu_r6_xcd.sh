#!/bin/bash
# Round 6: XCD-balanced history ranges (canary.hip xcd_rebalance): numerics,
# per-XCD end times with the balancing on, and a same-box A/B against
# FM_XCD_BALANCE=0 at 10k services and the 1,250-service shard.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_canary_ops.py tests/test_fastpath.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/xcd_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/xcd_tests.log; exit 1; }
tail -1 gpurun_out/xcd_tests.log
FOREMAST_HIP_LIB=$R/foremast_amd/_native/variants/libforemast_hip_timing.so SHAPES=10000 WGS=1:4 REPS=8 \
  timeout -k 10 200 python -u tools/front_timing.py > gpurun_out/xcd_timing.log 2>&1 || { echo timing failed; tail -5 gpurun_out/xcd_timing.log; exit 1; }
grep '^{' gpurun_out/xcd_timing.log
rm -f gpurun_out/xcd_ab.jsonl
for rep in 1 2 3; do
  for b in 0 1; do
    FM_XCD_BALANCE=$b timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/xcd_b.log 2>&1 || { echo "bench $b failed"; tail -5 gpurun_out/xcd_b.log; exit 1; }
    grep '^{' gpurun_out/xcd_b.log | sed "s/^{/{\"xcd_balance\": $b, \"services\": 10000, /" >> gpurun_out/xcd_ab.jsonl
    FM_XCD_BALANCE=$b timeout -k 10 120 python -u bench.py --services 1250 --steps 1000 --warmup 50 > gpurun_out/xcd_b.log 2>&1 || { echo "shard $b failed"; exit 1; }
    grep '^{' gpurun_out/xcd_b.log | sed "s/^{/{\"xcd_balance\": $b, \"services\": 1250, /" >> gpurun_out/xcd_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/xcd_ab.jsonl'):
    d=json.loads(l); print(d['xcd_balance'], d['services'], round(d['ms_per_step'],4))"
