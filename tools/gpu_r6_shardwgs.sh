#!/bin/bash
# Round 6: front kernel workgroups per CU (pairwise:history) at the
# 1,250-service shard (the per-rank size of the 8-GPU strong-scaling run).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/shard_wgs.jsonl
: > $OUT
for rep in 1 2; do
  for w in ${WGS:-1:4 1:3 1:2 0.5:3 0.5:2 1:1}; do
    timeout -k 10 120 python -u bench.py --services 1250 --steps 1000 --warmup 50 --front-wgs $w > gpurun_out/sw_b.log 2>&1 \
      || { echo "bench $w failed"; tail -5 gpurun_out/sw_b.log; exit 1; }
    grep '^{' gpurun_out/sw_b.log >> $OUT
    grep '^{' gpurun_out/sw_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', round(d['ms_per_step'],4), round(d['p50_decision_latency_ms'],4))"
  done
done
