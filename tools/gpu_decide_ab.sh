#!/bin/bash
# headline: decision on the comm stream (default) vs on the compute stream, interleaved, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/decide_ab.txt
rm -f $out
for i in 1 2 3 4; do
  for d in comm compute; do
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 --decide-on $d > gpurun_out/dab.jsonl 2>&1 || exit 1
    echo "$d $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dab.jsonl) $(grep -o '"p50_decision_latency_ms": [0-9.]*' gpurun_out/dab.jsonl)" >> $out
  done
done
cat $out
