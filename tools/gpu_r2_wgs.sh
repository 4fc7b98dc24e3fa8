#!/bin/bash
# headline front-kernel role split sweep (pairwise:history workgroups per CU), two interleaved passes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/wgs_sweep.txt
for pass in 1 2; do
  for w in 1:4 1:5 1:6 0.5:4 0.75:4 1:8 2:6 0.5:5; do
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 --front-wgs $w > gpurun_out/wgs.jsonl 2>&1 || exit 1
    echo "wgs=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wgs.jsonl)" >> gpurun_out/wgs_sweep.txt
  done
done
echo done
