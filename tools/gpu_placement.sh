#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/placement.txt
rm -f $out
for i in 1 2; do
  for p in 0 2 64 512 1000 1500 3000; do
    PAD_MB=$p timeout -k 10 120 python tools/placement_probe.py --steps 300 --warmup 30 > gpurun_out/pp.jsonl 2>&1 || exit 1
    echo "pad=$p $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pp.jsonl)" >> $out
  done
done
cat $out
