#!/bin/bash
# A (baseline build, default split) vs B (in-tree build) at several front-kernel splits, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab_wgs.txt
rm -f $out
for i in 1 2 3; do
  FOREMAST_HIP_LIB=$GRAFT_REPO_ROOT/gpurun_ab_base.so timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/ab.jsonl 2>&1 || exit 1
  echo "A 1:4 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.jsonl)" >> $out
  for w in 1:2 1:3 1:4; do
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 --front-wgs $w > gpurun_out/ab.jsonl 2>&1 || exit 1
    echo "B $w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.jsonl)" >> $out
  done
done
cat $out
