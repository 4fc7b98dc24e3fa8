#!/bin/bash
# rolling-bands kernel A/B: A = gpurun_ab_base.so, B = in-tree build, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab_rolling.txt
rm -f $out
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then lib=$GRAFT_REPO_ROOT/gpurun_ab_base.so; else lib=$GRAFT_REPO_ROOT/foremast_amd/_native/libforemast_hip.so; fi
    FOREMAST_HIP_LIB=$lib timeout -k 10 120 python tools/rolling_bench.py > gpurun_out/rb.jsonl 2>&1 || exit 1
    echo "$v $(grep -o '"window": [0-9]*, "ms": [0-9.]*' gpurun_out/rb.jsonl | tr '\n' ' ')" >> $out
  done
done
cat $out
