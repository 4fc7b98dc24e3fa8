#!/bin/bash
# Same-box A/B of two builds of the HIP library on the headline bench:
# A = $GRAFT_REPO_ROOT/gpurun_ab_base.so (baseline build), B = the in-tree build.
# usage: tools/gpu_ab_lib.sh [rounds] [extra bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=${1:-4}; shift || true
out=gpurun_out/ab_lib.txt
rm -f $out
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then lib=$GRAFT_REPO_ROOT/gpurun_ab_base.so; else lib=$GRAFT_REPO_ROOT/foremast_amd/_native/libforemast_hip.so; fi
    FOREMAST_HIP_LIB=$lib timeout -k 10 120 python bench.py --steps 300 --warmup 30 "$@" > gpurun_out/ab.jsonl 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.jsonl)" >> $out
  done
done
cat $out
