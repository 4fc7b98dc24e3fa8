#!/bin/bash
# Round 6: XCD balancing parameters A/B at 10k services: off, the default
# (a third of the way per tick past a 1.5 % spread) and a faster variant
# (half-way past 0.75 %: variants/libforemast_hip_bal2.so).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/xcd2_ab.jsonl
L=$R/foremast_amd/_native/libforemast_hip.so
V=$R/foremast_amd/_native/variants/libforemast_hip_bal2.so
for rep in 1 2 3; do
  for cfg in off:0:$L def:1:$L bal2:1:$V; do
    IFS=: read tag b lib <<< "$cfg"
    FM_XCD_BALANCE=$b FOREMAST_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/xcd2_b.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/xcd2_b.log; exit 1; }
    grep '^{' gpurun_out/xcd2_b.log | sed "s/^{/{\"xcd\": \"$tag\", /" >> gpurun_out/xcd2_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/xcd2_ab.jsonl'):
    d=json.loads(l); print(d['xcd'], round(d['ms_per_step'],4))"
