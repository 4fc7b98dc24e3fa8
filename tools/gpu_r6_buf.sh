#!/bin/bash
# Round 6: history rows through buffer loads (front kernel 111 -> 87 VGPRs,
# five waves per SIMD).  Numerics (canary ops, fast path == general path),
# then a same-box A/B: round-5 canary.hip (variants/libforemast_hip_r5.so),
# the new masked path with flat loads (variants/libforemast_hip_flat.so) and
# the default build, at several pairwise:history workgroup ratios, 10k
# services and the 1,250-service shard; then a kernel table of the default.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
V=$R/foremast_amd/_native/variants
run() { name=$1; secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; rc=$?; echo "$name rc=$rc"; return $rc; }
run buf_tests 400 python -u -m pytest tests/test_canary_ops.py -m gpu -x -v \
    --timeout 120 --timeout-method thread || { tail -30 gpurun_out/buf_tests.log; exit 1; }
rm -f gpurun_out/buf_ab.jsonl
one() { lib=$1; tag=$2; wgs=$3; svc=$4; steps=$5
  FOREMAST_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --services $svc --front-wgs $wgs --steps $steps --warmup 20 \
    > gpurun_out/buf_b.log 2>&1 || { echo "bench $tag $wgs $svc failed"; tail -5 gpurun_out/buf_b.log; return 1; }
  grep '^{' gpurun_out/buf_b.log | sed "s/^{/{\"lib\": \"$tag\", \"services\": $svc, /" >> gpurun_out/buf_ab.jsonl; }
L=$R/foremast_amd/_native/libforemast_hip.so
for rep in 1 2 3; do
  one $V/libforemast_hip_r5.so r5 1:4 10000 400 || exit 1
  FM_FRONT_LDS=0 one $L buf_occ5 1:4 10000 400 || exit 1
  one $L buf_cap4 1:4 10000 400 || exit 1
  FM_FRONT_LDS=41984 one $L buf_cap3 1:4 10000 400 || exit 1
  FM_FRONT_LDS=41984 one $L buf_cap3 1:3 10000 400 || exit 1
  one $V/libforemast_hip_r5.so r5 1:4 1250 1000 || exit 1
  one $L buf_cap4 1:4 1250 1000 || exit 1
  FM_FRONT_LDS=41984 one $L buf_cap3 1:4 1250 1000 || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/buf_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['services'], d['config']['front_wgs_per_cu'], round(d['ms_per_step'],4))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/buf_prof" -o hl -- python3 "$R/bench.py" --steps 100 --warmup 10 > "$R/gpurun_out/buf_prof.log" 2>&1; echo "prof rc=$?"
