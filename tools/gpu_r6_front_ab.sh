#!/bin/bash
# A/B of the front kernel's history role on one box: the committed library
# (FOREMAST_HIP_LIB=..._a.so) against the working tree's, after the
# numerics tests of the new one; headline and the 1,250-service shard,
# interleaved, three passes each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/front_ab_r6.jsonl
: > $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_canary_ops.py tests/test_fastpath.py > gpurun_out/fab_tests.log 2>&1 || { tail -30 gpurun_out/fab_tests.log; exit 1; }
tail -2 gpurun_out/fab_tests.log
A=$R/foremast_amd/_native/libforemast_hip_a.so
B=$R/foremast_amd/_native/libforemast_hip.so
for pass in 1 2 3; do
  for v in a b; do
    if [ $v = a ]; then L=$A; else L=$B; fi
    FOREMAST_HIP_LIB=$L timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 > gpurun_out/fab.log 2>&1 || exit 1
    grep '^{' gpurun_out/fab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['lib']='$v'; d['shard']=10000; open('$OUT','a').write(json.dumps(d)+'\n'); print('$v', '10k', round(d['ms_per_step'],4))"
    FOREMAST_HIP_LIB=$L timeout -k 10 120 python -u bench.py --services 1250 --steps 2000 --warmup 100 > gpurun_out/fab.log 2>&1 || exit 1
    grep '^{' gpurun_out/fab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['lib']='$v'; d['shard']=1250; open('$OUT','a').write(json.dumps(d)+'\n'); print('$v', '1250', round(d['ms_per_step'],4))"
  done
done
