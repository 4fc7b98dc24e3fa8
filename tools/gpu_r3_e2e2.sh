#!/bin/bash
# Round 3: e2e configs 2 / 4 / 3 after the job-list identity and upload work (each twice: host-noise range)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r3_e2e2.jsonl
rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 600 "$@" 2>gpurun_out/r3g_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b c2e2e python benchmarks/bench_configs.py --config 2e2e --steps 30 --warmup 3 &&
b c4e2e_log300 python benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 --hpa-log-interval 300 &&
b c3e2e python benchmarks/bench_configs.py --config 3e2e --steps 30 --warmup 3 &&
b c2e2e_b python benchmarks/bench_configs.py --config 2e2e --steps 30 --warmup 3 &&
b c4e2e python benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3
echo rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/r3_e2e2.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["tag"], round(d["ms_per_step"], 3), c.get("span_ms_median_rank0"))
PY
