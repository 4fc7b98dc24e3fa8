#!/bin/bash
# Round 3: e2e benches of configs 2 and 4 (Brain.run_once over the shipped SQLite topology) after the host-path work
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r3_e2e.jsonl
rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 600 "$@" 2>gpurun_out/r3e_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b c2e2e python benchmarks/bench_configs.py --config 2e2e --steps 30 --warmup 3 &&
b c4e2e python benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 &&
b c4e2e_log300 python benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 --hpa-log-interval 300
echo rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/r3_e2e.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["tag"], round(d["ms_per_step"], 3), c.get("rows_per_cycle_rank0"), c.get("span_ms_median_rank0"), c.get("model_cache"))
PY
