#!/bin/bash
# Round 3: the production cycle on the shipped topology (REST service process + SQLite),
# vs the in-memory store, and with a concurrent /metrics scraper.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r3_store.jsonl
rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 400 "$@" 2>gpurun_out/r3s_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b sqlite python benchmarks/bench_configs.py --config 3e2e --store sqlite --steps 50 --warmup 5 &&
b memory python benchmarks/bench_configs.py --config 3e2e --store memory --steps 50 --warmup 5 &&
b sqlite_scrape python benchmarks/bench_configs.py --config 3e2e --store sqlite --steps 50 --warmup 5 --scrape-interval 0.02
echo rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/r3_store.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["tag"], round(d["ms_per_step"], 3), c.get("span_ms_median_rank0"), c.get("rest_poller"), c.get("scraper"))
PY
