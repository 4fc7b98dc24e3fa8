#!/bin/bash
# Round 3: GPU tests (model fast path parity, gather kernel) + e2e benches of configs 2 and 4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r3_models.jsonl
rm -f $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_r3_models.log 2>&1 || { tail -40 gpurun_out/gputests_r3_models.log; exit 1; }
tail -1 gpurun_out/gputests_r3_models.log
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 600 "$@" 2>gpurun_out/r3m_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b c2e2e python benchmarks/bench_configs.py --config 2e2e --steps 30 --warmup 3 &&
b c2cached python benchmarks/bench_configs.py --config 2 --cached &&
b c4e2e python benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 &&
b c4e2e_log300 python benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 --hpa-log-interval 300
echo rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/r3_models.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["tag"], round(d["ms_per_step"], 3), c.get("rows_per_cycle_rank0"), c.get("span_ms_median_rank0"), c.get("model_cache"))
PY
