#!/bin/bash
# Round 3 full validation: every GPU test, smoke, the headline bench, configs 2 / 4 (H=256x2 mv) / 2e2e
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_r3_full.log 2>&1 || { tail -40 gpurun_out/gputests_r3_full.log; exit 1; }
tail -1 gpurun_out/gputests_r3_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3.log 2>&1 || { tail -20 gpurun_out/smoke_r3.log; exit 1; }
tail -1 gpurun_out/smoke_r3.log
out=gpurun_out/r3_full.jsonl; rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 600 "$@" 2>gpurun_out/r3f_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b bench python bench.py --gpus 1 --steps 20 --warmup 5 &&
b c2 python benchmarks/bench_configs.py --config 2 &&
b c2b python benchmarks/bench_configs.py --config 2 &&
b c4mv python benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate &&
b c4 python benchmarks/bench_configs.py --config 4 &&
b c2e2e python benchmarks/bench_configs.py --config 2e2e --steps 30 --warmup 3
echo rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/r3_full.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["tag"], round(d["ms_per_step"], 3), c.get("span_ms_median_rank0"))
PY
