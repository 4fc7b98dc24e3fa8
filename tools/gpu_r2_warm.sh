#!/bin/bash
# Driver-shaped runs with the time-based warm-up (--warmup-min-ms, default 300)
# and the graph-captured publish (--publish graph) vs eager, at the full fleet
# and at the 1,250-service shard with a real RCCL group (--rccl-self).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/warm_probe.jsonl
rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 200 python bench.py "$@" 2>gpurun_out/warm_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b short_eager --gpus 1 --steps 20 --warmup 5 &&
b short_graph --gpus 1 --steps 20 --warmup 5 --publish graph &&
b long_eager --steps 300 --warmup 30 &&
b long_graph --steps 300 --warmup 30 --publish graph &&
b shard_short_eager --services 1250 --steps 20 --warmup 5 --rccl-self &&
b shard_short_graph --services 1250 --steps 20 --warmup 5 --rccl-self --publish graph &&
b shard_long_eager --services 1250 --steps 2000 --warmup 100 --rccl-self &&
b shard_long_graph --services 1250 --steps 2000 --warmup 100 --rccl-self --publish graph &&
b shard_long_graph3 --services 1250 --steps 2000 --warmup 100 --rccl-self --publish graph --pipeline 3 &&
b shard_short_norccl --services 1250 --steps 20 --warmup 5
echo rc=$?
cat $out | python -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['ms_per_step'],4), d.get('warmup_extra_steps'), round(d['p50_decision_latency_ms'],4))"
