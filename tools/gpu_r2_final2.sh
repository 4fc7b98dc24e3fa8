#!/bin/bash
# Final validation of the bench defaults + eager RCCL publish host-overhead knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/final2.jsonl
rm -f $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_final2.log 2>&1 || { tail -20 gpurun_out/gputests_final2.log; exit 1; }
tail -1 gpurun_out/gputests_final2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke2.log 2>&1 || exit 1
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 200 "$@" 2>gpurun_out/f2_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b driver1 python bench.py --gpus 1 --steps 20 --warmup 5 &&
b driver2 python bench.py --gpus 1 --steps 20 --warmup 5 &&
b long python bench.py --steps 300 --warmup 30 &&
b sh_eager_aeh env TORCH_NCCL_ASYNC_ERROR_HANDLING=1 python bench.py --services 1250 --steps 2000 --warmup 100 --rccl-self --publish eager &&
b sh_eager_norec env TORCH_NCCL_ASYNC_ERROR_HANDLING=1 TORCH_NCCL_AVOID_RECORD_STREAMS=1 python bench.py --services 1250 --steps 2000 --warmup 100 --rccl-self --publish eager &&
b sh_graph_aeh env TORCH_NCCL_ASYNC_ERROR_HANDLING=1 python bench.py --services 1250 --steps 2000 --warmup 100 --rccl-self --publish graph
echo rc=$?
cat $out | python -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], round(d['ms_per_step'],4), d.get('warmup_extra_steps'), round(d['p50_decision_latency_ms'],4), d['config'].get('publish'))"
