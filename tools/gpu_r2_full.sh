#!/bin/bash
# Full GPU validation of the tree: pytest -m gpu, smoke, headline bench, config sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputests_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_full.jsonl 2>&1 || exit 1
tail -1 gpurun_out/bench_full.jsonl
