#!/bin/bash
# GPU-box session: GPU tests, the headline bench and (optionally) the e2e brain
# configs.  Usage on the box (through gpurun):
#   bash tools/gpu_check.sh [tests] [bench] [e2e] [configs]
# Each step runs under its own time limit; the first failing step ends the call.
# Output: gpurun_out/check_*.log, gpurun_out/check_e2e.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
steps="$*"
[ -z "$steps" ] && steps="tests bench"
rc=0
run() { name=$1; secs=$2; shift 2; echo "== $name" >&2
        timeout -k 10 "$secs" "$@" > "gpurun_out/check_$name.log" 2>&1; rc=$?
        echo "$name rc=$rc"; tail -3 "gpurun_out/check_$name.log"; return $rc; }
e2e() { tag=$1; shift; echo "== e2e $tag" >&2
        timeout -k 10 400 python -u benchmarks/bench_configs.py "$@" > "gpurun_out/check_e2e_$tag.log" 2>&1; rc=$?
        echo "e2e $tag rc=$rc"
        grep '^{' "gpurun_out/check_e2e_$tag.log" | sed "s/^{/{\"tag\": \"$tag\", /" >> gpurun_out/check_e2e.jsonl
        return $rc; }
for s in $steps; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $rc ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $rc ;;
    bench) run bench 300 python bench.py --steps 20 --warmup 5 || exit $rc ;;
    e2e) rm -f gpurun_out/check_e2e.jsonl
         e2e c3e2e --config 3e2e --steps 30 --warmup 3 &&
         e2e c2e2e --config 2e2e --steps 30 --warmup 3 &&
         e2e c4e2e --config 4e2e --steps 20 --warmup 3 || exit $rc ;;
    e2ehttp) e2e c3e2e_http --config 3e2e --source http --steps 70 --warmup 3 --prom-workers 8 &&
         e2e c3e2e_http60 --config 3e2e --source http --poll-seconds 60 --window 60 --steps 12 --warmup 2 --prom-workers 8 &&
         e2e c2e2e_http --config 2e2e --source http --steps 20 --warmup 3 --prom-workers 8 || exit $rc ;;
    configs) for c in 1 2 3 4 5; do run "c$c" 300 python benchmarks/bench_configs.py --config $c || exit $rc; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
