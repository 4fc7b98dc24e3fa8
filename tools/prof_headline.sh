#!/bin/bash
# Headline evidence on one GPU: bench JSON lines (10k fleet, 1,250-service
# shard), rocprofv3 kernel stats, and kernel/copy timelines of the last ticks.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
run() { name=$1; secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1; rc=$?; echo "$name rc=$rc"; return $rc; }
run hl_bench 120 python3 "$R/bench.py" &&
run hl_bench1250 120 python3 "$R/bench.py" --services 1250 --steps 1000 --warmup 50 &&
cd /tmp && export TMPDIR=/tmp &&
run hl_prof 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/hl_prof" -o hl -- python3 "$R/bench.py" --steps 100 --warmup 10 &&
run hl_tl10k 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/hl_tl10k" -o tl -- python3 "$R/bench.py" --steps 50 --warmup 10 &&
run hl_tl1250 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/hl_tl1250" -o tl -- python3 "$R/bench.py" --services 1250 --steps 200 --warmup 10
