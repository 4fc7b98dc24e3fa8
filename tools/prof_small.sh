#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_s1250" -o s -- python3 "$R/bench.py" --services 1250 --steps 100 --warmup 10 > "$R/gpurun_out/prof_s1250.log" 2>&1
echo rc=$?
