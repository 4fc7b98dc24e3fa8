#!/bin/bash
# Round 6 first GPU pass: the RCCL start-up path of the brain (board +
# agreement on a real RCCL group, 2-rank board exchange), the headline bench
# and a fresh rocprofv3 kernel table of the headline tick.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
run() { name=$1; secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1; rc=$?; echo "$name rc=$rc"; return $rc; }
run r6_board_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_board_backend.py tests/test_board.py
run r6_bench 200 python -u bench.py &&
run r6_bench1250 200 python -u bench.py --services 1250 --steps 1000 --warmup 50 &&
cd /tmp && export TMPDIR=/tmp &&
run r6_hl_prof 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r6_hl_prof" -o hl -- python3 "$R/bench.py" --steps 100 --warmup 10
