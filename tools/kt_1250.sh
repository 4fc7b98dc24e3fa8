R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/kt_g" -o kt -- python3 "$R/bench.py" --services 1250 --steps 100 --warmup 10 > "$R/gpurun_out/kt_g.log" 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/kt_ng" -o kt -- python3 "$R/bench.py" --services 1250 --steps 100 --warmup 10 --no-graph > "$R/gpurun_out/kt_ng.log" 2>&1
