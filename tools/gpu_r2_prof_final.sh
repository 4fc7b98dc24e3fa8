#!/bin/bash
# rocprofv3 kernel tables of the final bench defaults: full fleet and the
# 1,250-service shard publishing through a real RCCL group (graph publish)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pf_10k" -o pf -- python3 "$R/bench.py" --steps 100 --warmup 10 --warmup-min-ms 0 > "$R/gpurun_out/pf_10k.log" 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pf_1250" -o pf -- python3 "$R/bench.py" --services 1250 --steps 500 --warmup 10 --warmup-min-ms 0 --rccl-self > "$R/gpurun_out/pf_1250.log" 2>&1 &&
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/pf_10k" > "$R/gpurun_out/kernels_final_10k.txt" &&
python3 "$R/tools/prof_summary.py" "$R/gpurun_out/pf_1250" > "$R/gpurun_out/kernels_final_1250_rccl.txt"
echo rc=$?
head -12 "$R/gpurun_out/kernels_final_10k.txt"; head -12 "$R/gpurun_out/kernels_final_1250_rccl.txt"
