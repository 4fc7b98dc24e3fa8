#!/bin/bash
# Config 2 (Holt-Winters grid fit) memory traffic: FETCH_SIZE and WRITE_SIZE
# (derived from the TCC->EA read/write requests) in separate passes, plus the
# busy clock, for the achieved-bandwidth check of hw2_fit_kernel against the
# measured HBM floor.  Summaries: gpurun_out/pmc_c2_<pass>.txt.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
declare -A PASS
PASS[fetch]="FETCH_SIZE"
PASS[write]="WRITE_SIZE"
PASS[busy]="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES"
for p in fetch write busy; do
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc ${PASS[$p]} -d "$R/gpurun_out/pmc_c2_$p" -o r -- \
    python3 "$R/benchmarks/bench_configs.py" --config 2 --steps 2 --warmup 1 > "$R/gpurun_out/pmc_c2_$p.log" 2>&1
  rc=$?
  echo "c2 $p rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_c2_$p" --kernel hw > "$R/gpurun_out/pmc_c2_$p.txt"
  rm -rf "$R/gpurun_out/pmc_c2_$p"
done
