#!/bin/bash
# VALU / SALU / LDS instruction counts of the scan fit by phase (PMC): the
# kernel's FOREMAST_HW_SCAN_DEBUG modes stop after the row setup (1) or skip
# the season laps (2); 0 is the full fit.  Config-2 shape, kernel-trace +
# counters only.  Output: gpurun_out/pmc_hwscan_phases.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
set -e
A="--rows 40000 --m ${PMC_M:-1440} --reps 2 --methods scan"
: > "$R/gpurun_out/pmc_hwscan_phases.txt"
for mode in 0 1 2; do
  FOREMAST_HW_SCAN_DEBUG=$mode timeout -k 10 120 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$R/gpurun_out/pmc_phase_$mode" -o p -- python3 "$R/tools/hw_scan_ab.py" $A > "$R/gpurun_out/pmc_phase_$mode.log" 2>&1
  echo "== FOREMAST_HW_SCAN_DEBUG=$mode" >> "$R/gpurun_out/pmc_hwscan_phases.txt"
  (cd "$R" && python3 tools/pmc_summary.py "gpurun_out/pmc_phase_$mode" --kernel fit_kernel) >> "$R/gpurun_out/pmc_hwscan_phases.txt"
  rm -rf "$R/gpurun_out/pmc_phase_$mode"
done
echo done
