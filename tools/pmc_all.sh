#!/bin/bash
# Hardware-counter passes (kernel-trace + PMC only) for the headline tick and
# configs 2 / 4 (or the targets given as arguments).  Results: gpurun_out/pmc_<target>_<pass>/; summarise with
# tools/pmc_summary.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
# one derived memory counter per pass: FETCH_SIZE + WRITE_SIZE together exceed
# what the hardware can collect in one pass (rocprofiler error 38)
declare -A PASS
PASS[fetch]="FETCH_SIZE"
PASS[write]="WRITE_SIZE"
PASS[inst]="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES"
PASS[busy]="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"
PASS[lds]="SQ_LDS_BANK_CONFLICT"
for target in ${@:-bench c2 c4}; do
  case $target in
    bench) cmd=("$R/bench.py" --steps 3 --warmup 1) ;;
    c2) cmd=("$R/benchmarks/bench_configs.py" --config 2 --steps 1 --warmup 1) ;;
    c4) cmd=("$R/benchmarks/bench_configs.py" --config 4 --steps 1 --warmup 1) ;;
  esac
  for p in inst busy lds fetch write; do
    timeout -k 10 150 rocprofv3 --kernel-trace --pmc ${PASS[$p]} -d "$R/gpurun_out/pmc_${target}_$p" -o r -- \
      python3 "${cmd[@]}" > "$R/gpurun_out/pmc_${target}_$p.log" 2>&1
    rc=$?
    echo "$target $p rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
    # keep only the per-kernel summary (the databases exceed what gpurun copies back)
    python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_${target}_$p" > "$R/gpurun_out/pmc_${target}_$p.txt"
    rm -rf "$R/gpurun_out/pmc_${target}_$p"
  done
done
