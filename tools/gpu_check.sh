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
    tests) run tests 900 python -u -m pytest tests -m gpu --maxfail 8 -v --timeout 120 --timeout-method thread || exit $rc ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $rc ;;
    bench) run bench 300 python bench.py --steps 20 --warmup 5 || exit $rc ;;
    e2e) rm -f gpurun_out/check_e2e.jsonl
         e2e c3e2e --config 3e2e --steps 30 --warmup 3 &&
         e2e c2e2e --config 2e2e --steps 30 --warmup 3 &&
         e2e c4e2e --config 4e2e --steps 20 --warmup 3 || exit $rc ;;
    e2ehttp) e2e c3e2e_http --config 3e2e --source http --steps 70 --warmup 3 --prom-workers 8 &&
         e2e c3e2e_http60 --config 3e2e --source http --poll-seconds 60 --window 60 --steps 12 --warmup 2 --prom-workers 8 &&
         e2e c2e2e_http --config 2e2e --source http --steps 20 --warmup 3 --prom-workers 8 || exit $rc ;;
    peerprobe) run peer_probe 150 python -u tools/peer_probe.py || exit $rc ;;
    lstm) V=$R/foremast_amd/_native/variants
          run lstm_tests 400 python -u -m pytest tests/test_model_ops.py -m gpu -k "lstm" -v --timeout 120 \
              --timeout-method thread || exit $rc
          run lstm_ab 200 python -u tools/lstm_ab.py || exit $rc
          # (A/B builds: tools/build_native.py --variant NAME:lstm:FLAGS, then
          #  env FOREMAST_HIP_LIB=$V/libforemast_hip_NAME.so python -u tools/lstm_ab.py)
          run config4 300 python -u benchmarks/bench_configs.py --config 4 || exit $rc
          run config4_stack 300 python -u benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate || exit $rc ;;
    lstm5) run lstm_tests 400 python -u -m pytest tests/test_model_ops.py -m gpu -k "lstm" -v --timeout 120 \
              --timeout-method thread || exit $rc
          run lstm_ab 200 python -u tools/lstm_ab.py || exit $rc
          run config4 300 python -u benchmarks/bench_configs.py --config 4 || exit $rc
          run config4_w30 300 python -u benchmarks/bench_configs.py --config 4 --steps 30 --warmup 30 || exit $rc ;;
    pmclstm) run pmclstm 420 bash tools/pmc_lstm.sh || exit $rc ;;
    r5tests) run r5tests 600 python -u -m pytest tests/test_fastpath_models.py tests/test_canary_ops.py tests/test_warm_restart.py \
                 tests/test_model_ops.py tests/test_fastpath.py -m gpu -x -v --timeout 120 --timeout-method thread \
                 || exit $rc ;;
    peer) run peer_test 300 python -u -m pytest tests/test_peer.py tests/test_board.py -x -v -s --timeout 200 \
              --timeout-method thread || exit $rc
          run peer_bench 240 env FOREMAST_DEVICE_INDEX=0 FOREMAST_DIST_BACKEND=gloo python bench.py --gpus 2 \
              --services 2500 --publish peer --steps 300 --warmup 20 || exit $rc ;;
    mixed) e2e c_mixed --config mixed --steps 20 --warmup 3 &&
         e2e c_mixed_canary --config mixed --mixed-class 0 --steps 20 --warmup 3 &&
         e2e c_mixed_cont --config mixed --mixed-class 1 --steps 20 --warmup 3 &&
         e2e c_mixed_hpa --config mixed --mixed-class 2 --steps 20 --warmup 3 &&
         e2e c2e2e --config 2e2e --steps 20 --warmup 3 &&
         e2e c4e2e --config 4e2e --steps 20 --warmup 3 || exit $rc ;;
    shard) run shard1250 200 python bench.py --services 1250 --steps 400 --warmup 20 || exit $rc
           run shard1250_prof 300 bash -c "cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_shard \
               -o shard -- python3 $R/bench.py --services 1250 --steps 200 --warmup 20" || exit $rc ;;
    httpbench) run httpbench 600 python -u tools/http_fetch_bench.py --services 10000 --cycles 8 \
               --out gpurun_out/http_fetch_bench.jsonl || exit $rc ;;
    hostprof) for c in 2e2e 4e2e mixed; do
           FOREMAST_PROFILE_CYCLES=gpurun_out/hostprof_$c.prof timeout -k 10 400 python -u benchmarks/bench_configs.py \
               --config $c --steps 12 --warmup 3 > gpurun_out/check_hostprof_$c.log 2>&1; rc=$?
           echo "hostprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
           python -c "import pstats,sys; p=pstats.Stats('gpurun_out/hostprof_$c.prof', stream=sys.stdout); \
               p.sort_stats('tottime').print_stats(70); p.sort_stats('cumtime').print_stats(70)" \
               > gpurun_out/hostprof_$c.txt || exit 1
         done ;;
    hostprof4) for c in 4e2e 2e2e; do
           FOREMAST_PROFILE_CYCLES=gpurun_out/hostprof_$c.prof timeout -k 10 400 python -u benchmarks/bench_configs.py \
               --config $c --steps 12 --warmup 3 > gpurun_out/check_hostprof_$c.log 2>&1; rc=$?
           echo "hostprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
           python -c "import pstats,sys; p=pstats.Stats('gpurun_out/hostprof_$c.prof', stream=sys.stdout); \
               p.sort_stats('tottime').print_stats(70); p.sort_stats('cumtime').print_stats(90)" \
               > gpurun_out/hostprof_$c.txt || exit 1
         done ;;
    hostprofmixed) FOREMAST_PROFILE_CYCLES=gpurun_out/hostprof_mixed.prof timeout -k 10 500 python -u \
               benchmarks/bench_configs.py --config mixed --steps 10 --warmup 3 > gpurun_out/check_hostprof_mixed.log 2>&1; rc=$?
           echo "hostprof mixed rc=$rc"; [ $rc -eq 0 ] || exit $rc
           python -c "import pstats,sys; p=pstats.Stats('gpurun_out/hostprof_mixed.prof', stream=sys.stdout); \
               p.sort_stats('tottime').print_stats(60); p.sort_stats('cumtime').print_stats(100)" \
               > gpurun_out/hostprof_mixed.txt || exit 1 ;;
    hostprof60) FOREMAST_PROFILE_CYCLES=gpurun_out/hostprof_3e2e_http60.prof timeout -k 10 500 python -u \
               benchmarks/bench_configs.py --config 3e2e --source http --poll-seconds 60 --window 60 --steps 8 \
               --warmup 2 --prom-workers 8 > gpurun_out/check_hostprof_3e2e_http60.log 2>&1; rc=$?
           echo "hostprof60 rc=$rc"; [ $rc -eq 0 ] || exit $rc
           python -c "import pstats,sys; p=pstats.Stats('gpurun_out/hostprof_3e2e_http60.prof', stream=sys.stdout); \
               p.sort_stats('tottime').print_stats(70); p.sort_stats('cumtime').print_stats(90)" \
               > gpurun_out/hostprof_3e2e_http60.txt || exit 1 ;;
    hostprofhttp) FOREMAST_PROFILE_CYCLES=gpurun_out/hostprof_2e2e_http.prof timeout -k 10 500 python -u \
               benchmarks/bench_configs.py --config 2e2e --source http --steps 8 --warmup 3 --prom-workers 8 \
               > gpurun_out/check_hostprof_2e2e_http.log 2>&1; rc=$?
           echo "hostprof 2e2e http rc=$rc"; [ $rc -eq 0 ] || exit $rc
           python -c "import pstats,sys; p=pstats.Stats('gpurun_out/hostprof_2e2e_http.prof', stream=sys.stdout); \
               p.sort_stats('tottime').print_stats(50); p.sort_stats('cumtime').print_stats(90)" \
               > gpurun_out/hostprof_2e2e_http.txt || exit 1 ;;
    restart) e2e c3e2e_restart --config 3e2e --steps 5 --warmup 2 --restart &&
         e2e c2e2e_restart --config 2e2e --steps 5 --warmup 2 --restart || exit $rc ;;
    savediag) FOREMAST_SAVE_DIAG=1 e2e c2e2e_savediag --config 2e2e --steps 5 --warmup 2 --restart || exit $rc ;;
    scanprobe) run scanprobe 200 python -u tools/hw_scan_probe.py || exit $rc
          run scanab 300 python -u tools/hw_scan_ab.py --rows 40000 --m 1440 288 720 --reps 5 || exit $rc
          run scanab_1pass 300 env FOREMAST_HW_SCAN_PASSES=1 python -u tools/hw_scan_ab.py --rows 40000 --m 1440 \
              --reps 5 --methods scan || exit $rc ;;
    pmcscan) run pmcscan 420 bash tools/pmc_hwscan.sh || exit $rc ;;
    configs) for c in 1 2 3 4 5; do run "c$c" 300 python benchmarks/bench_configs.py --config $c || exit $rc; done ;;
    steady) e2e c2e2e --config 2e2e --steps 20 --warmup 3 &&
            e2e c4e2e --config 4e2e --steps 20 --warmup 3 || exit $rc ;;
    tprof) for c in 2e2e 4e2e; do
             FOREMAST_TORCH_PROFILE=gpurun_out/tprof_$c.txt timeout -k 10 400 python -u benchmarks/bench_configs.py \
                 --config $c --steps 8 --warmup 3 > gpurun_out/check_tprof_$c.log 2>&1; rc=$?
             echo "tprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
           done ;;
    prof2e2e) cd /tmp && export TMPDIR=/tmp
          timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$R/gpurun_out/prof_c2e2e" -o c2e2e -- \
              python3 "$R/benchmarks/bench_configs.py" --config 2e2e --steps 10 --warmup 2 \
              > "$R/gpurun_out/check_prof_c2e2e.log" 2>&1; rc=$?
          echo "prof_c2e2e rc=$rc"; cd "$R"; [ $rc -eq 0 ] || exit $rc ;;
    profc4) cd /tmp && export TMPDIR=/tmp
          timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c4" -o c4 -- \
              python3 "$R/benchmarks/bench_configs.py" --config 4 --steps 10 --warmup 3 \
              > "$R/gpurun_out/check_prof_c4.log" 2>&1; rc=$?
          echo "prof_c4 rc=$rc"; cd "$R"; [ $rc -eq 0 ] || exit $rc ;;
    prof60) cd /tmp && export TMPDIR=/tmp
          timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3_60" -o c3 -- \
              python3 "$R/benchmarks/bench_configs.py" --config 3e2e --source http --poll-seconds 60 --window 60 \
              --steps 6 --warmup 2 --prom-workers 8 > "$R/gpurun_out/check_prof_c3_60.log" 2>&1; rc=$?
          echo "prof_c3_60 rc=$rc"; cd "$R"; [ $rc -eq 0 ] || exit $rc ;;
    prof) cd /tmp && export TMPDIR=/tmp
          timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_headline" -o headline -- \
              python3 "$R/bench.py" --steps 50 --warmup 10 > "$R/gpurun_out/check_prof_headline.log" 2>&1; rc=$?
          echo "prof_headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
          timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2e2e" -o c2e2e -- \
              python3 "$R/benchmarks/bench_configs.py" --config 2e2e --steps 10 --warmup 2 \
              > "$R/gpurun_out/check_prof_c2e2e.log" 2>&1; rc=$?
          echo "prof_c2e2e rc=$rc"; cd "$R"; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
