mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gc_probe.py --config 2e2e --steps 20 --warmup 3 > gpurun_out/gc0.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/gc_probe.py --freeze --config 2e2e --steps 20 --warmup 3 > gpurun_out/gc1.log 2>&1 || exit 1
for f in gc0 gc1; do grep "^GC" gpurun_out/$f.log; grep '^{' gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['ms_per_step'],3), round(d['p50_decision_latency_ms'],3), d['config']['cycle_ms_max_rank0'])"; done
