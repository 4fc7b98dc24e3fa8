"""bench.py contract (the driver's round-end benchmark): one JSON line with
the fields BASELINE.json names, on a small fleet so it runs in seconds."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--pipeline", "1"], ["--mode", "overlap"], ["--no-graph"]])
def test_bench_json_contract(extra):
    out = _bench("--services", "300", "--steps", "4", "--warmup", "2", *extra)
    assert REQUIRED <= set(out)
    assert out["metric"].startswith("metric windows scored/sec")
    assert out["n_gpus"] == 1 and out["steps"] == 4 and out["warmup"] == 2
    assert out["config"]["global_batch"] == 300 * 8 and out["config"]["seq_len"] == 10080
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert abs(out["value"] - 300 * 8 / (out["ms_per_step"] / 1e3)) / out["value"] < 1e-6
    # the fault injection of the synthetic fleet is visible in the verdicts
    assert 0 < out["services_flagged"] < 300


@pytest.mark.gpu
def test_bench_modes_agree_on_verdicts():
    flagged = {m: _bench("--services", "300", "--steps", "2", "--warmup", "1", "--mode", m)["services_flagged"]
               for m in ("front", "overlap", "serial")}
    assert len(set(flagged.values())) == 1, flagged


def _bench_cpu(*args, env=None):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--services", "64",
                        "--hist", "1440", "--steps", "2", "--warmup", "1", *args], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, env=env)
    return r


def test_bench_self_launches_ranks_on_cpu():
    """VERDICT r1 (next #2b/c): ``--gpus N`` without a launcher spawns N ranks,
    the verdict gather runs over gloo, and the JSON line reports ranks, backend
    and distinct devices (0 here: CPU ranks are never counted as GPUs)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r2 = _bench_cpu("--gpus", "2", env=env)
    assert r2.returncode == 0, r2.stderr[-2000:]
    o2 = json.loads([ln for ln in r2.stdout.splitlines() if ln.startswith("{")][0])
    assert len([ln for ln in r2.stdout.splitlines() if ln.startswith("{")]) == 1     # rank 0 only
    assert o2["n_ranks"] == 2 and o2["backend"] == "gloo" and o2["n_gpus"] == 0
    assert o2["config"]["parallelism"] == "dp2" and REQUIRED <= set(o2)
    r1 = _bench_cpu(env=env)
    o1 = json.loads([ln for ln in r1.stdout.splitlines() if ln.startswith("{")][0])
    assert o1["n_ranks"] == 1 and o1["backend"] == "none"
    # the sharded fleet verdict gathered on rank 0 equals the single-rank one
    assert o1["services_flagged"] == o2["services_flagged"] > 0


def test_bench_rejects_gpus_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = _bench_cpu("--gpus", "2", env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_extra_warmup_steps_count():
    """The untimed warm-up top-up: zero once the warm-up lasted long enough,
    otherwise enough steps to reach the minimum at the (MAX-reduced) step
    time, capped; a pure function of its inputs, so ranks agree."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.extra_warmup_steps(400.0, 0.5, 300.0) == 0
    assert bench.extra_warmup_steps(300.0, 0.5, 300.0) == 0
    n = bench.extra_warmup_steps(2.75, 0.55, 300.0)
    assert 2.75 + n * 0.55 >= 300.0 and 2.75 + (n - 2) * 0.55 < 300.0
    assert bench.extra_warmup_steps(0.0, 0.0, 300.0, cap=1000) == 1000
    assert bench.extra_warmup_steps(1.0, 0.08, 0.0) == 0
