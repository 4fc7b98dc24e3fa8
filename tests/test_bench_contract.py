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
