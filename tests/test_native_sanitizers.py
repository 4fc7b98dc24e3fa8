"""The native host runtime under AddressSanitizer + UBSan and ThreadSanitizer
(truncated / mutated Prometheus documents, threaded count and pack)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_clean_under_asan_ubsan_tsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools/sanitize_host.sh"), str(tmp_path)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.count("clean") == 2
