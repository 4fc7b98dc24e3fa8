"""docs/INVENTORY.md maps SURVEY.md §2 line by line to code and tests; this
keeps every test it cites and every module path it names real."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(ROOT, "docs", "INVENTORY.md")


def _text() -> str:
    with open(DOC, encoding="utf-8") as f:
        return f.read()


def test_cited_tests_exist():
    text = _text()
    missing = []
    # `tests/test_x.py::test_y` opens a run of `::test_z` citations of the same file
    for cell in re.findall(r"`[^`]+`(?:, `[^`]+`)*", text):
        current = None
        for ref in re.findall(r"`([^`]+)`", cell):
            m = re.match(r"(tests/test_\w+\.py)(?:::(test_\w+))?", ref)
            if m:
                current = m.group(1)
                name = m.group(2)
            elif ref.startswith("::test_") and current:
                name = ref[2:].rstrip("*")
            else:
                continue
            path = os.path.join(ROOT, current)
            if not os.path.exists(path):
                missing.append(current)
                continue
            if name:
                src = open(path, encoding="utf-8").read()
                pat = name.rstrip("_") if name.endswith("_") else name
                if not re.search(r"def " + re.escape(pat), src):
                    missing.append(f"{current}::{name}")
    assert not missing, missing


def test_cited_modules_exist():
    text = _text()
    missing = []
    for ref in set(re.findall(r"`((?:foremast_amd/)?(?:api|controller|engine|models|ops|parallel|service|"
                              r"trigger|dashboard|emitter|demo|deploy|utils)/\w+\.py)", text)):
        path = ref if ref.startswith("foremast_amd/") else "foremast_amd/" + ref
        if not os.path.exists(os.path.join(ROOT, path)):
            missing.append(ref)
    for ref in set(re.findall(r"`(csrc/kernels/\w+\.hip|tools/\w+\.(?:py|sh))", text)):
        if not os.path.exists(os.path.join(ROOT, ref)):
            missing.append(ref)
    assert not missing, missing
