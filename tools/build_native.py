#!/usr/bin/env python3
"""Build the native libraries in-tree.

* ``foremast_amd/_native/libforemast_hip.so`` — every ``csrc/kernels/*.hip``
  compiled by ``hipcc --offload-arch=gfx950`` (CDNA4 only, no other targets).
* ``foremast_amd/_native/libforemast_rt.so`` — host-side C++ runtime
  (``csrc/runtime/*.cpp``: Prometheus/Wavefront response parsing, the series
  packer) compiled with g++.

The libraries expose a plain C ABI consumed through ``ctypes`` by
``foremast_amd/ops/_lib.py`` and ``foremast_amd/engine/native_rt.py``; they do
not link against libtorch, so they build on a CPU-only box and load anywhere.

Usage: ``python tools/build_native.py [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OUT = ROOT / "foremast_amd" / "_native"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("FOREMAST_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CXX = shutil.which("g++") or "c++"

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
    "-munsafe-fp-atomics", f"-I{CSRC / 'include'}", "-Wno-unused-result",
]
CXX_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-pthread", f"-I{CSRC / 'include'}", "-Wall", "-Wno-unused-function"]


def _stale(obj: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"native build failed: {cmd[-1]}")


def build(force: bool = False, jobs: int = 4) -> list[Path]:
    OUT.mkdir(parents=True, exist_ok=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = sorted((CSRC / "include").glob("*.h"))
    built = []

    # --- HIP kernel library -------------------------------------------------
    hip_srcs = sorted((CSRC / "kernels").glob("*.hip"))
    objs, jobs_list = [], []
    for src in hip_srcs:
        obj = BUILD / (src.stem + ".hip.o")
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            jobs_list.append([HIPCC, *HIP_FLAGS, *_file_flags(src), "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    lib = OUT / "libforemast_hip.so"
    if objs and (force or jobs_list or _stale(lib, objs)):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib)])
    if objs:
        built.append(lib)

    # --- host runtime library ----------------------------------------------
    cpp_srcs = sorted((CSRC / "runtime").glob("*.cpp"))
    cobjs, cjobs = [], []
    for src in cpp_srcs:
        obj = BUILD / (src.stem + ".o")
        cobjs.append(obj)
        if force or _stale(obj, [src, *headers]):
            cjobs.append([CXX, *CXX_FLAGS, "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, cjobs))
    rlib = OUT / "libforemast_rt.so"
    if cobjs and (force or cjobs or _stale(rlib, cobjs)):
        _run([CXX, "-shared", "-pthread", *map(str, cobjs), "-o", str(rlib)])
    if cobjs:
        built.append(rlib)
    return built


def _file_flags(src: Path) -> list[str]:
    """Per-file hipcc flags: a ``// fm-hipcc-flags: ...`` line in the first 40 lines."""
    with open(src) as f:
        for _, line in zip(range(40), f):
            if line.startswith("// fm-hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def build_variant(name: str, flags: list[str], stems: list[str], jobs: int = 4) -> Path:
    """An A/B build of the HIP library: the default objects with ``stems``'
    sources recompiled under ``flags`` in place of their own per-file flags
    -> ``_native/variants/libforemast_hip_<name>.so`` (select it with
    ``FOREMAST_HIP_LIB``)."""
    build(False, jobs)
    vdir = BUILD / f"variant_{name}"
    vdir.mkdir(parents=True, exist_ok=True)
    objs, cmds = [], []
    for src in sorted((CSRC / "kernels").glob("*.hip")):
        if src.stem in stems:
            obj = vdir / (src.stem + ".hip.o")
            cmds.append([HIPCC, *HIP_FLAGS, *flags, "-c", str(src), "-o", str(obj)])
        else:
            obj = BUILD / (src.stem + ".hip.o")
        objs.append(obj)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, cmds))
    out = OUT / "variants" / f"libforemast_hip_{name}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out)])
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--variant", action="append", default=[],
                    help="NAME:FILE[,FILE]:FLAG[,FLAG] -- an A/B build of the HIP library")
    a = ap.parse_args()
    for p in build(a.force, a.j):
        print(p.relative_to(ROOT))
    for v in a.variant:
        name, stems, flags = v.split(":", 2)
        print(build_variant(name, flags.split(",") if flags else [], stems.split(","), a.j).relative_to(ROOT))


if __name__ == "__main__":
    main()
