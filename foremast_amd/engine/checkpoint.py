"""Versioned checkpoint of engine state (SURVEY.md §5 "Checkpoint / resume").

Layout: ``<dir>/engine-<step>.safetensors`` holding every tensor (HPA
hysteresis state, per-job fitted bounds, LSTM weights) plus a JSON metadata
blob (job ids per row, config fingerprint, wall clock) in the safetensors
header; ``<dir>/LATEST`` names the newest file.  Writes are atomic
(tmp + rename), loads never execute anything from the file.
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

import torch
from safetensors.torch import load_file, save_file

FORMAT_VERSION = "foremast-amd/engine-checkpoint/1"


def save(dirpath: str, tensors: dict[str, torch.Tensor], meta: dict, step: int | None = None) -> Path:
    d = Path(dirpath)
    d.mkdir(parents=True, exist_ok=True)
    step = int(time.time()) if step is None else step
    path = d / f"engine-{step}.safetensors"
    tmp = d / f".engine-{step}.tmp"
    md = {"format": FORMAT_VERSION, "meta": json.dumps(meta), "saved_at": str(time.time())}
    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, str(tmp), metadata=md)
    os.replace(tmp, path)
    latest_tmp = d / ".LATEST.tmp"
    latest_tmp.write_text(path.name)
    os.replace(latest_tmp, d / "LATEST")
    return path


def load_latest(dirpath: str) -> tuple[dict[str, torch.Tensor], dict] | None:
    d = Path(dirpath)
    lf = d / "LATEST"
    if not lf.exists():
        return None
    path = d / lf.read_text().strip()
    if not path.exists():
        return None
    from safetensors import safe_open
    with safe_open(str(path), framework="pt") as f:
        md = f.metadata() or {}
    if md.get("format") != FORMAT_VERSION:
        raise ValueError(f"unsupported checkpoint format {md.get('format')!r}")
    return load_file(str(path)), json.loads(md.get("meta", "{}"))
