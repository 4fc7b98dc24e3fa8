"""Which candidate pairs the half-wave scan gets wrong: per-candidate relative
SSE error against the fp64 oracle (even pair index = half 0 of a wave)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from foremast_amd.ops import smoothing as SM  # noqa: E402

rng = np.random.default_rng(0)
T, m, R = 10080, 288, 3
t = np.arange(T)
x = (10 + np.sin(2 * np.pi * t / m)[None] + rng.normal(0, 0.05, (R, T))).astype(np.float32)
g = SM.default_grid(2)
_, _, _, s0 = SM.ref_es_fit(x, 2, 10, m, g)
r = SM.es_fit(torch.from_numpy(x).cuda(), T, 2, 10, m, method="scan")
rel = np.abs(r.sse.cpu().numpy() - s0) / s0
print(os.environ.get("FOREMAST_HW_SCAN_LPP"), np.array2string(rel[0], precision=1, max_line_width=300))
print("state l", r.model is None)
