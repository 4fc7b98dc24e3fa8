"""Localise scan-fit discrepancies: per candidate slot (even = .x, odd = .y
of a wave's pair) relative SSE error against the fp64 oracle, for the default
grid, a grid of duplicated pairs and a pair-swapped grid."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from foremast_amd.ops import smoothing as SM  # noqa: E402

rng = np.random.default_rng(0)
T, m, R = 10080, 1440, 4
t = np.arange(T)
x = (10 + np.sin(2 * np.pi * t / m)[None] + 0.0005 * t + rng.normal(0, 0.05, (R, T))).astype(np.float32)
g = SM.default_grid(2)
grids = {"default": g, "dup": np.repeat(g[::2], 2, axis=0)[:26], "swap": g[[i ^ 1 for i in range(26)]]}
for name, gr in grids.items():
    _, _, _, s0 = SM.ref_es_fit(x, 2, 10, m, gr)
    for meth in ("scan", "serial"):
        r = SM.es_fit(torch.from_numpy(x).cuda(), T, 2, 10, m, grid=gr, method=meth, half_season=False)
        rel = np.abs(r.sse.cpu().numpy() - s0) / s0
        print(name, meth, "even max", float(rel[:, 0::2].max()), "odd max", float(rel[:, 1::2].max()),
              "row0", np.array2string(rel[0], precision=1, max_line_width=400))
