"""A/B timing of fm_es_fit between the in-tree library and other builds
(paths in argv[1:]) on the config-2 shape; prints one JSON line."""
import ctypes
import json
import sys

import torch

from foremast_amd.ops import canary as C
from foremast_amd.ops import smoothing as SM
from foremast_amd.ops._lib import LIB, ptr, stream_of

R, T, m, H = 40000, 10080, 1440, 10
dev = torch.device("cuda")
hist, _, _ = C.synth_fleet(R // 4, 4, T, 1, 10, 0, device=dev)
grid = torch.from_numpy(SM.default_grid(2)).to(dev)
G = grid.shape[0]
P = R * G
season = torch.empty((m, P), device=dev)
sse = torch.empty((R, G), device=dev)
state = torch.empty((P, 3), device=dev)
nobs = torch.empty((P,), dtype=torch.int32, device=dev)
fc = torch.empty((R, H), device=dev)
sig = torch.empty((R,), device=dev)
best = torch.empty((R,), dtype=torch.int32, device=dev)
args = [ptr(hist), hist.stride(0), T, R, ptr(grid), G, m, 2, ptr(season), ptr(sse), ptr(state), ptr(nobs), H,
        ptr(fc), ptr(sig), ptr(best), stream_of(hist)]
args_tree = args[:-1] + [0, args[-1]]      # in-tree API has keep_season before the stream
def load(path):
    """Libraries named *old* have the pre-keep_season signature."""
    lib = ctypes.CDLL(path)
    legacy = "old" in path.rsplit("/", 1)[-1]
    lib.fm_es_fit.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                              ctypes.c_int, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] + \
                             [ctypes.c_void_p] * 3 + ([] if legacy else [ctypes.c_int]) + [ctypes.c_void_p]
    a = args if legacy else args_tree
    return lambda: lib.fm_es_fit(*a)


runs = [("tree", lambda: LIB.call("fm_es_fit", *args_tree))] + [(p.rsplit("/", 1)[-1], load(p)) for p in sys.argv[1:]]
out = {}
for rep in range(2):
    for name, fn in runs:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[f"{name}#{rep}"] = round(e0.elapsed_time(e1) / 5, 3)
print(json.dumps(out))
