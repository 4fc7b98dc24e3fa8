"""GPU-vs-CPU component check of the least-squares projection kernel."""
import numpy as np
import torch

from foremast_amd.ops import lsq as LQ

T, H, R = 10080, 50, 64
rng = np.random.default_rng(9)
t = np.arange(T)
x = (10 + np.sin(2 * np.pi * t / 1440)[None] * rng.uniform(.5, 2, (R, 1)) + 0.0005 * t
     + rng.normal(0, .05, (R, T))).astype(np.float32)
ut, fmap, vs, rank = LQ._basis(T, H, 60.0)
XT = torch.from_numpy(ut)
Zc, yyc, shc, nvc = LQ.lsq_project(torch.from_numpy(x), T, XT)
Zg, yyg, shg, nvg = LQ.lsq_project(torch.from_numpy(x).cuda(), T, XT.cuda())
Zg, yyg, shg, nvg = (a.cpu() for a in (Zg, yyg, shg, nvg))
print("shift max diff", (shg - shc).abs().max().item())
print("nvalid", nvg[:4].tolist(), nvc[:4].tolist())
print("yy rel diff", ((yyg - yyc) / yyc).abs().max().item(), yyg[:3].tolist(), yyc[:3].tolist())
d = (Zg - Zc).abs()
print("Z max abs diff", d.max().item(), "argmax", divmod(int(d.argmax()), 32))
print("Z row0", Zg[0, :6].tolist(), Zc[0, :6].tolist())
print("sse gpu", (yyg.double() - (Zg.double() ** 2).sum(1))[:4].tolist())
print("sse cpu", (yyc.double() - (Zc.double() ** 2).sum(1))[:4].tolist())
