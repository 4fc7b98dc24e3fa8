"""The kernels as torch operators (ops/library.py): schema + fake-tensor
checks with torch.library.opcheck (CPU reference implementations), results
equal to the Python entry points, and on the GPU the op names in a
torch.profiler trace."""
import numpy as np
import pytest
import torch

from foremast_amd.ops import canary as C
from foremast_amd.ops import library as L  # noqa: F401  (registers torch.ops.foremast.*)
from foremast_amd.ops import misc as MI
from foremast_amd.ops import smoothing as SM

ops = torch.ops.foremast
CHECKS = ("test_schema", "test_faketensor")


def _fleet(S=6, M=4, T=600, seed=0):
    h, b, c = C.synth_fleet(S, M, T, 3, 10, 0, seed=seed, fault_rate=0.3)
    return h.contiguous(), b.contiguous(), c.contiguous()


def test_ops_registered():
    for name in L.OPS:
        assert hasattr(ops, name), name


def test_opcheck_pairwise_and_decide():
    h, b, c = _fleet()
    torch.library.opcheck(ops.pairwise_tests, (c, b, "ALL", 0.05, 20, 20, 5), test_utils=CHECKS)
    pv, st, d = ops.pairwise_tests(c, b, "ALL", 0.05, 20, 20, 5)
    pv0, _, d0 = C.pairwise_tests(c, b, C.PairwiseConfig("ALL"))
    torch.testing.assert_close(pv, pv0, equal_nan=True)
    assert torch.equal(d, d0)
    M = 4
    thr = torch.full((M,), 2.0)
    bound = torch.full((M,), 3, dtype=torch.int32)
    minlb = torch.zeros(M)
    args = (h, c, 600, M, thr, bound, minlb, d, 0.8, 10)
    torch.library.opcheck(ops.stats_decide, args, test_utils=CHECKS)
    stats, flags, count, score, valid = ops.stats_decide(*args)
    torch.library.opcheck(ops.service_reduce, (count, score, valid, M), test_utils=CHECKS)
    assert ops.service_reduce(count, score, valid, M).shape == (6, 4)


def test_opcheck_models():
    x = torch.from_numpy(np.sin(np.arange(400)[None, :] * 2 * np.pi / 24).repeat(3, 0).astype(np.float32) + 5)
    grid = torch.from_numpy(SM.default_grid(2))
    torch.library.opcheck(ops.es_fit, (x, 400, 2, 5, 24, grid), test_utils=CHECKS)
    fc, sig, best, sse = ops.es_fit(x, 400, 2, 5, 24, grid)
    assert fc.shape == (3, 5) and sse.shape == (3, grid.shape[0])
    xf = torch.from_numpy(np.tile(np.sin(np.arange(2016) * 2 * np.pi / 288)[None, :], (2, 1)).astype(np.float32))
    torch.library.opcheck(ops.fft_seasonal, (xf, 2016, 30.0, 1008.0), test_utils=CHECKS)
    assert ops.fft_seasonal(xf, 2016, 30.0, 1008.0)[1].tolist() == [288.0, 288.0]
    g = MI.CallGraph.from_edges(4, [0, 0, 1], [1, 2, 3], [0.5, 0.5, 1.0])
    a = torch.tensor([0, 0, 0, 1.0])
    args = (torch.from_numpy(g.rowptr), torch.from_numpy(g.col), torch.from_numpy(g.weight), a, 2)
    torch.library.opcheck(ops.downstream_impact, args, test_utils=CHECKS)
    assert ops.downstream_impact(*args).tolist() == [0.5, 1.0, 0.0, 0.0]
    xr = torch.randn(3, 200)
    torch.library.opcheck(ops.rolling_stats, (xr, 200, 20, 1), test_utils=CHECKS)


@pytest.mark.gpu
def test_gpu_ops_in_profiler(cuda):
    from torch.profiler import ProfilerActivity, profile
    h, b, c = _fleet()
    hg, bg, cg = h.to(cuda), b.to(cuda), c.to(cuda)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        pv, st, d = ops.pairwise_tests(cg, bg, "ALL", 0.05, 20, 20, 5)
        torch.cuda.synchronize()
    names = {e.key for e in prof.key_averages()}
    assert "foremast::pairwise_tests" in names
    pv0, _, _ = C.pairwise_tests(c, b, C.PairwiseConfig("ALL"))
    np.testing.assert_allclose(np.nan_to_num(pv.cpu().numpy()), np.nan_to_num(pv0.numpy()), rtol=2e-4, atol=2e-6)
