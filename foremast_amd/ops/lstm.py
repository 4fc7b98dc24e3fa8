"""K6 LSTM forward on bf16 MFMA (csrc/kernels/lstm.hip).

Weights use torch.nn.LSTM conventions (gate order i, f, g, o; W_ih [4H, I],
W_hh [4H, H], b = b_ih + b_hh).  ``pack_lstm`` swizzles them into the
per-wave register-fragment layout the kernel loads with one 16-B load per
fragment, folding the input projection and bias into an extra K step."""
from __future__ import annotations

import numpy as np
import torch

from ._lib import LIB, check, ptr, require_native, stream_of

SUPPORTED_H = (32, 64, 128)              # register-resident single-layer kernel (lstm.hip)
STACK_H = (32, 64, 128, 256)             # streamed-weight 1-2 layer kernel (lstm_stack.hip)
STACK_TILING = {256: (4, 2), 128: (2, 2), 64: (2, 2), 32: (2, 2)}   # H -> (row tiles / wave, column tiles)
# two layers at H = 256: the row-streamed BT = 64 kernel (one row tile at a
# time, its cells beside the next tile's MFMAs, every weight fragment feeding
# 64 sequences; 4.6 ms at 10k x 240 and 29.6 at 80k, vs 6.8 / 35.9 for the
# layer-pipelined BT = 32 kernel and 8.2 / 42.0 for 4 x 2,
# profiles/lstm_stack_rs_r3.jsonl); weights packed with the same RT = 4
STACK_TILING_2L = {256: (4, 202)}
STACK_TILING_ALT = {256: ((4, 2), (4, 1), (2, 2), (2, 1),            # instantiated alternatives (lstm_stack.hip);
                          (4, 201), (2, 201), (4, 202),              # nct 201: layer-pipelined, 2 layers, 1 tile; 202: row-streamed, 2 tiles;
                          (4, 211), (4, 212), (4, 213), (4, 214),    # 211-213: its ablations (timing only, wrong h);
                          (8, 216))}                                 # 214: A one k-step ahead (correct h);
                                                                     # 216: 16x16 tiles, 48 sequences (pack_t16):
                                                                     # 209 workgroups instead of 157 at 10k, but
                                                                     # 4.65 vs 4.06 ms -- every row tile re-reads B
                                                                     # from LDS (profiles/lstm_stack_t16_ab_r6.jsonl)


def stack_tiling(H: int, layers: int = 1) -> tuple[int, int]:
    """(row tiles per wave, column tiles per workgroup) of the stacked kernel
    at hidden size H; ``FM_LSTM_STACK_TILING=RT:NCT`` overrides it at H = 256
    (A/B of fill vs streamed-weight reuse; the packed weights depend on RT,
    so pack and run under the same setting).  A ``p`` suffix (``4:1p``)
    selects the layer-pipelined two-layer kernel (nct 201)."""
    import os
    env = os.environ.get("FM_LSTM_STACK_TILING")
    if env and H in STACK_TILING_ALT:
        kind = env[-1] if env[-1] == "p" else ""
        rt, nct = (int(v) for v in env.rstrip("p").split(":"))
        nct += 200 if kind else 0
        check((rt, nct) in STACK_TILING_ALT[H], f"FM_LSTM_STACK_TILING {env} not instantiated for H={H}")
        if nct > 200 and layers != 2:
            return rt, 2 if rt == 4 else 1                  # the pipelined kernels are two-layer only
        return rt, nct
    if layers == 2 and H in STACK_TILING_2L:
        return STACK_TILING_2L[H]
    return STACK_TILING[H]


def _bf16_bits(a: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return u.astype(np.uint16)


def bf16_round(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


LOG2E = 1.4426950408889634
GATE_SCALES = (-LOG2E, -LOG2E, -2.0 * LOG2E, -LOG2E)   # i, f, g, o


def gate_scales(H: int) -> np.ndarray:
    """[4H] per-gate-row scale the packed weights carry (csrc/include/fm_lstm_cell.h):
    exp2 of a scaled pre-activation is e^{-x} (i, f, o) or e^{-2x} (g)."""
    return np.repeat(np.asarray(GATE_SCALES, np.float64), H).astype(np.float32)


def _scaled_rows(a: np.ndarray, H: int) -> np.ndarray:
    """Gate rows (first axis 4H) times their scale, in fp32."""
    s = gate_scales(H)
    return (a.astype(np.float32) * (s if a.ndim == 1 else s[:, None])).astype(np.float32)


def pack_lstm(w_ih: torch.Tensor, w_hh: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """-> uint8 tensor [H/16, 2, KS, 64, 16 bytes] (bf16 fragments of the
    gate-scaled weights, :func:`gate_scales`)."""
    w_ih = w_ih.detach().float().cpu().numpy()
    w_hh = w_hh.detach().float().cpu().numpy()
    b = bias.detach().float().cpu().numpy()
    H4, I = w_ih.shape
    H = H4 // 4
    w_ih, w_hh, b = _scaled_rows(w_ih, H), _scaled_rows(w_hh, H), _scaled_rows(b, H)
    check(H in SUPPORTED_H, f"hidden size must be one of {SUPPORTED_H}")
    check(I <= 15, "input features must be <= 15 (folded into one K step with the bias)")
    KS = H // 16 + 1
    nw = H // 16
    out = np.zeros((nw, 2, KS, 64, 8), np.float32)
    lane = np.arange(64)
    r, hh = lane & 31, lane >> 5
    for w in range(nw):
        for rt in range(2):
            gate, unit = r >> 3, 16 * w + 8 * rt + (r & 7)
            trow = gate * H + unit
            for ks in range(KS):
                for j in range(8):
                    if ks < KS - 1:
                        out[w, rt, ks, :, j] = w_hh[trow, 16 * ks + 8 * hh + j]
                    else:
                        kk = 8 * hh + j
                        v = np.where(kk < I, w_ih[trow, np.minimum(kk, I - 1)] if I > 0 else 0.0,
                                     np.where(kk == I, b[trow], 0.0))
                        out[w, rt, ks, :, j] = v
    return torch.from_numpy(_bf16_bits(out).view(np.uint8).copy())


def pack_aug(aug: np.ndarray, H: int, RT: int) -> np.ndarray:
    """Augmented gate matrix [4H, K] (columns in the B operand's k order,
    K a multiple of 16) -> bf16 A fragments [H/(8 RT) waves, RT, K/16, 64 lanes, 8]
    as uint16: wave w, row tile rt holds the gate rows [i f g o] x 8 units of
    units 8 RT w + 8 rt + (0..7) (lane l: row l & 31, k half l >> 5); the
    rows carry their gate scale (:func:`gate_scales`)."""
    K = aug.shape[1]
    KS = K // 16
    nw = H // (8 * RT)
    aug = _scaled_rows(aug, H)
    lane = np.arange(64)
    r, hh = lane & 31, lane >> 5
    out = np.zeros((nw, RT, KS, 64, 8), np.float32)
    for w in range(nw):
        for rt in range(RT):
            trow = (r >> 3) * H + 8 * RT * w + 8 * rt + (r & 7)
            for ks in range(KS):
                cols = 16 * ks + 8 * hh[:, None] + np.arange(8)[None, :]
                out[w, rt, ks] = aug[trow[:, None], cols]
    return _bf16_bits(out)


def pack_t16(aug: np.ndarray, H: int) -> np.ndarray:
    """Augmented gate matrix [4H, K] (columns in the kernel's k-step order, K
    a multiple of 32) -> bf16 A fragments of v_mfma_f32_16x16x32_bf16 for
    lstm_stack2_t16_kernel: [8 waves, H/32 row tiles, K/32, 64 lanes, 8] as
    uint16.  Row tile rt of wave w is hidden units 32 w + 4 rt + (0..3), rows
    ordered unit-major, gate-minor (row 4u + gate), so a lane's four
    accumulators are one unit's [i f g o]; lane l holds row l & 15, k
    8 (l >> 4) + (0..7) of each 32-k step; rows carry their gate scale."""
    K = aug.shape[1]
    KS = K // 32
    nw, rt_n = 8, H // 32
    aug = _scaled_rows(aug, H)
    lane = np.arange(64)
    r, q4 = lane & 15, lane >> 4
    out = np.zeros((nw, rt_n, KS, 64, 8), np.float32)
    for w in range(nw):
        for rt in range(rt_n):
            trow = (r & 3) * H + 32 * w + 4 * rt + (r >> 2)
            for ks in range(KS):
                cols = 32 * ks + 8 * q4[:, None] + np.arange(8)[None, :]
                out[w, rt, ks] = aug[trow[:, None], cols]
    return _bf16_bits(out)


def pack_stack(layers: list[tuple[torch.Tensor, torch.Tensor, torch.Tensor]], H: int) -> list[torch.Tensor]:
    """[(W_ih, W_hh, b_ih + b_hh)] per layer (torch.nn.LSTM conventions) ->
    the stacked kernel's per-layer fragment buffers (uint8), for the tiling
    ``stack_tiling(H, len(layers))`` picks (pack and run under the same
    FM_LSTM_STACK_TILING)."""
    RT, nct = stack_tiling(H, len(layers))
    if nct == 216:
        return _pack_stack_t16(layers, H)
    out = []
    for li, (w_ih, w_hh, b) in enumerate(layers):
        w_ih, w_hh, b = (t.detach().float().cpu().numpy() for t in (w_ih, w_hh, b))
        I = w_ih.shape[1]
        if li == 0:
            check(I <= 15, "layer-0 input features must be <= 15 (x, then the bias, in one K step)")
            aug = np.zeros((4 * H, H + 16), np.float32)
            aug[:, :H] = w_hh
            aug[:, H:H + I] = w_ih
            aug[:, H + I] = b
        else:
            check(I == H, "stacked layers take the previous layer's h")
            aug = np.zeros((4 * H, 2 * H + 16), np.float32)
            aug[:, :H] = w_hh
            aug[:, H:2 * H] = w_ih
            aug[:, 2 * H] = b
        out.append(torch.from_numpy(pack_aug(aug, H, RT).view(np.uint8).copy()))
    return out


def _pack_stack_t16(layers, H: int) -> list[torch.Tensor]:
    """pack_stack for the 16x16-tile kernel: layer 0 K order [x, 1 | pad to
    32, h0_{t-1}], layer 1 [h1_{t-1}, h0_t, 1 | pad to 32]."""
    check(len(layers) == 2 and H == 256, "the 16x16-tile kernel is the two-layer H = 256 form")
    out = []
    for li, (w_ih, w_hh, b) in enumerate(layers):
        w_ih, w_hh, b = (t.detach().float().cpu().numpy() for t in (w_ih, w_hh, b))
        I = w_ih.shape[1]
        if li == 0:
            check(I <= 15, "layer-0 input features must be <= 15 (x, then the bias, in one K step)")
            aug = np.zeros((4 * H, 32 + H), np.float32)
            aug[:, :I] = w_ih
            aug[:, I] = b
            aug[:, 32:] = w_hh
        else:
            check(I == H, "stacked layers take the previous layer's h")
            aug = np.zeros((4 * H, 2 * H + 32), np.float32)
            aug[:, :H] = w_hh
            aug[:, H:2 * H] = w_ih
            aug[:, 2 * H] = b
        out.append(torch.from_numpy(pack_t16(aug, H).view(np.uint8).copy()))
    return out


def lstm_stack_forward(xa: torch.Tensor, packed: list[torch.Tensor], H: int):
    """xa [B, L, 16] bf16 augmented input -> (h_L, c_L) [B, H] f32 of the TOP
    layer; 1 or 2 layers (``pack_stack``), H in STACK_H."""
    check(xa.dim() == 3 and xa.shape[2] == 16 and xa.dtype == torch.bfloat16 and xa.is_contiguous(),
          "xa must be contiguous [B, L, 16] bfloat16")
    check(H in STACK_H and len(packed) in (1, 2), f"H must be one of {STACK_H}, 1 or 2 layers")
    require_native(xa)
    B, L, _ = xa.shape
    d = xa.device
    hT = torch.empty((B, H), dtype=torch.float32, device=d)
    cT = torch.empty((B, H), dtype=torch.float32, device=d)
    w0 = packed[0].to(d)
    w1 = packed[1].to(d) if len(packed) > 1 else None
    rt, nct = stack_tiling(H, len(packed))
    LIB.call("fm_lstm_stack", ptr(xa), B, L, H, len(packed), ptr(w0), ptr(w1), ptr(hT), ptr(cT), rt, nct,
             stream_of(xa))
    return hT, cT


def lstm_features_mv(hist: torch.Tensor, T: int, S: int, M: int, L: int, period: float):
    """Multivariate input, one row per service: [z(metric 0..M-1), sin, cos, 1]
    of the last L samples -> (xa [S, L, 16] bf16, mu [S*M], sd [S*M])."""
    check(hist.dim() == 2 and hist.dtype == torch.float32 and hist.stride(1) == 1 and hist.shape[0] >= S * M,
          "hist must be [S*M, T] float32")
    check(0 < L <= T <= hist.shape[1] and 0 < M <= 13, "bad window / metric count (M + 3 <= 16)")
    require_native(hist)
    d = hist.device
    xa = torch.empty((S, L, 16), dtype=torch.bfloat16, device=d)
    mu = torch.empty((S * M,), dtype=torch.float32, device=d)
    sd = torch.empty((S * M,), dtype=torch.float32, device=d)
    LIB.call("fm_lstm_features_mv", ptr(hist), hist.stride(0), T, S, M, L, float(period), ptr(xa), ptr(mu), ptr(sd),
             stream_of(hist))
    return xa, mu, sd


def augment(x: torch.Tensor) -> torch.Tensor:
    """[B, L, I] float -> the kernel's augmented input [B, L, 16] bf16
    (features at k < I, 1.0 at k = I for the bias, zeros above)."""
    B, L, I = x.shape
    check(I <= 15, "input features must be <= 15 (folded into one K step with the bias)")
    xa = torch.zeros((B, L, 16), dtype=torch.bfloat16, device=x.device)
    if I:
        xa[..., :I] = x.to(torch.bfloat16)
    xa[..., I] = 1.0
    return xa


def lstm_forward(x: torch.Tensor, packed: torch.Tensor, H: int, h0=None, c0=None, return_seq: bool = False):
    """x [B, L, I] float32 -> (h_L [B,H], c_L [B,H], seq [B,L,H] bf16 or None)."""
    check(x.dim() == 3 and x.dtype == torch.float32 and x.is_contiguous(), "x must be contiguous [B, L, I] float32")
    require_native(x)
    check(x.is_cuda, "lstm_forward runs on the GPU; use ref_lstm_forward on CPU")
    return lstm_forward_packed(augment(x), packed, H, h0, c0, return_seq)


def lstm_forward_packed(xa: torch.Tensor, packed: torch.Tensor, H: int, h0=None, c0=None, return_seq: bool = False):
    """xa [B, L, 16] bf16 augmented input (``augment`` / ``lstm_features``)."""
    check(xa.dim() == 3 and xa.shape[2] == 16 and xa.dtype == torch.bfloat16 and xa.is_contiguous(),
          "xa must be contiguous [B, L, 16] bfloat16")
    check(H in SUPPORTED_H, f"hidden size must be one of {SUPPORTED_H}")
    require_native(xa)
    B, L, _ = xa.shape
    d = xa.device
    hT = torch.empty((B, H), dtype=torch.float32, device=d)
    cT = torch.empty((B, H), dtype=torch.float32, device=d)
    seq = torch.empty((B, L, H), dtype=torch.bfloat16, device=d) if return_seq else None
    pk = packed.to(d)
    for t in (h0, c0):
        check(t is None or (t.is_contiguous() and t.dtype == torch.float32 and tuple(t.shape) == (B, H)),
              "h0/c0 must be contiguous [B, H] float32")
    LIB.call("fm_lstm_forward", ptr(xa), B, L, H, ptr(pk), ptr(h0), ptr(c0), ptr(hT), ptr(cT), ptr(seq),
             stream_of(xa))
    return hT, cT, seq


def lstm_forward_hist(hist: torch.Tensor, T: int, L: int, period: float, I: int, packed: torch.Tensor, H: int,
                      rm: torch.Tensor | None = None, shift: torch.Tensor | None = None,
                      lim: torch.Tensor | None = None, dk: int = 0, B: int | None = None):
    """The univariate forecaster's LSTM straight from the history rows
    (csrc/kernels/lstm.hip ``fm_lstm_forward_hist``): the window features
    (z-score, daily phase) are computed in the kernel, no [B, L, 16] input.
    Sequence b reads row ``rm[b]`` of ``hist`` (or row b), dense columns
    [T - L, T) at ``c - (shift[b] - dk)`` below ``lim[b] + dk`` (a resident
    grid row, engine/fastpath.LazyHist) or the row as is.
    -> (h_L [B, H], c_L [B, H], mu [B], sd [B])."""
    check(hist.dim() == 2 and hist.dtype == torch.float32 and hist.stride(1) == 1, "hist must be [R, T] float32")
    check(H in SUPPORTED_H and 0 <= I <= 3 and 0 < L <= T and period > 0, "bad LSTM / window parameters")
    check((shift is None) == (lim is None), "shift and lim go together")
    require_native(hist)
    B = int(rm.numel()) if rm is not None else (hist.shape[0] if B is None else B)
    d = hist.device
    for t in (rm, shift, lim):
        check(t is None or (t.dtype == torch.int32 and t.is_contiguous() and t.numel() == B), "int32 [B] row maps")
    if rm is None:
        check(hist.shape[0] >= B and hist.shape[1] >= T, "hist too small")
    hT = torch.empty((B, H), dtype=torch.float32, device=d)
    cT = torch.empty((B, H), dtype=torch.float32, device=d)
    mu = torch.empty((B,), dtype=torch.float32, device=d)
    sd = torch.empty((B,), dtype=torch.float32, device=d)
    LIB.call("fm_lstm_forward_hist", ptr(hist), hist.stride(0), T, ptr(rm), ptr(shift), ptr(lim), int(dk), B, L, H,
             float(period), I, ptr(packed.to(d)), ptr(hT), ptr(cT), ptr(mu), ptr(sd), stream_of(hist))
    return hT, cT, mu, sd


def lstm_head(hT: torch.Tensor, W: torch.Tensor, bias: torch.Tensor, mu: torch.Tensor, sd: torch.Tensor,
              Hout: int) -> torch.Tensor:
    """fc [B, Hout] = mu + sd * (hT @ W.T + bias), a horizon past W's rows
    repeating its last step (``fm_lstm_head``, one pass)."""
    B, H = hT.shape
    Hz = W.shape[0]
    check(hT.is_contiguous() and hT.dtype == torch.float32 and W.shape == (Hz, H) and W.is_contiguous()
          and bias.numel() == Hz and mu.numel() == B and sd.numel() == B and 1 <= Hz <= 64, "bad LSTM head shapes")
    require_native(hT)
    fc = torch.empty((B, Hout), dtype=torch.float32, device=hT.device)
    LIB.call("fm_lstm_head", ptr(hT), B, H, ptr(W), ptr(bias.contiguous()), Hz, ptr(mu.contiguous()),
             ptr(sd.contiguous()), int(Hout), ptr(fc), stream_of(hT))
    return fc


def lstm_features(hist: torch.Tensor, T: int, L: int, period: float, I: int = 3):
    """Augmented forecaster input straight from the packed history (GPU):
    -> (xa [R, L, 16] bf16, mu [R], sd [R]).  Features [z, sin, cos][:I] of the
    last L samples (z-score over the window's finite samples, missing -> 0)."""
    check(hist.dim() == 2 and hist.dtype == torch.float32 and hist.stride(1) == 1, "hist must be [R, T] float32")
    check(0 < L <= T <= hist.shape[1] and 0 <= I <= 3, "bad window / feature count")
    require_native(hist)
    R = hist.shape[0]
    d = hist.device
    xa = torch.empty((R, L, 16), dtype=torch.bfloat16, device=d)
    mu = torch.empty((R,), dtype=torch.float32, device=d)
    sd = torch.empty((R,), dtype=torch.float32, device=d)
    LIB.call("fm_lstm_features", ptr(hist), hist.stride(0), T, R, L, float(period), I, ptr(xa), ptr(mu), ptr(sd),
             stream_of(hist))
    return xa, mu, sd


def _rd_gates(w: torch.Tensor, H: int) -> torch.Tensor:
    """Gate-row weights as the kernel sees them: rounded to bf16 after the
    gate scale, the scale divided out again."""
    s = torch.from_numpy(gate_scales(H))
    s = s if w.dim() == 1 else s[:, None]
    return bf16_round(w.float() * s) / s


def ref_lstm_forward(x: torch.Tensor, w_ih, w_hh, bias, h0=None, c0=None, emulate_bf16: bool = True):
    """fp32 reference; with emulate_bf16 the (gate-scaled) weights, inputs and
    the recurrent h are rounded to bf16 exactly where the kernel rounds them."""
    B, L, I = x.shape
    H = w_hh.shape[1]
    rd = bf16_round if emulate_bf16 else (lambda t: t)
    rw = (lambda t: _rd_gates(t, H)) if emulate_bf16 else (lambda t: t.float())
    Wi, Wh, b = rw(w_ih.float()), rw(w_hh.float()), rw(bias.float())
    h = torch.zeros(B, H) if h0 is None else h0.float().clone()
    c = torch.zeros(B, H) if c0 is None else c0.float().clone()
    hr = rd(h)
    xs = rd(x.float())
    for t in range(L):
        g = hr @ Wh.T + xs[:, t] @ Wi.T + b
        i, f, gg, o = g.chunk(4, dim=1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        hr = rd(h)
    return h, c


def ref_lstm_stack(x: torch.Tensor, layers: list, emulate_bf16: bool = True):
    """fp32 reference of the stacked kernel: [(W_ih, W_hh, b)] per layer; with
    emulate_bf16 weights, inputs and every h that feeds a GEMM (the recurrent
    h and layer 0's h into layer 1) are rounded to bf16 as in the kernel.
    -> (h_L, c_L) of the top layer."""
    rd = bf16_round if emulate_bf16 else (lambda t: t)
    B, L, _ = x.shape
    seq = rd(x.float())
    h = c = None
    for w_ih, w_hh, b in layers:
        H = w_hh.shape[1]
        rw = (lambda t: _rd_gates(t, H)) if emulate_bf16 else (lambda t: t.float())   # noqa: B023
        Wi, Wh, bb = rw(w_ih.float()), rw(w_hh.float()), rw(b.float())
        h = torch.zeros(B, H)
        c = torch.zeros(B, H)
        hr = rd(h)
        out = []
        for t in range(L):
            g = hr @ Wh.T + seq[:, t] @ Wi.T + bb
            i, f, gg, o = g.chunk(4, dim=1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
            hr = rd(h)
            out.append(hr)
        seq = torch.stack(out, 1)
    return h, c
