"""LSTM forecaster for HPA / ClusterAutoScaler prediction (BASELINE config 4;
docs/guides/design.md:81-85 "Deep Learning (LSTM)", README.md:58-59).

Inference runs the hand-written bf16 MFMA LSTM kernels (``ops.lstm``) over the
last ``window`` samples, then a linear head maps h_T to ``horizon`` future
points.  Two input modes:

* univariate (``n_metrics=None``): one sequence per series, features
  [z, sin, cos] of the daily phase;
* multivariate (``n_metrics=M``, the reference's "LSTM for 3+ metrics",
  docs/guides/design.md:81-85): one sequence per SERVICE whose features are
  the z-scores of all M metrics plus the phase; the head forecasts all M.

H in {32, 64, 128} with one layer runs the register-resident kernel
(lstm.hip); H = 256 and/or two stacked layers run the streamed-weight kernel
(lstm_stack.hip), which keeps layer 0's h on chip for layer 1.  Training
(``fit``) uses torch autograd on an ``nn.LSTM`` with identical parameters —
the reference trained Keras models offline too (foremast-brain/faq.md:10);
the trained weights are what the HIP forward consumes.  Weights persist via
``engine.checkpoint`` (safetensors).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import lstm as LS


class LSTMForecaster:
    def __init__(self, hidden: int = 128, window: int = 240, horizon: int = 60, n_features: int = 3,
                 seed: int = 0, device="cpu", period: float = 1440.0, layers: int = 1, n_metrics: int | None = None):
        assert hidden in LS.STACK_H and layers in (1, 2)
        self.M = n_metrics
        if n_metrics is not None:
            assert 1 <= n_metrics <= 13, "multivariate input: M z-scores + sin + cos + bias in one 16-wide K step"
            n_features = n_metrics + 2
        self.H, self.L, self.horizon, self.I = hidden, window, horizon, n_features
        self.layers = layers
        self.period = period
        self.device = torch.device(device)
        g = torch.Generator().manual_seed(seed)
        self.lstm = torch.nn.LSTM(n_features, hidden, num_layers=layers, batch_first=True)
        self.head = torch.nn.Linear(hidden, horizon * (n_metrics or 1))
        k = 1.0 / math.sqrt(hidden)
        with torch.no_grad():
            for p in list(self.lstm.parameters()) + list(self.head.parameters()):
                p.copy_(torch.empty_like(p).uniform_(-k, k, generator=g))
        self._packed = None

    @classmethod
    def default(cls, device="cpu") -> "LSTMForecaster":
        return cls(device=device)

    # ------------------------------------------------------------------ params
    def state_dict(self) -> dict[str, torch.Tensor]:
        sd = {f"lstm.{k}": v.detach().cpu() for k, v in self.lstm.state_dict().items()}
        sd.update({f"head.{k}": v.detach().cpu() for k, v in self.head.state_dict().items()})
        return sd

    def load_state_dict(self, sd: dict[str, torch.Tensor]) -> None:
        self.lstm.load_state_dict({k[5:]: v for k, v in sd.items() if k.startswith("lstm.")})
        self.head.load_state_dict({k[5:]: v for k, v in sd.items() if k.startswith("head.")})
        self._packed = None
        self._head_dev = None

    @property
    def stacked(self) -> bool:
        """Streamed-weight kernel (H = 256 or two layers)."""
        return self.layers > 1 or self.H not in LS.SUPPORTED_H

    def packed(self):
        if self._packed is None:
            l = self.lstm
            if self.stacked:
                ws = [(getattr(l, f"weight_ih_l{k}"), getattr(l, f"weight_hh_l{k}"),
                       getattr(l, f"bias_ih_l{k}") + getattr(l, f"bias_hh_l{k}")) for k in range(self.layers)]
                self._packed = [p.to(self.device) for p in LS.pack_stack(ws, self.H)]
            else:
                self._packed = LS.pack_lstm(l.weight_ih_l0, l.weight_hh_l0,
                                            l.bias_ih_l0 + l.bias_hh_l0).to(self.device)
        return self._packed

    def _run(self, xa: torch.Tensor) -> torch.Tensor:
        if self.stacked:
            return LS.lstm_stack_forward(xa, self.packed(), self.H)[0]
        return LS.lstm_forward_packed(xa, self.packed(), self.H)[0]

    # ------------------------------------------------------------------ features
    def features(self, hist: torch.Tensor, T: int):
        """[R, L, I] float32: z-scored value, sin/cos of the daily phase."""
        L = min(self.L, T)
        win = hist[:, T - L:T].float()
        ok = torch.isfinite(win)
        n = ok.sum(1).clamp(min=1)
        mu = torch.where(ok, win, torch.zeros_like(win)).sum(1) / n
        var = torch.where(ok, (win - mu[:, None]) ** 2, torch.zeros_like(win)).sum(1) / n
        sd = var.sqrt().clamp(min=1e-6)
        z = torch.where(ok, (win - mu[:, None]) / sd[:, None], torch.zeros_like(win))
        t = torch.arange(T - L, T, device=hist.device, dtype=torch.float32)
        ph = 2 * math.pi * t / self.period
        feats = [z, torch.sin(ph).expand_as(z), torch.cos(ph).expand_as(z)][: self.I]
        return torch.stack(feats, -1).contiguous(), mu, sd

    def features_mv(self, hist: torch.Tensor, T: int):
        """Multivariate features [S, L, M + 2] (rows of ``hist`` are services x M)."""
        M = self.M
        R = hist.shape[0]
        x, mu, sd = self.features_uni(hist, T)            # [R, L, 3]: z, sin, cos
        S = R // M
        z = x[..., 0].reshape(S, M, -1).permute(0, 2, 1)   # [S, L, M]
        return torch.cat([z, x[: S * M: M, :, 1:3]], -1).contiguous(), mu, sd

    def features_uni(self, hist, T):
        I, self.I = self.I, 3
        try:
            return self.features(hist, T)
        finally:
            self.I = I

    @property
    def reads_rows(self) -> bool:
        """The GPU forward takes history rows directly (:meth:`forecast_rows`):
        univariate, one layer, register-resident kernel."""
        return self.M is None and not self.stacked

    @torch.no_grad()
    def forecast_rows(self, src: torch.Tensor, rm: torch.Tensor | None, shift: torch.Tensor | None,
                      lim: torch.Tensor | None, dk: int, T: int, H: int, B: int | None = None):
        """:meth:`forecast` of the rows ``src[rm]`` of a resident grid
        (LazyHist's row map / alignment), read by the LSTM kernel itself: the
        window is never gathered and no feature tensor is written."""
        assert self.reads_rows and src.is_cuda
        L = min(self.L, T)
        hT, _, mu, sd = LS.lstm_forward_hist(src, T, L, self.period, self.I, self.packed(), self.H, rm, shift, lim,
                                             dk, B)
        return self._head(hT, mu, sd, hT.shape[0], H)

    def _head(self, hT, mu, sd, R: int, H: int):
        if hT.is_cuda and self.M is None and self.H in (32, 64, 128, 256) and self.horizon <= 64:
            # linear head + de-normalisation in one kernel (fm_lstm_head)
            dev = hT.device
            hw = getattr(self, "_head_dev", None)
            if hw is None or hw[0] != dev:
                hw = self._head_dev = (dev, self.head.weight.detach().float().contiguous().to(dev),
                                       self.head.bias.detach().float().contiguous().to(dev))
            return LS.lstm_head(hT, hw[1], hw[2], mu, sd, H), sd.contiguous()
        W = self.head.weight.to(hT.device)
        b = self.head.bias.to(hT.device)
        z = hT @ W.T + b                                    # [rows, horizon (x M)]
        if self.M is not None:
            z = z.reshape(-1, self.M, self.horizon).reshape(R, self.horizon)
        if H > self.horizon:
            z = torch.cat([z, z[:, -1:].expand(-1, H - self.horizon)], 1)
        fc = mu[:, None] + sd[:, None] * z[:, :H]
        return fc.contiguous(), sd.contiguous()

    @torch.no_grad()
    def forecast(self, hist: torch.Tensor, T: int, H: int):
        """-> (forecast [R, H] in data units, sigma [R]) with sigma = window std.
        Multivariate models take rows as services x M (R % M == 0)."""
        R = hist.shape[0]
        if self.M is not None:
            assert R % self.M == 0, "multivariate forecaster: rows must be services x n_metrics"
        L = min(self.L, T)
        if hist.is_cuda and self.reads_rows and hist.stride(1) == 1 and hist.dtype == torch.float32:
            return self.forecast_rows(hist, None, None, None, 0, T, H, B=R)
        if hist.is_cuda:
            # features written by a HIP kernel straight into the bf16 augmented layout
            if self.M is not None:
                xa, mu, sd = LS.lstm_features_mv(hist, T, R // self.M, self.M, L, self.period)
            else:
                xa, mu, sd = LS.lstm_features(hist, T, L, self.period, self.I)
            hT = self._run(xa)
        else:
            x, mu, sd = self.features_mv(hist, T) if self.M is not None else self.features(hist, T)
            with torch.no_grad():
                _, (h, _) = self.lstm(x)
                hT = h[-1]
        return self._head(hT, mu, sd, R, H)

    # ------------------------------------------------------------------ training
    def fit(self, hist: torch.Tensor, T: int, epochs: int = 2, batch: int = 256, lr: float = 1e-3,
            max_windows: int = 4096, seed: int = 0) -> list[float]:
        """Train on sliding windows of the history (next-``horizon`` targets).

        Data-parallel when torch.distributed is initialised: every rank samples
        windows from its own shard of rows and the gradients are averaged with
        ONE all-reduce of a flat buffer per step (C4, SURVEY §2.5: the whole
        model is ~70k parameters, so one bucket; ring all-reduce over xGMI is
        per-link bound and a single message amortises its latency)."""
        dev = hist.device
        lstm = self.lstm.to(dev)
        head = self.head.to(dev)
        rng = np.random.default_rng(seed)
        L, Hz = min(self.L, T - self.horizon - 1), self.horizon
        R = hist.shape[0]
        ends = rng.integers(L, T - Hz, size=max_windows)
        rows = rng.integers(0, R, size=max_windows)
        opt = torch.optim.Adam(list(lstm.parameters()) + list(head.parameters()), lr=lr)
        losses = []
        for _ in range(epochs):
            for s in range(0, max_windows, batch):
                e, r = ends[s:s + batch], rows[s:s + batch]
                idx = torch.as_tensor(e[:, None] + np.arange(-L, Hz)[None, :], device=dev)
                seg = hist[torch.as_tensor(r, device=dev)[:, None], idx].float()
                seg = torch.nan_to_num(seg, nan=0.0)
                t = torch.as_tensor(e[:, None] + np.arange(-L, 0)[None, :], device=dev, dtype=torch.float32)
                ph = 2 * math.pi * t / self.period
                if self.M is None:
                    win, tgt = seg[:, :L], seg[:, L:]
                    mu, sd = win.mean(1, keepdim=True), win.std(1, keepdim=True).clamp(min=1e-6)
                    x = torch.stack([(win - mu) / sd, torch.sin(ph), torch.cos(ph)][: self.I], -1)
                    target = (tgt - mu) / sd
                else:
                    # rows are services: all M metric rows of service r // M
                    M = self.M
                    svc = torch.as_tensor((r // M) * M, device=dev)[:, None] + torch.arange(M, device=dev)[None, :]
                    seg = torch.nan_to_num(hist[svc[:, :, None], idx[:, None, :]].float(), nan=0.0)  # [b, M, L+Hz]
                    win, tgt = seg[..., :L], seg[..., L:]
                    mu, sd = win.mean(2, keepdim=True), win.std(2, keepdim=True).clamp(min=1e-6)
                    x = torch.cat([((win - mu) / sd).permute(0, 2, 1), torch.sin(ph)[..., None],
                                   torch.cos(ph)[..., None]], -1)
                    target = ((tgt - mu) / sd).reshape(len(r), -1)
                _, (h, _) = lstm(x)
                pred = head(h[-1])
                loss = torch.nn.functional.mse_loss(pred, target)
                opt.zero_grad()
                loss.backward()
                _allreduce_grads(list(lstm.parameters()) + list(head.parameters()))
                opt.step()
                losses.append(float(loss.item()))
        self.lstm, self.head = lstm.cpu(), head.cpu()
        self._packed = None
        return losses


def _allreduce_grads(params: list[torch.nn.Parameter]) -> None:
    from ..parallel import dist as D
    if not D.is_dist():
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    torch.distributed.all_reduce(flat)
    flat /= torch.distributed.get_world_size()
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def smoke_forward(device) -> None:
    """Tiny LSTM forecast through the HIP kernel (used by __graft_entry__.smoke)."""
    m = LSTMForecaster(hidden=64, window=48, horizon=8, device=device)
    hist = torch.randn(70, 96, device=device).cumsum(1).contiguous()
    fc, sd = m.forecast(hist, 96, 8)
    torch.cuda.synchronize(device)
    assert torch.isfinite(fc).all()
    print("smoke: lstm forecast", tuple(fc.shape))
