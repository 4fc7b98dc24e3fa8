"""ctypes binding of ``libforemast_hip.so`` (the CDNA4 kernel library).

Every kernel has a plain C entry point taking raw device pointers and the HIP
stream handle of the caller's current torch stream, so launches land on the
same stream torch uses (and are captured by ``torch.cuda.CUDAGraph`` on ROCm,
which records HIP stream captures).

Policy: a GPU tensor is ALWAYS scored by the native kernel.  If the library is
missing on a machine with a GPU the import-time check raises
:class:`NativeLibraryMissing` instead of silently falling back to the CPU
reference path (the CPU path is only for CPU tensors).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_NATIVE_DIR = Path(__file__).resolve().parent.parent / "_native"
_LIB_PATH = Path(os.environ.get("FOREMAST_HIP_LIB", _NATIVE_DIR / "libforemast_hip.so"))

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u32 = ctypes.c_uint32
c_float = ctypes.c_float

# name -> argtypes (all return int = hipError_t)
_SIGS: dict[str, list] = {
    "fm_pairwise_tests": [c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_i64, c_int, c_int, c_float, c_int,
                          c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_stats_decide": [c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_i64, c_int, c_void_p, c_void_p, c_void_p,
                        c_float, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_service_reduce": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p],
    "fm_hist_stats": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p],
    "fm_window_decide": [c_void_p, c_void_p, c_i64, c_int, c_i64, c_int, c_void_p, c_void_p, c_void_p, c_float,
                         c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_compact_anomalies": [c_void_p, c_int, c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_void_p, c_void_p,
                             c_void_p, c_void_p],
    "fm_synth_fleet": [c_void_p, c_i64, c_i64, c_i64, c_int, c_i64, c_int, c_int, c_int, c_int, c_float, c_float,
                       c_u32, c_void_p],
    "fm_es_fit": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                  c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "fm_hw_scan_fit": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_int, c_int] + [c_void_p] * 9
                      + [c_float, c_int, c_void_p],
    "fm_hw_scan_supported": [c_int, c_int, c_int],
    "fm_hw_scan_set_probe": [c_void_p],
    "fm_ipc_handle_size": [],
    "fm_ipc_get_handle": [c_void_p, c_void_p, c_void_p],
    "fm_ipc_open": [c_void_p, c_void_p],
    "fm_ipc_close": [c_void_p],
    "fm_peer_publish": [c_void_p, c_void_p, c_i64, c_void_p, ctypes.c_uint, c_void_p, c_void_p],
    "fm_peer_wait": [c_void_p, c_int, c_i64, ctypes.c_uint, ctypes.c_longlong, c_void_p, c_void_p],
    "fm_peer_ack": [c_void_p, c_int, ctypes.c_uint, c_void_p],
    "fm_peer_wait_ctr": [c_void_p, c_int, c_i64, c_void_p, ctypes.c_uint, ctypes.c_longlong, c_void_p, c_void_p, c_int,
                         c_void_p],
    "fm_peer_publish_ctr": [c_void_p, c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "fm_peer_ack_ctr": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p],
    # buf ld rm shift lim dk T kmax t_new slots params m kind season sse state nobs cur ld_c n hor H S M thr bound
    # minlb diff pair_factor valid lastk upper lower sigma fc Hf hostv cap ctr par out_idx out_val last3 stream
    "fm_es_band_step": [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                        c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int,
                        c_void_p, c_int, c_i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int,
                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_lstm_forward_hist": [c_void_p, c_i64, c_int, c_void_p, c_void_p, c_void_p, c_int, c_i64, c_int, c_int,
                             c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_grid_retire": [c_void_p, c_i64, c_i64, c_int, c_int, c_void_p, c_void_p],
    "fm_hpa_score_slots": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                           ctypes.c_double, c_float, c_float, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p],
    "fm_lstm_head": [c_void_p, c_i64, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "fm_es_update": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "fm_band_decide": [c_void_p, c_i64, c_int, c_void_p, c_i64, c_void_p, c_i64, c_int, c_void_p, c_void_p,
                       c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                       c_void_p],
    "fm_fft_seasonal": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                        c_i64, c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_phase_profile": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_bivariate": [c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "fm_hpa_score": [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                     ctypes.c_double, c_float, c_float, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_downstream_impact": [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p, c_void_p],
    "fm_segment_max": [c_void_p, c_void_p, c_i64, c_int, c_void_p, c_void_p],
    "fm_gather_cols": [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_i64, c_void_p],
    "fm_selftest_lanes": [c_void_p, c_void_p, c_void_p],
    "fm_decide_services": [c_void_p, c_void_p, c_i64, c_int, c_i64, c_int, c_void_p, c_void_p, c_void_p, c_float,
                           c_void_p, c_int, c_int, c_float, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_pvalues_only": [c_void_p, c_i64, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "fm_pairwise_suff": [c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_void_p],
    "fm_pairwise_suff_v": [c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_int, c_void_p],
    "fm_hist_stats_capped": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_void_p],
    "fm_pvalues": [c_void_p, c_i64, c_int, c_int, c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                   c_void_p],
    "fm_canary_rows": [c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_void_p, c_i64, c_int, c_i64, c_void_p,
                       c_void_p, c_void_p],
    "fm_lsq_project": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_void_p],
    "fm_lsq_residual": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_stream_read": [c_void_p, c_i64, c_void_p, c_int, c_void_p],
    "fm_lstm_forward": [c_void_p, c_i64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p],
    "fm_lstm_forward_nct": [c_void_p, c_i64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_int, c_void_p],
    "fm_lstm_forward_v": [c_void_p, c_i64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_int, c_int, c_void_p],
    "fm_tick_front": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_i64, c_int,
                      c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fm_tick_front_rm": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_void_p, c_i64, c_int, c_void_p, c_i64, c_int,
                         c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p],
    "fm_hist_stats_rm": [c_void_p, c_i64, c_int, c_i64, c_void_p, c_int, c_void_p, c_void_p],
    "fm_copy_d2h_async": [c_void_p, c_void_p, c_i64, c_void_p],
    "fm_memcpy_sync": [c_void_p, c_void_p, c_i64],
    "fm_board_copy": [c_void_p, c_void_p, c_i64],
    "fm_rolling_stats": [c_void_p, c_i64, c_int, c_i64, c_int, c_int, c_void_p, c_void_p, c_i64, c_void_p],
    "fm_pvalues_range": [c_void_p, c_i64, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "fm_lstm_stack": [c_void_p, c_i64, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                      c_void_p],
    "fm_lstm_features_mv": [c_void_p, c_i64, c_int, c_i64, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p,
                            c_void_p],
    "fm_lstm_features": [c_void_p, c_i64, c_int, c_i64, c_int, c_float, c_int, c_void_p, c_void_p, c_void_p,
                         c_void_p],
}


class NativeLibraryMissing(RuntimeError):
    pass


class _Lib:
    def __init__(self) -> None:
        self._lib = None
        self._err: str | None = None

    def load(self):
        if self._lib is not None:
            return self._lib
        if not _LIB_PATH.exists():
            raise NativeLibraryMissing(
                f"{_LIB_PATH} not built; run `python tools/build_native.py` (or __graft_entry__.build())")
        lib = ctypes.CDLL(str(_LIB_PATH))
        for name, argt in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argt
            fn.restype = c_int
        self._lib = lib
        return lib

    def register(self, name: str, argtypes: list) -> None:
        _SIGS[name] = argtypes
        if self._lib is not None:
            fn = getattr(self._lib, name)
            fn.argtypes = argtypes
            fn.restype = c_int

    def available(self) -> bool:
        try:
            self.load()
            return True
        except (NativeLibraryMissing, OSError):
            return False

    def call(self, name: str, *args) -> None:
        lib = self.load()
        fn = getattr(lib, name)
        rc = fn(*args)
        if rc != 0:
            raise RuntimeError(f"{name} failed with hipError {rc}")


LIB = _Lib()


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def require_native(t: torch.Tensor) -> None:
    """GPU tensors must go through the HIP kernels; fail loudly otherwise."""
    if t.is_cuda and not LIB.available():
        raise NativeLibraryMissing(f"HIP kernel library missing ({_LIB_PATH}); refusing eager fallback on GPU")


def check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)
