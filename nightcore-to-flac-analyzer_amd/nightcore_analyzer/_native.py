"""ctypes binding of libncgpu.so (the C ABI declared in include/ncgpu.h).

This is the only door from Python into the MI355X engine.  There is no CPU
fallback: if the shared library or a HIP device is missing, every entry point
raises ``NativeUnavailable`` — the product path fails loudly instead of
silently computing something else.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

# NCGPU_LIB: another build of the library (A/B timing of kernel variants, tools/ab_bench.sh)
_LIB_PATH = Path(os.environ.get("NCGPU_LIB") or Path(__file__).resolve().parent / "_lib" / "libncgpu.so")
_lock = threading.Lock()
_lib = None

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
F32 = C.c_float
D = C.c_double
SZ = C.c_size_t

# name -> (restype, argtypes); mirrors include/ncgpu.h
SIGNATURES = {
    "nc_abi_version": (I32, []),
    "nc_last_error": (C.c_char_p, []),
    "nc_create": (I32, [I32, C.POINTER(P)]),
    "nc_profile_enable": (I32, [P, I32]),
    "nc_profile_read": (I32, [P, C.c_char_p, C.POINTER(D), C.POINTER(I32)]),
    "nc_profile_read_span": (I32, [P, C.c_char_p, C.POINTER(D), C.POINTER(I32)]),
    "nc_profile_read_busy": (I32, [P, C.POINTER(D), C.POINTER(D), C.POINTER(I32)]),
    "nc_profile_dump_spans": (I32, [P, P, I32, P, P, P, I32, C.POINTER(I32)]),
    "nc_destroy": (I32, [P]),
    "nc_num_cu": (I32, [P]),
    "nc_trim_workspace_bytes": (SZ, [P, I32]),
    "nc_trim_bounds": (I32, [P, P, P, P, I32, I64, F32, P, P, P, SZ, P]),
    "nc_window_stage_workspace_bytes": (SZ, [P, I32, I32, I32]),
    "nc_window_stage": (I32, [P, P, P, P, I32, I32, I32, P, P, P, P, SZ, P]),
    "nc_tempo_beats_workspace_bytes": (SZ, [I64]),
    "nc_tempo_beats": (I32, [P, P, P, P, I32, I32, P, I32, P, P, P, I32, I32, P, P, P, P, P,
                             I64, P, SZ, P]),
    "nc_tempo_prior": (I32, [P, P, P, P, P, P, P, P, I32, P, P]),
    "nc_ibi_from_beats": (I32, [P, P, P, P, I32, I32, I32, P, P, P]),
    "nc_chroma_workspace_bytes": (SZ, [P, I32, I64]),
    "nc_chroma_mean": (I32, [P, P, P, P, I32, I64, I64, P, P, P, P, P, SZ, P]),
    "nc_chroma_lag": (I32, [P, P, P, P, I32, P, P]),
    "nc_chroma_lag_margin": (I32, [P, P, P, P, I32, P, P, P]),
    "nc_xcorr_peak": (I32, [P, P, P, I32, I32, P, P]),
    "nc_window_stage_tuning": (I32, [P, P, P, P, I32, I32, I32, P, P, P, P, P, I32, P, P, P, P, P, SZ, P]),
    "nc_chroma_mean_shared": (I32, [P, P, P, P, I32, I64, I64, P, P, P, P, P, I64, P, P, P, P, P, SZ, P]),
    "nc_window_energy": (I32, [P, P, P, I32, I32, P, P]),
    "nc_energy_gate": (I32, [P, P, P, P, I32, D, P, P]),
    "nc_collect_valid": (I32, [P, P, P, P, P, P, I32, I32, P, P, P]),
    "nc_pitch_hz": (I32, [P, P, I32, P, P, P, P]),
    "nc_bootstrap_job_bytes": (SZ, [I32, I32]),
    "nc_bootstrap_ratio": (I32, [P, P, P, P, P, P, I32, I32, P, D, D, D, D, I32, P, P, P, P, P, P, P,
                                 SZ, P]),
    "nc_ibi_onset_workspace_bytes": (SZ, [P, I32, I64]),
    "nc_ibi_onset": (I32, [P, P, P, P, I32, I64, I32, P, P, P, SZ, P]),
    "nc_ibi_tempogram_workspace_bytes": (SZ, [P, I32, I64, I32, I32]),
    "nc_ibi_tempogram": (I32, [P, P, P, I32, I64, I32, I32, P, P, SZ, P]),
    "nc_ibi_range_workspace_bytes": (SZ, [P, I32, I64]),
    "nc_ibi_mel_range": (I32, [P, P, P, P, I32, P, P, I32, I64, P, P, SZ, P]),
    "nc_ibi_onset_range": (I32, [P, I32, P, I32, I64, P, P, P, I64, P]),
    "nc_ibi_tempogram_tiles": (I32, [P, P, P, I32, I64, I32, I32, P, P, P, P, SZ, P]),
    "nc_ibi_tempogram_reduce": (I32, [P, P, P, I32, I32, I32, P, P]),
    "nc_xcorr_search": (I32, [P, P, P, P, I32, I32, P, P, P, P, P, P, P, P, P, P, I32, P, P, P]),
    "nc_align_workspace_bytes": (SZ, [P, I32, I32, I64, I64, I32]),
    "nc_align_offsets": (I32, [P, P, P, P, P, P, I32, P, I32, I32, I64, I64, P, P, P, P, SZ, P]),
    "nc_spectral_workspace_bytes": (SZ, [I64, I32, I64]),
    "nc_spectral_stats": (I32, [P, P, P, P, P, P, P, I32, I64, I64, F32, P, P, P, P, SZ, P]),
    "nc_resample_poly": (I32, [P, P, P, P, I32, P, P, P, I64, P, I32, I32, I32, I64, P]),
    "nc_pcm16_to_f32": (I32, [P, P, I64, P, P]),
    "nc_create_rate": (I32, [I32, I32, C.POINTER(P)]),
    "nc_window_energy_blocks": (I32, [P, P, P, I32, P, P, P, I32, I32, P, P]),
    "nc_melodia_salience": (I32, [P, P, P, P, P, I32, I64, I32, F32, P, I32, P, P, P, P]),
}


class NativeUnavailable(RuntimeError):
    """libncgpu.so or a HIP device is not available (no CPU fallback exists)."""


class NativeError(RuntimeError):
    """An engine entry point returned a non-zero status."""


def lib_path() -> Path:
    return _LIB_PATH


def load():
    """Load libncgpu.so and bind the declared symbols (idempotent)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # torch-ROCm ships its own libamdhip64; load it first so libncgpu.so binds to
        # the same HIP runtime instance (one device context, shared streams).
        import torch  # noqa: F401
        if not _LIB_PATH.exists():
            raise NativeUnavailable(
                f"{_LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        lib = C.CDLL(str(_LIB_PATH), mode=os.RTLD_LOCAL if hasattr(os, "RTLD_LOCAL") else 0)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols() -> list[str]:
    lib = load()
    return [n for n in SIGNATURES if getattr(lib, n, None) is not None]


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().nc_last_error()
        raise NativeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


class Context:
    """One engine context per (device, thread) — holds the read-only tables."""

    def __init__(self, device: int = 0, sr: int = 22050):
        lib = load()
        h = P()
        rc = lib.nc_create(int(device), C.byref(h)) if sr == 22050 else \
            lib.nc_create_rate(int(device), int(sr), C.byref(h))
        if rc != 0:
            msg = lib.nc_last_error()
            raise NativeUnavailable(f"nc_create(device={device}, sr={sr}) failed: {msg.decode() if msg else rc}")
        self.lib = lib
        self.h = h
        self.device = device
        self.sr = int(sr)

    def close(self):
        if getattr(self, "h", None):
            self.lib.nc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def call(self, name: str, *args):
        fn = getattr(self.lib, name, None)
        if fn is None:
            raise NativeUnavailable(f"{name} not exported by {_LIB_PATH}")
        check(fn(self.h, *args), name)
