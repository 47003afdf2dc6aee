"""Windowed waveform cross-correlation speed estimator (drop-in for the
reference's nightcore_analyzer/xcorr.py).

``estimate_speed_xcorr`` (xcorr.py:54-162): the dot-product search and the
decisions run on the MI355X (``nc_xcorr_search``); the reference's integer
geometry (edge trim, linspace window positions, stride candidates) is planned
on the host exactly as the reference computes it.
``find_content_offset`` (xcorr.py:165-259, the intro search of
``pipeline.run(auto_align=True)``): 2:1 resample, RMS envelopes, the 30-speed
stretch / correlate / cosine-score search, all on the MI355X
(``nc_align_offsets``); a batch of pairs is searched at once by the engine.
"""
from __future__ import annotations

from pathlib import Path
from typing import Tuple, Union

import numpy as np

XCORR_SR: int = 22050
XCORR_N_WINDOWS: int = 20
XCORR_WINDOW_SEC: float = 3.0
XCORR_SEARCH_RANGE: float = 0.05
XCORR_SKIP_EDGES: float = 0.10
XCORR_RMS_GATE: float = 1e-3
XCORR_QUALITY_GOOD: float = 0.70
XCORR_QUALITY_FAIR: float = 0.40
ALIGN_SR: int = 11025
ALIGN_HOP: int = 512
ALIGN_SPEED_LO: float = 1.03
ALIGN_SPEED_HI: float = 1.50
ALIGN_N_SPEEDS: int = 30
ALIGN_MAX_OFFSET: float = 120.0
ALIGN_MIN_OFFSET: float = 1.0


def estimate_speed_xcorr_arrays(ya: np.ndarray, yb: np.ndarray, sr: int = XCORR_SR,
                                n_windows: int = XCORR_N_WINDOWS, window_sec: float = XCORR_WINDOW_SEC,
                                search_range: float = XCORR_SEARCH_RANGE,
                                skip_edges: float = XCORR_SKIP_EDGES) -> Tuple[float, float]:
    from .engine import get_engine
    from .ops import xcorr_speed
    return xcorr_speed(get_engine(), ya, yb, sr, n_windows, window_sec, search_range, skip_edges)


def estimate_speed_xcorr(path_a: Union[str, Path], path_b: Union[str, Path], sr: int = XCORR_SR,
                         n_windows: int = XCORR_N_WINDOWS, window_sec: float = XCORR_WINDOW_SEC,
                         search_range: float = XCORR_SEARCH_RANGE,
                         skip_edges: float = XCORR_SKIP_EDGES) -> Tuple[float, float]:
    """speed_A / speed_B and the median normalised correlation; (1.0, 0.0) with < 3 matches."""
    from .io import load_audio
    ya, _ = load_audio(str(path_a), sr=sr)
    yb, _ = load_audio(str(path_b), sr=sr)
    return estimate_speed_xcorr_arrays(ya, yb, sr, n_windows, window_sec, search_range, skip_edges)


def find_content_offset(src_audio: np.ndarray, nc_audio: np.ndarray, sr: int, *, speed_lo: float = ALIGN_SPEED_LO,
                        speed_hi: float = ALIGN_SPEED_HI, n_speeds: int = ALIGN_N_SPEEDS,
                        max_offset_sec: float = ALIGN_MAX_OFFSET) -> Tuple[float, float]:
    """(offset_sec, speed_est): seconds of src_audio before the content that matches the
    start of nc_audio, and the speed of the best (speed, lag) envelope match."""
    from .engine import get_engine
    eng = get_engine()
    sig = eng.upload_signals([np.asarray(src_audio, np.float32), np.asarray(nc_audio, np.float32)])
    return eng.align_offsets(sig.buf, sig.off[:1], sig.length[:1], sig.off[1:], sig.length[1:], sr,
                             speed_lo, speed_hi, n_speeds, max_offset_sec)[0]


def quality_label(quality: float) -> str:
    if quality >= XCORR_QUALITY_GOOD:
        return "good match"
    if quality >= XCORR_QUALITY_FAIR:
        return "moderate match"
    return "poor match — possible content mismatch or heavy lossy artefacts"
