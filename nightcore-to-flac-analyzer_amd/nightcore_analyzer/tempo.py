"""Per-window tempo estimation and the hop-64 full-signal IBI pass
(drop-in for the reference's nightcore_analyzer/tempo.py), on the MI355X.

``estimate_tempo`` (tempo.py:27-77): onset strength (hop 512) -> tempogram
mean -> prior-weighted tempo argmax -> DP beat tracker; fewer than 4 beats ->
None; librosa.feature.tempo gives the identical tempo, so the two estimators
always agree and the result is the tempogram-grid BPM 60*sr/(hop*L).
``estimate_ibis_global`` (tempo.py:120-173): the same at hop 64 over the whole
signal with a streamed (not materialised) tempogram mean.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np

from .io import SAMPLE_RATE, AudioWindow

MIN_BEATS: int = 4
AGREEMENT_TOLERANCE: float = 0.08
HOP_LENGTH: int = 512
IBI_HOP_LENGTH: int = 64
IBI_MIN_IBIS: int = 4


MIN_RATE, MAX_RATE = 8000, 48000   # rates the per-rate tables are built for (nc_create_rate)


def require_rate(sr, what: str) -> None:
    """The chroma / CQT / tuning tables are built for io.SAMPLE_RATE (the rate io.load_audio
    returns, io.py:44-55): the pitch seams raise for another rate instead of analysing with
    the wrong tables.  (The tempo seams take any rate in MIN_RATE..MAX_RATE: rate_engine.)"""
    if int(sr) != SAMPLE_RATE:
        raise ValueError(f"{what}: sample rate {sr} Hz is not supported by the MI355X engine, whose tables "
                         f"are built for {SAMPLE_RATE} Hz; load or resample the audio at {SAMPLE_RATE} Hz "
                         f"(io.load_audio(path, sr={SAMPLE_RATE}))")


def rate_engine(sr, what: str):
    """This thread's engine for audio at ``sr`` Hz: the reference passes sr through to librosa
    (tempo.py:44-50, 139-164), so the mel bank and the tempogram windows are built for that rate
    (engine.get_engine(sr=...), a context from nc_create_rate) rather than resampling."""
    from .engine import get_engine
    sr = int(sr)
    if not MIN_RATE <= sr <= MAX_RATE:
        raise ValueError(f"{what}: sample rate {sr} Hz is outside the engine's {MIN_RATE}..{MAX_RATE} Hz")
    return get_engine(sr=sr)


def estimate_tempo(window: AudioWindow, start_bpm: float = 120.0) -> Optional[float]:
    """tempo.py:27-77 for one window, at window.sample_rate."""
    from .ops import window_tempos
    return window_tempos(rate_engine(window.sample_rate, "estimate_tempo"), [window.audio], [start_bpm])[0]


def batch_estimate_tempo(windows: List[AudioWindow], log: Optional[Callable[[str], None]] = None,
                         start_bpm: float = 120.0) -> List[Optional[float]]:
    """All windows in one device batch per sample rate; the same log lines as tempo.py:102-110."""
    from .ops import window_tempos
    n = len(windows)
    res: List[Optional[float]] = [None] * n
    by_rate: dict = {}
    for i, w in enumerate(windows):
        by_rate.setdefault(int(w.sample_rate), []).append(i)
    for sr, idx in by_rate.items():
        got = window_tempos(rate_engine(sr, "batch_estimate_tempo"), [windows[i].audio for i in idx],
                            [start_bpm] * len(idx))
        for i, g in zip(idx, got):
            res[i] = g
    if log:
        for i, w in enumerate(windows):
            log(f"    tempo window {i + 1}/{n}  [{w.start_sec:.1f}–{w.end_sec:.1f} s]")
        log(f"    {sum(1 for r in res if r is not None)}/{n} windows yielded a confident tempo estimate")
    return res


# the hop-64 beat tracker keeps its DP ring and penalty table (both ~ the 8 s tempogram window in
# frames) in LDS: up to ~26 kHz at hop 64 (beat.hip launch_tempo_beats); the streamed tempogram
# runs hops 64 and 512 with an even window (ibi.hip tg_acw): e.g. 48 kHz at hop 512
IBI_MAX_WINDOW_FRAMES = 3276


def estimate_ibis_global(y: np.ndarray, sr: int, hop_length: int = IBI_HOP_LENGTH,
                         min_ibis: int = IBI_MIN_IBIS, start_bpm: float = 120.0) -> Optional[np.ndarray]:
    from .ops import ibis
    eng = rate_engine(sr, "estimate_ibis_global")
    win = int(8.0 * int(sr)) // int(hop_length)
    if win > IBI_MAX_WINDOW_FRAMES:
        raise ValueError(f"estimate_ibis_global: an 8 s tempogram window at {sr} Hz / hop {hop_length} is "
                         f"{win} frames, more than the beat tracker's {IBI_MAX_WINDOW_FRAMES}; use hop_length=512")
    if int(hop_length) not in (64, 512) or win % 2:
        raise ValueError(f"estimate_ibis_global: the streamed tempogram runs hop_length 64 or 512 with an even "
                         f"8 s window; {sr} Hz / hop {hop_length} gives {win} frames")
    return ibis(eng, [y], [start_bpm], hop=hop_length, min_ibis=min_ibis)[0]
