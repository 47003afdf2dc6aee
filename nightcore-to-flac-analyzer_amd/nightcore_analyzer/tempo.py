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


def require_rate(sr, what: str) -> None:
    """The engine's STFT / mel / tempogram / CQT tables are built for io.SAMPLE_RATE (the
    rate io.load_audio returns, io.py:44-55).  Another rate raises instead of being
    analysed with the wrong tables."""
    if int(sr) != SAMPLE_RATE:
        raise ValueError(f"{what}: sample rate {sr} Hz is not supported by the MI355X engine, whose tables "
                         f"are built for {SAMPLE_RATE} Hz; load or resample the audio at {SAMPLE_RATE} Hz "
                         f"(io.load_audio(path, sr={SAMPLE_RATE}))")


def estimate_tempo(window: AudioWindow, start_bpm: float = 120.0) -> Optional[float]:
    """tempo.py:27-77 for one window, at window.sample_rate."""
    from .engine import get_engine
    from .ops import window_tempos
    require_rate(window.sample_rate, "estimate_tempo")
    return window_tempos(get_engine(), [window.audio], [start_bpm])[0]


def batch_estimate_tempo(windows: List[AudioWindow], log: Optional[Callable[[str], None]] = None,
                         start_bpm: float = 120.0) -> List[Optional[float]]:
    """All windows in one device batch; the same log lines as tempo.py:102-110."""
    from .engine import get_engine
    from .ops import window_tempos
    n = len(windows)
    for w in windows:
        require_rate(w.sample_rate, "batch_estimate_tempo")
    res = window_tempos(get_engine(), [w.audio for w in windows], [start_bpm] * n) if n else []
    if log:
        for i, w in enumerate(windows):
            log(f"    tempo window {i + 1}/{n}  [{w.start_sec:.1f}–{w.end_sec:.1f} s]")
        log(f"    {sum(1 for r in res if r is not None)}/{n} windows yielded a confident tempo estimate")
    return res


def estimate_ibis_global(y: np.ndarray, sr: int, hop_length: int = IBI_HOP_LENGTH,
                         min_ibis: int = IBI_MIN_IBIS, start_bpm: float = 120.0) -> Optional[np.ndarray]:
    from .engine import get_engine
    from .ops import ibis
    require_rate(sr, "estimate_ibis_global")
    return ibis(get_engine(), [y], [start_bpm], hop=hop_length, min_ibis=min_ibis)[0]
