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

from .io import AudioWindow

MIN_BEATS: int = 4
AGREEMENT_TOLERANCE: float = 0.08
HOP_LENGTH: int = 512
IBI_HOP_LENGTH: int = 64
IBI_MIN_IBIS: int = 4


def estimate_tempo(window: AudioWindow, start_bpm: float = 120.0) -> Optional[float]:
    from .engine import get_engine
    from .ops import window_tempos
    return window_tempos(get_engine(), [window.audio], [start_bpm])[0]


def batch_estimate_tempo(windows: List[AudioWindow], log: Optional[Callable[[str], None]] = None,
                         start_bpm: float = 120.0) -> List[Optional[float]]:
    """All windows in one device batch; the same log lines as tempo.py:102-110."""
    from .engine import get_engine
    from .ops import window_tempos
    n = len(windows)
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
    if sr != 22050:
        raise NotImplementedError("the engine's tables are built for sr = 22050 (io.SAMPLE_RATE)")
    return ibis(get_engine(), [y], [start_bpm], hop=hop_length, min_ibis=min_ibis)[0]
