"""Pitch-shift detection by chromagram cross-correlation
(drop-in for the reference's nightcore_analyzer/pitch.py), on the MI355X.

Faithful to the reference including its 1/3 quirk:
``chroma_cqt(bins_per_octave=36)`` keeps librosa's default n_chroma = 12, so
the 12-lag cyclic cross-correlation finds whole-semitone lags and
``_chroma_shift_for_chunk`` divides by 3.0 — reported shifts are one third of
the true semitone shift.  MELODIA refinement needs essentia, which is not
installed; as in the reference (pitch.py:178-201) it is then skipped.
"""
from __future__ import annotations

import math
from typing import Callable, List, Optional, Tuple

import numpy as np

CHROMA_BINS_PER_OCTAVE: int = 36
CHROMA_HOP_LENGTH: int = 512
CHUNK_SEC: float = 20.0
MIN_CHUNKS: int = 3
MELODIA_AGREE_ST: float = 1.5
MAX_MELODIA_FRAMES: int = 2000
_REF_HZ: float = 440.0


def _mean_chroma(audio: np.ndarray, sr: int) -> np.ndarray:
    """Time-averaged 12-bin CQT chroma (pitch.py:55-64)."""
    from .engine import get_engine
    from .ops import chroma_means
    return chroma_means(get_engine(), [audio])[0][0]


def _cyclic_xcorr_peak(src_chroma: np.ndarray, nc_chroma: np.ndarray) -> int:
    """Wrapped argmax_k dot(src, roll(nc, -k)) (pitch.py:67-85), on the device."""
    import torch
    from .engine import get_engine
    from .ops import chroma_lags
    eng = get_engine()
    n = len(src_chroma)
    if n != 12:
        raise ValueError("the engine's cross-correlation kernel is 12-bin (n_chroma = 12)")
    d = torch.tensor(np.concatenate([src_chroma, nc_chroma]).astype(np.float32), device=eng.dev)
    return chroma_lags(eng, d, [0], [1])[0]


def _chroma_shift_for_chunk(src_chunk: np.ndarray, nc_chunk: np.ndarray, sr: int) -> float:
    from .engine import get_engine
    from .ops import chroma_means, chroma_lags
    eng = get_engine()
    _, _, dev_chroma = chroma_means(eng, [src_chunk, nc_chunk])
    return chroma_lags(eng, dev_chroma, [0], [1])[0] / 3.0


def _chunk_plan(n_src: int, n_nc: int, sr: int):
    cn = int(CHUNK_SEC * sr)
    n = min(n_src // cn, n_nc // cn)
    if n < 1:
        return [(0, n_src, 0, n_nc)]
    return [(i * cn, (i + 1) * cn, i * cn, (i + 1) * cn) for i in range(n)]


def estimate_pitch_chroma(src_audio: np.ndarray, nc_audio: np.ndarray, sr: int,
                          log: Optional[Callable[[str], None]] = None):
    """pitch.py:100-173: per-20 s-chunk lags, median shift, seed-0 bootstrap CI, Hz lists."""
    from .engine import get_engine
    from .ops import chroma_means, chroma_lags, shift_bootstrap
    eng = get_engine()
    plan = _chunk_plan(len(src_audio), len(nc_audio), sr)
    arrays = []
    for a, b, c, d in plan:
        arrays += [src_audio[a:b], nc_audio[c:d]]
    _, _, dev_chroma = chroma_means(eng, arrays)
    n = len(plan)
    lags = chroma_lags(eng, dev_chroma, list(range(0, 2 * n, 2)), list(range(1, 2 * n, 2)))
    shift_sts = np.array([lag / 3.0 for lag in lags])
    point_st = float(np.median(shift_sts))
    if n >= MIN_CHUNKS:
        ci_lo, ci_hi = shift_bootstrap(eng, shift_sts)
    else:
        ci_lo = ci_hi = point_st
        if log:
            log(f"    Only {n} chunk(s) available (need ≥ {MIN_CHUNKS}) — "
                "pitch CI is degenerate; estimate may be less reliable.")
    src_hz: List[Optional[float]] = [_REF_HZ] * n
    nc_hz: List[Optional[float]] = [_REF_HZ * (2.0 ** (st / 12.0)) for st in shift_sts]
    if log:
        log(f"    Chroma xcorr: {point_st:+.3f} st  95% CI [{ci_lo:+.3f}, {ci_hi:+.3f}] st"
            f"  ({n} chunk{'s' if n != 1 else ''})")
    return src_hz, nc_hz, point_st, (ci_lo, ci_hi), n


def _try_import_essentia():
    try:
        import essentia.standard as es  # type: ignore[import]
        return es
    except Exception:
        return None


def estimate_pitch_melodia(src_audio, nc_audio, sr, log=None):
    """pitch.py:187-241 — requires essentia; absent here, so skipped (returns None)."""
    es = _try_import_essentia()
    if es is None:
        if log:
            log("    essentia not available — skipping MELODIA refinement")
        return None
    raise NotImplementedError("MELODIA refinement (essentia) is outside the MI355X engine (SURVEY.md §8f)")


def estimate_pitch_combined(src_audio: np.ndarray, nc_audio: np.ndarray, sr: int,
                            log: Optional[Callable[[str], None]] = None
                            ) -> Tuple[List[Optional[float]], List[Optional[float]], str]:
    src_hz, nc_hz, chroma_st, _, _ = estimate_pitch_chroma(src_audio, nc_audio, sr, log=log)
    mel = estimate_pitch_melodia(src_audio, nc_audio, sr, log=log)
    if mel is not None:
        src_m, nc_m = mel
        sm = float(np.median([v for v in src_m if v is not None]))
        nm = float(np.median([v for v in nc_m if v is not None]))
        if sm > 0 and nm > 0:
            mst = 12.0 * math.log2(nm / sm)
            if abs(mst - chroma_st) <= MELODIA_AGREE_ST:
                return src_m, nc_m, "chroma+melodia"
    return src_hz, nc_hz, "chroma_xcorr"
