"""Pitch-shift detection by chromagram cross-correlation
(drop-in for the reference's nightcore_analyzer/pitch.py), on the MI355X.

Faithful to the reference including its 1/3 quirk:
``chroma_cqt(bins_per_octave=36)`` keeps librosa's default n_chroma = 12, so
the 12-lag cyclic cross-correlation finds whole-semitone lags and
``_chroma_shift_for_chunk`` divides by 3.0 — reported shifts are one third of
the true semitone shift.  MELODIA refinement needs essentia, which is not
installed; as in the reference (pitch.py:178-201) it is then skipped, unless the
opt-in device restatement is asked for (``backend="device"`` or NC_MELODIA=device:
nightcore_analyzer/melodia.py, parity unpinned).
"""
from __future__ import annotations

import math
import os
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
    from .tempo import require_rate
    require_rate(sr, "_mean_chroma")
    return chroma_means(get_engine(), [audio])[0][0]


def _cyclic_xcorr_peak(src_chroma: np.ndarray, nc_chroma: np.ndarray) -> int:
    """Wrapped argmax_k dot(src, roll(nc, -k)) (pitch.py:67-85) for vectors of any length,
    on the device (nc_xcorr_peak)."""
    from .engine import get_engine
    from .ops import xcorr_peaks
    a, b = np.asarray(src_chroma), np.asarray(nc_chroma)
    if a.ndim != 1 or a.shape != b.shape:
        raise ValueError(f"_cyclic_xcorr_peak: vectors of equal length expected, got {a.shape} and {b.shape}")
    return xcorr_peaks(get_engine(), a[None, :], b[None, :])[0]


def _chroma_shift_for_chunk(src_chunk: np.ndarray, nc_chunk: np.ndarray, sr: int) -> float:
    from .engine import get_engine
    from .ops import chroma_means, chroma_lags
    from .tempo import require_rate
    require_rate(sr, "_chroma_shift_for_chunk")
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
    from .tempo import require_rate
    require_rate(sr, "estimate_pitch_chroma")
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


def melodia_backend(backend: Optional[str] = None) -> Optional[str]:
    """Which MELODIA runs: "essentia" (the reference's), "device" (opt-in restatement on the
    MI355X, parity unpinned) or None (skipped, the reference's behaviour without essentia).
    ``backend`` (or NC_MELODIA when None) = "device" opts in; anything else keeps the default."""
    choice = backend if backend is not None else os.environ.get("NC_MELODIA", "")
    if choice == "device":
        return "device"
    return "essentia" if _try_import_essentia() is not None else None


def estimate_pitch_melodia(src_audio, nc_audio, sr, log=None, backend: Optional[str] = None):
    """pitch.py:187-241: PredominantPitchMelodia (frame 2048, hop 128) on both signals -> voiced
    F0 lists (Hz), each thinned to at most MAX_MELODIA_FRAMES by a fixed stride; None when the
    step is skipped, when extraction fails or when a side has no voiced frame.  By default this
    is essentia's own CPU algorithm where essentia is installed, and skipped otherwise (the
    reference's behaviour; essentia is not in this image).  ``backend="device"`` (or
    NC_MELODIA=device) runs the opt-in restatement instead: the frame front end on the MI355X,
    contours and melody selection on the host (melodia.py; parity unpinned: no essentia output
    exists here to check it against)."""
    which = melodia_backend(backend)
    if which is None:
        if log:
            log("    essentia not available — skipping MELODIA refinement")
        return None
    es = _try_import_essentia() if which == "essentia" else None

    def extract(audio):
        if which == "device":
            from .melodia import predominant_pitch_melodia
            from .tempo import require_rate
            require_rate(sr, "estimate_pitch_melodia")
            return predominant_pitch_melodia([audio], sr)[0]
        f0, _ = es.PredominantPitchMelodia(frameSize=2048, hopSize=128, sampleRate=float(sr))(
            np.asarray(audio, dtype=np.float32))
        return f0

    def voiced_f0(audio):
        try:
            f0 = np.asarray(extract(audio))
            v = f0[f0 > 0.0]
            if v.size == 0:
                return None
            if v.size > MAX_MELODIA_FRAMES:
                v = v[::v.size // MAX_MELODIA_FRAMES]
            return v
        except Exception as exc:           # noqa: BLE001 - reported, never raised (pitch.py:223-226)
            from ._native import NativeUnavailable
            if isinstance(exc, NativeUnavailable):
                raise                      # the device backend without its library fails loudly
            if log:
                log(f"    MELODIA extraction failed: {exc}")
            return None

    vs = voiced_f0(src_audio)
    vn = voiced_f0(nc_audio)
    if vs is None or vn is None:
        return None
    if log:
        st = 12.0 * math.log2(float(np.median(vn)) / float(np.median(vs)))
        log(f"    MELODIA: {st:+.6f} st  ({len(vs)} src / {len(vn)} nc voiced frames)")
    return [float(v) for v in vs], [float(v) for v in vn]


def melodia_choice(mel, chroma_st: float, log: Optional[Callable[[str], None]] = None):
    """estimate_pitch_combined's acceptance rule (pitch.py:272-291): the MELODIA lists when
    their median shift is within MELODIA_AGREE_ST of the chroma shift, else None (logged)."""
    if mel is None:
        return None
    src_m, nc_m = mel
    sm = float(np.median([v for v in src_m if v is not None]))
    nm = float(np.median([v for v in nc_m if v is not None]))
    if sm > 0 and nm > 0:
        mst = 12.0 * math.log2(nm / sm)
        if abs(mst - chroma_st) <= MELODIA_AGREE_ST:
            return src_m, nc_m
        if log:
            log(f"    MELODIA ({mst:+.3f} st) disagrees with chroma ({chroma_st:+.3f} st) by "
                f"{abs(mst - chroma_st):.2f} st > {MELODIA_AGREE_ST} st threshold — using chroma only")
    return None


def estimate_pitch_combined(src_audio: np.ndarray, nc_audio: np.ndarray, sr: int,
                            log: Optional[Callable[[str], None]] = None, backend: Optional[str] = None
                            ) -> Tuple[List[Optional[float]], List[Optional[float]], str]:
    src_hz, nc_hz, chroma_st, _, _ = estimate_pitch_chroma(src_audio, nc_audio, sr, log=log)
    pick = melodia_choice(estimate_pitch_melodia(src_audio, nc_audio, sr, log=log, backend=backend), chroma_st, log)
    if pick is not None:
        return pick[0], pick[1], "chroma+melodia"
    return src_hz, nc_hz, "chroma_xcorr"
