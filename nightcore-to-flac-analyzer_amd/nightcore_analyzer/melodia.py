"""MELODIA predominant-pitch estimation on the MI355X — OPT-IN and PARITY UNPINNED.

The reference refines its chroma pitch estimate with essentia's ``PredominantPitchMelodia``
(frameSize 2048, hopSize 128, every other parameter at essentia's default; pitch.py:187-241)
when essentia is installed, and skips the step otherwise.  essentia is not installed in this
image, so this module is a restatement of the published algorithm (Salamon & Gomez, "Melody
extraction from polyphonic music signals using pitch contour characteristics", IEEE TASLP
2012, with essentia 2.1's default parameters), not a port of essentia's code: nothing here is
checked against essentia's own output.  It runs only when asked for
(``pitch.estimate_pitch_melodia(..., backend="device")`` or ``NC_MELODIA=device``); the default
path keeps the reference's behaviour (essentia when importable, otherwise the step is skipped
with the reference's log line).

* Frame front end on the device (``nc_melodia_salience``, csrc/melodia.hip): windowed
  8192-point spectrum per 128-sample hop, the 100 largest spectral peaks, the 600-bin harmonic
  salience function, its peaks.  CPU restatement for the tests: oracle/melodia_ref.py.
* Contour creation (``pitch_contours``: PitchContours) and melody selection
  (``contours_melody``: PitchContoursMelody: voicing filter, octave-duplicate and pitch-outlier
  removal against a smoothed melody pitch mean, per-frame pick by total salience) on the host:
  sequential decisions over a few hundred contours.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

FRAME = 2048                 # frameSize (pitch.py:211)
HOP = 128                    # hopSize (pitch.py:212)
FFT = 4 * FRAME              # Windowing zeroPadding = 3 frameSize
BIN_CENTS = 10.0             # binResolution
REF_HZ = 55.0                # referenceFrequency
N_BINS = 600                 # 6000 cents / binResolution
MIN_HZ, MAX_HZ = 80.0, 20000.0
PEAK_FRAME_THRESHOLD = 0.9
PEAK_DISTRIBUTION_THRESHOLD = 0.9
PITCH_CONTINUITY = 27.5625   # cents per millisecond
TIME_CONTINUITY = 100.0      # ms
MIN_DURATION = 100.0         # ms
VOICING_TOLERANCE = 0.2
FILTER_ITERATIONS = 3
SALPK = 128                  # salience peaks kept per frame (NC_MELODIA_SALPK)


def window(n: int = FRAME) -> np.ndarray:
    """essentia's Windowing "hann" (symmetric, 0.5 - 0.5 cos(2 pi i / (n - 1))), normalised to
    an area of 1 and scaled by 2, in f64 -> f32."""
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / (n - 1))
    return (2.0 * w / w.sum()).astype(np.float32)


def n_frames(length: int, hop: int = HOP) -> int:
    """Frames of FrameCutter(startFromZero=False): centred at t hop while t hop - FRAME/2 < length."""
    return -(-(int(length) + FRAME // 2) // hop)


def cent_bin(hz: float) -> int:
    return int(np.floor(1200.0 / BIN_CENTS * np.log2(hz / REF_HZ) + 0.5))


@dataclass
class SaliencePeaks:
    """Per-frame salience peaks of one file: counts [T], bins [T, SALPK], saliences [T, SALPK]
    (row t's first counts[t] entries, by salience descending)."""
    counts: np.ndarray
    bins: np.ndarray
    sal: np.ndarray

    def frame(self, t: int) -> Tuple[np.ndarray, np.ndarray]:
        n = int(self.counts[t])
        return self.bins[t, :n].astype(np.float64), self.sal[t, :n].astype(np.float64)


def salience_peaks(eng, arrays: Sequence[np.ndarray], sr: int = 22050, hop: int = HOP) -> List[SaliencePeaks]:
    """nc_melodia_salience over every file of ``arrays`` (host float32) in one launch."""
    import torch
    from .engine import _Upload
    sig = eng.upload_signals([np.asarray(a, np.float32) for a in arrays])
    T = np.array([n_frames(n, hop) for n in sig.length], np.int64)
    fb = np.concatenate([[0], np.cumsum(T)]).astype(np.int64)
    total = int(fb[-1])
    up = _Upload()
    up.add("off", sig.off, np.int64)
    up.add("len", sig.length, np.int64)
    up.add("fb", fb, np.int64)
    d = up.commit(eng.dev)
    win = getattr(eng, "_melodia_win", None)
    if win is None:
        win = eng._melodia_win = torch.from_numpy(window()).to(eng.dev)
    cnt = torch.zeros(max(1, total), dtype=torch.int32, device=eng.dev)
    bins = torch.zeros((max(1, total), SALPK), dtype=torch.int32, device=eng.dev)
    sal = torch.zeros((max(1, total), SALPK), dtype=torch.float32, device=eng.dev)
    eng.call("nc_melodia_salience", sig.buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(), d["fb"].data_ptr(),
             len(T), total, hop, float(sr), win.data_ptr(), max(0, cent_bin(MIN_HZ)), cnt.data_ptr(), bins.data_ptr(),
             sal.data_ptr(), eng.stream())
    c, b, s = cnt.cpu().numpy(), bins.cpu().numpy(), sal.cpu().numpy()
    return [SaliencePeaks(c[fb[i]:fb[i + 1]], b[fb[i]:fb[i + 1]], s[fb[i]:fb[i + 1]]) for i in range(len(T))]


# ------------------------------------------------------------------------------ contours
@dataclass
class Contour:
    start: int                 # first frame
    bins: np.ndarray           # salience bin per frame (float)
    sal: np.ndarray            # salience per frame

    @property
    def end(self) -> int:
        return self.start + len(self.bins)


def pitch_contours(peaks: SaliencePeaks, sr: int = 22050, hop: int = HOP) -> List[Contour]:
    """PitchContours: (1) per frame, peaks below PEAK_FRAME_THRESHOLD x the frame's largest are
    non-salient; (2) salient peaks below mean - PEAK_DISTRIBUTION_THRESHOLD x std (over all salient
    peaks) become non-salient; (3) repeatedly the largest remaining salient peak starts a contour,
    tracked forward and backward frame by frame to the nearest peak within the pitch continuity
    (salient first, else non-salient, a run of at most the time continuity in non-salient peaks,
    trailing non-salient peaks dropped); contours shorter than the minimum duration are discarded.
    Every peak joins at most one contour."""
    fd = hop / sr
    cont_bins = PITCH_CONTINUITY * 1000.0 * fd / BIN_CENTS
    gap_max = (TIME_CONTINUITY / 1000.0) / fd
    min_len = (MIN_DURATION / 1000.0) / fd
    T = len(peaks.counts)
    # per frame: arrays of bins, saliences and a state (1 salient, 2 non-salient, 0 used)
    fb, fs, st = [], [], []
    for t in range(T):
        b, s = peaks.frame(t)
        state = np.full(len(b), 1, np.int8)
        if len(s):
            state[s < PEAK_FRAME_THRESHOLD * s.max()] = 2
        fb.append(b)
        fs.append(s)
        st.append(state)
    sal_all = np.concatenate([s[x == 1] for s, x in zip(fs, st)]) if T else np.zeros(0)
    if len(sal_all):
        thr = sal_all.mean() - PEAK_DISTRIBUTION_THRESHOLD * sal_all.std()
        for s, x in zip(fs, st):
            x[(x == 1) & (s < thr)] = 2
    # salient peaks in one array, visited largest first
    cand = [(t, j) for t in range(T) for j in np.flatnonzero(st[t] == 1)]
    order = sorted(cand, key=lambda tj: (-fs[tj[0]][tj[1]], tj[0], fb[tj[0]][tj[1]]))

    def nearest(t, last, state):
        x = st[t]
        m = x == state
        if not m.any():
            return -1
        d = np.abs(fb[t] - last)
        d = np.where(m & (d <= cont_bins), d, np.inf)
        j = int(np.argmin(d))
        return j if np.isfinite(d[j]) else -1

    def track(t0, last, step):
        got, gap = [], 0
        t = t0 + step
        while 0 <= t < T:
            j = nearest(t, last, 1)
            if j >= 0:
                gap = 0
            else:
                j = nearest(t, last, 2)
                if j < 0:
                    break
                gap += 1
                if gap > gap_max:
                    break
            got.append((t, j, gap > 0))
            st[t][j] = 0
            last = fb[t][j]
            t += step
        while got and got[-1][2]:      # trailing non-salient peaks leave the contour (and the pool)
            got.pop()
        return got

    contours = []
    for t, j in order:
        if st[t][j] != 1:
            continue
        st[t][j] = 0
        fwd = track(t, fb[t][j], 1)
        bwd = track(t, fb[t][j], -1)
        pts = [(tt, jj) for tt, jj, _ in reversed(bwd)] + [(t, j)] + [(tt, jj) for tt, jj, _ in fwd]
        if len(pts) >= min_len:
            contours.append(Contour(pts[0][0], np.array([fb[tt][jj] for tt, jj in pts]),
                                    np.array([fs[tt][jj] for tt, jj in pts])))
    contours.sort(key=lambda c: (c.start, c.bins[0]))
    return contours


def _melody_pitch_mean(contours: Sequence[Contour], T: int, smooth: int) -> np.ndarray:
    """Salience-weighted mean contour bin per frame, gaps filled linearly (edges held), then a
    centred moving average over ``smooth`` frames (the 5 s melody pitch mean)."""
    num = np.zeros(T)
    den = np.zeros(T)
    for c in contours:
        num[c.start:c.end] += c.bins * c.sal
        den[c.start:c.end] += c.sal
    have = den > 0
    if not have.any():
        return np.zeros(T)
    m = np.zeros(T)
    m[have] = num[have] / den[have]
    idx = np.arange(T)
    m = np.interp(idx, idx[have], m[have])
    k = max(1, int(smooth))
    c = np.cumsum(np.concatenate([[0.0], m]))
    lo = np.clip(idx - k // 2, 0, T)
    hi = np.clip(idx + k // 2 + 1, 0, T)
    return (c[hi] - c[lo]) / (hi - lo)


def contours_melody(contours: Sequence[Contour], T: int, sr: int = 22050, hop: int = HOP) -> np.ndarray:
    """PitchContoursMelody -> pitch (Hz) per frame, 0 where unvoiced (guessUnvoiced False):
    voicing (contours whose mean salience is below mean - VOICING_TOLERANCE x std of the
    contours' mean saliences are dropped), then FILTER_ITERATIONS rounds of octave-duplicate
    removal (of two overlapping contours 1150-1250 cents apart, the one further from the melody
    pitch mean goes) and pitch-outlier removal (contours more than 1250 cents from the melody
    pitch mean go), the mean recomputed after each; finally per frame the present contour with
    the largest total salience, its bin as Hz, within [MIN_HZ, MAX_HZ]."""
    pitch = np.zeros(T)
    if not contours:
        return pitch
    fd = hop / sr
    means = np.array([c.sal.mean() for c in contours])
    thr = means.mean() - VOICING_TOLERANCE * means.std()
    sel = [c for c, m in zip(contours, means) if m >= thr]
    smooth = int(round(5.0 / fd))
    dup_lo, dup_hi = 1150.0 / BIN_CENTS, 1250.0 / BIN_CENTS
    outlier = 1250.0 / BIN_CENTS
    mpm = _melody_pitch_mean(sel, T, smooth)
    for _ in range(FILTER_ITERATIONS):
        drop = set()
        for a in range(len(sel)):
            for b in range(a + 1, len(sel)):
                ca, cb = sel[a], sel[b]
                lo, hi = max(ca.start, cb.start), min(ca.end, cb.end)
                if hi <= lo or a in drop or b in drop:
                    continue
                pa = ca.bins[lo - ca.start:hi - ca.start]
                pb = cb.bins[lo - cb.start:hi - cb.start]
                if dup_lo < abs(pa.mean() - pb.mean()) < dup_hi:
                    ref = mpm[lo:hi].mean()
                    drop.add(a if abs(pa.mean() - ref) > abs(pb.mean() - ref) else b)
        sel = [c for i, c in enumerate(sel) if i not in drop]
        mpm = _melody_pitch_mean(sel, T, smooth)
        sel = [c for c in sel if abs(c.bins.mean() - mpm[c.start:c.end].mean()) <= outlier]
        mpm = _melody_pitch_mean(sel, T, smooth)
    best = np.full(T, -np.inf)
    for c in sel:
        tot = c.sal.sum()
        seg = slice(c.start, c.end)
        better = tot > best[seg]
        best[seg] = np.where(better, tot, best[seg])
        hz = REF_HZ * 2.0 ** (c.bins * BIN_CENTS / 1200.0)
        pitch[seg] = np.where(better, hz, pitch[seg])
    pitch[(pitch < MIN_HZ) | (pitch > MAX_HZ)] = 0.0
    return pitch


def melody_from_peaks(peaks: SaliencePeaks, sr: int = 22050, hop: int = HOP) -> np.ndarray:
    return contours_melody(pitch_contours(peaks, sr, hop), len(peaks.counts), sr, hop)


def predominant_pitch_melodia(audios: Sequence[np.ndarray], sr: int = 22050, eng=None) -> List[np.ndarray]:
    """Pitch (Hz per 128-sample frame, 0 = unvoiced) of every signal, the front end of all of
    them in one device launch."""
    from .engine import get_engine
    eng = eng or get_engine()
    return [melody_from_peaks(p, sr) for p in salience_peaks(eng, audios, sr)]
