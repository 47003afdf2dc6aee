"""CPU restatement of the MELODIA frame front end (test infrastructure only: imported by tests/,
never by the product path).  PARITY UNPINNED: it restates the published algorithm (Salamon &
Gomez 2012) with essentia 2.1's default PredominantPitchMelodia parameters as the reference calls
it (pitch.py:210-215: frameSize 2048, hopSize 128), but essentia itself is not installed here, so
no essentia output pins it.  It is the checker of csrc/melodia.hip (nc_melodia_salience): f64
spectra and salience, the same decisions.

Per frame t (FrameCutter startFromZero=False: samples [t hop - 1024, t hop + 1024), zeros
outside the signal):
  Windowing("hann", normalized, zeroPadding 3 frameSize) -> Spectrum (|rfft| of 8192 points)
  -> SpectralPeaks (local maxima in bins 1..4095, parabolic interpolation, 100 largest)
  -> PitchSalienceFunction (600 bins of 10 cents from 55 Hz, 20 harmonics, 0.8^h, cos^2 within
     one semitone, peaks within 40 dB of the largest)
  -> PitchSalienceFunctionPeaks (local maxima in [bin(80 Hz), 599], salience > 0)."""
from __future__ import annotations

import numpy as np

FRAME, HOP, FFT = 2048, 128, 8192
N_BINS, SEMI, NH = 600, 10, 20


def window(n: int = FRAME) -> np.ndarray:
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / (n - 1))
    return (2.0 * w / w.sum()).astype(np.float32)


def n_frames(length: int, hop: int = HOP) -> int:
    return -(-(int(length) + FRAME // 2) // hop)


def frame_mag(y: np.ndarray, t: int, hop: int = HOP, win=None) -> np.ndarray:
    win = window() if win is None else win
    s0 = t * hop - FRAME // 2
    fr = np.zeros(FRAME, np.float64)
    a, b = max(0, s0), min(len(y), s0 + FRAME)
    if b > a:
        fr[a - s0:b - s0] = y[a:b]
    return np.abs(np.fft.rfft(fr * win.astype(np.float64), FFT))


def spectral_peaks(mag: np.ndarray, sr: float, max_peaks: int = 100):
    l, c, r = mag[:-2], mag[1:-1], mag[2:]
    k = np.flatnonzero((c > l) & (c >= r) & (c > 0)) + 1
    L, C, R = mag[k - 1], mag[k], mag[k + 1]
    pos = k + 0.5 * (L - R) / (L - 2 * C + R)
    val = C - 0.25 * (L - R) * (pos - k)
    order = np.lexsort((k, -val))[:max_peaks]
    return pos[order] * sr / FFT, val[order]


def cent_bin(f):
    return np.floor(120.0 * np.log2(np.asarray(f, np.float64) / 55.0) + 0.5).astype(np.int64)


def salience(freqs: np.ndarray, mags: np.ndarray) -> np.ndarray:
    sal = np.zeros(N_BINS)
    if len(mags) == 0:
        return sal
    amin = mags.max() * 0.01
    nbw = np.cos(np.arange(SEMI + 1) / SEMI * np.pi / 2) ** 2
    for f, a in zip(freqs, mags):
        if a <= amin:
            continue
        for h in range(NH):
            hb = int(cent_bin(f / (h + 1)))
            if hb < 0:
                break
            lo, hi = max(0, hb - SEMI), min(N_BINS - 1, hb + SEMI)
            for b in range(lo, hi + 1):
                sal[b] += a * 0.8 ** h * nbw[abs(b - hb)]
    return sal


def salience_peaks(sal: np.ndarray, min_bin: int, max_out: int = 128):
    b = np.arange(max(min_bin, 0), N_BINS)
    c = sal[b]
    left = np.where(b > 0, sal[np.maximum(b - 1, 0)], -np.inf)
    right = np.where(b + 1 < N_BINS, sal[np.minimum(b + 1, N_BINS - 1)], -np.inf)
    m = (c > left) & (c >= right) & (c > 0)
    bb, cc = b[m], c[m]
    order = np.lexsort((bb, -cc))[:max_out]
    return bb[order], cc[order]


def frame_salience_peaks(y: np.ndarray, t: int, sr: float = 22050.0, hop: int = HOP):
    """(bins, saliences) of frame t, ordered by salience (descending), ties by bin."""
    mag = frame_mag(y, t, hop)
    f, a = spectral_peaks(mag, sr)
    return salience_peaks(salience(f, a), int(cent_bin(80.0)))


# ------------------------------------------------------------------------------ contours + melody
# The host stage of MELODIA, restated for the tests from the published algorithm (Salamon &
# Gomez 2012, sections II-C and II-D) with essentia 2.1's default PitchContours /
# PitchContoursMelody parameters.  PARITY UNPINNED like the front end: essentia is absent.  It is
# written independently of nightcore_analyzer/melodia.py (plain per-frame lists and explicit
# scans, no vectorised shortcuts) so that an indexing, pool or tie-breaking slip in either one
# shows up as a difference.  Choices the paper leaves open, taken the same way in both (and
# named here so a reader can check them against essentia when it is available):
#   * pitch continuity 27.5625 cents/ms x 1000 x hop / sr / 10 cents = 16 bins at 22 050 Hz, a
#     peak continues a contour when |bin - last bin| <= 16; the nearest such peak wins, ties to the
#     earlier peak of the frame (frames list peaks by salience, descending);
#   * a run of non-salient peaks longer than the time continuity (100 ms) ends the contour before
#     the peak that would exceed it (that peak stays in the pool); the contour's trailing
#     non-salient peaks are dropped from it but stay used;
#   * minimum duration 100 ms: a contour needs at least ceil(100 ms / frame) frames;
#   * seeds: the largest remaining salient peak, ties to the earlier frame, then the lower bin;
#   * voicing: contours whose mean salience is below mean - 0.2 std (population std) of the
#     contours' mean saliences are unvoiced;
#   * melody pitch mean: per frame the salience-weighted mean bin of the present contours, gaps
#     interpolated linearly (ends held), a centred 5 s moving average (shortened at the ends);
#   * octave duplicates: two overlapping contours whose mean bins over the overlap are 1150-1250
#     cents apart; the one farther (over the overlap) from the melody pitch mean goes;
#   * pitch outliers: contours whose mean bin is more than 1250 cents from the melody pitch mean
#     over their frames go; three iterations, the mean recomputed after each removal step;
#   * output: per frame the present contour with the largest total salience (ties to the earlier
#     contour in (start, first bin) order), 55 Hz x 2^(bin / 120), 0 outside [80, 20000] Hz.
PITCH_CONT_CENTS_PER_MS = 27.5625
TIME_CONT_MS = 100.0
MIN_DUR_MS = 100.0
FRAME_THR = 0.9
DIST_THR = 0.9
VOICING_TOL = 0.2
ITERATIONS = 3


def contours_ref(frames, sr: float = 22050.0, hop: int = HOP):
    """frames[t] = (bins, saliences) of frame t (salience descending) -> list of contours
    (start frame, [bins], [saliences]), sorted by (start, first bin)."""
    fd = hop / sr
    cont = PITCH_CONT_CENTS_PER_MS * 1000.0 * fd / 10.0
    max_gap = TIME_CONT_MS / 1000.0 / fd
    min_frames = MIN_DUR_MS / 1000.0 / fd
    T = len(frames)
    # pool[t] = list of [bin, salience, state]: state 1 salient, 2 non-salient, 0 used
    pool = []
    for bins, sals in frames:
        row = [[float(b), float(s), 1] for b, s in zip(bins, sals)]
        top = max((r[1] for r in row), default=0.0)
        for r in row:
            if r[1] < FRAME_THR * top:
                r[2] = 2
        pool.append(row)
    sal_vals = [r[1] for row in pool for r in row if r[2] == 1]
    if sal_vals:
        mu = sum(sal_vals) / len(sal_vals)
        sd = (sum((v - mu) ** 2 for v in sal_vals) / len(sal_vals)) ** 0.5
        for row in pool:
            for r in row:
                if r[2] == 1 and r[1] < mu - DIST_THR * sd:
                    r[2] = 2

    def pick(t, last, state):
        best, bd = None, None
        for r in pool[t]:
            if r[2] != state:
                continue
            d = abs(r[0] - last)
            if d <= cont and (bd is None or d < bd):
                best, bd = r, d
        return best

    def walk(t0, last, step):
        out, run = [], 0
        t = t0 + step
        while 0 <= t < T:
            r = pick(t, last, 1)
            if r is not None:
                run = 0
            else:
                r = pick(t, last, 2)
                if r is None:
                    break
                run += 1
                if run > max_gap:
                    break
            r[2] = 0
            out.append((t, r, run > 0))
            last = r[0]
            t += step
        while out and out[-1][2]:
            out.pop()
        return out

    result = []
    while True:
        seed, st = None, None
        for t in range(T):
            for r in pool[t]:
                if r[2] == 1 and (seed is None or r[1] > seed[1] or (r[1] == seed[1] and (t, r[0]) < (st, seed[0]))):
                    seed, st = r, t
        if seed is None:
            break
        seed[2] = 0
        fwd = walk(st, seed[0], 1)
        bwd = walk(st, seed[0], -1)
        pts = [(t, r) for t, r, _ in reversed(bwd)] + [(st, seed)] + [(t, r) for t, r, _ in fwd]
        if len(pts) >= min_frames:
            result.append((pts[0][0], [r[0] for _, r in pts], [r[1] for _, r in pts]))
    result.sort(key=lambda c: (c[0], c[1][0]))
    return result


def _pitch_mean_ref(contours, T, smooth):
    num, den = [0.0] * T, [0.0] * T
    for start, bins, sals in contours:
        for i, (b, s) in enumerate(zip(bins, sals)):
            num[start + i] += b * s
            den[start + i] += s
    known = [t for t in range(T) if den[t] > 0]
    if not known:
        return [0.0] * T
    m = [0.0] * T
    for t in known:
        m[t] = num[t] / den[t]
    # linear interpolation over the gaps, ends held
    for t in range(T):
        if den[t] > 0:
            continue
        prev = max((k for k in known if k < t), default=None)
        nxt = min((k for k in known if k > t), default=None)
        if prev is None:
            m[t] = m[nxt]
        elif nxt is None:
            m[t] = m[prev]
        else:
            m[t] = m[prev] + (m[nxt] - m[prev]) * (t - prev) / (nxt - prev)
    half = max(1, int(smooth)) // 2
    out = []
    for t in range(T):
        lo, hi = max(0, t - half), min(T, t + half + 1)
        out.append(sum(m[lo:hi]) / (hi - lo))
    return out


def melody_ref(contours, T, sr: float = 22050.0, hop: int = HOP):
    """Pitch (Hz) per frame from contours_ref's contours (0 = unvoiced)."""
    pitch = [0.0] * T
    if not contours:
        return np.array(pitch)
    fd = hop / sr
    means = [sum(s) / len(s) for _, _, s in contours]
    mu = sum(means) / len(means)
    sd = (sum((v - mu) ** 2 for v in means) / len(means)) ** 0.5
    sel = [c for c, v in zip(contours, means) if v >= mu - VOICING_TOL * sd]
    smooth = int(round(5.0 / fd))
    mpm = _pitch_mean_ref(sel, T, smooth)

    def overlap_mean(c, lo, hi):
        start, bins, _ = c
        seg = bins[lo - start:hi - start]
        return sum(seg) / len(seg)

    for _ in range(ITERATIONS):
        gone = set()
        for i in range(len(sel)):
            for j in range(i + 1, len(sel)):
                if i in gone or j in gone:
                    continue
                a, b = sel[i], sel[j]
                lo, hi = max(a[0], b[0]), min(a[0] + len(a[1]), b[0] + len(b[1]))
                if hi <= lo:
                    continue
                ma, mb = overlap_mean(a, lo, hi), overlap_mean(b, lo, hi)
                if 115.0 < abs(ma - mb) < 125.0:
                    ref = sum(mpm[lo:hi]) / (hi - lo)
                    gone.add(i if abs(ma - ref) > abs(mb - ref) else j)
        sel = [c for k, c in enumerate(sel) if k not in gone]
        mpm = _pitch_mean_ref(sel, T, smooth)
        keep = []
        for c in sel:
            start, bins, _ = c
            ref = sum(mpm[start:start + len(bins)]) / len(bins)
            if abs(sum(bins) / len(bins) - ref) <= 125.0:
                keep.append(c)
        sel = keep
        mpm = _pitch_mean_ref(sel, T, smooth)
    best = [None] * T
    for start, bins, sals in sel:
        tot = sum(sals)
        for i, b in enumerate(bins):
            t = start + i
            if best[t] is None or tot > best[t]:
                best[t] = tot
                hz = 55.0 * 2.0 ** (b * 10.0 / 1200.0)
                pitch[t] = hz if 80.0 <= hz <= 20000.0 else 0.0
    return np.array(pitch)


def predominant_pitch_ref(y: np.ndarray, sr: float = 22050.0, hop: int = HOP):
    """The whole oracle: front end of every frame, contours, melody (Hz per frame)."""
    T = n_frames(len(y), hop)
    frames = [frame_salience_peaks(y, t, sr, hop) for t in range(T)]
    return melody_ref(contours_ref(frames, sr, hop), T, sr, hop)
