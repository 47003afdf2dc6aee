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
