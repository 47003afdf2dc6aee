"""Known-answer tests of the librosa restatement (oracle/ncref.py) from first
principles — the only pinning available for librosa arithmetic, which is absent
from this image ("parity unpinned" against real librosa)."""
import numpy as np
import pytest
import scipy.signal

from oracle import ncref, refglue
from nightcore_analyzer import synth

SR = 22050


def _clicks(n, period, amp=0.5):
    y = np.zeros(n, np.float32)
    t = np.arange(600) / SR
    burst = (amp * np.exp(-t / 0.005) * np.sin(2 * np.pi * 1500 * t)).astype(np.float32)
    for b in range(0, n - 600, period):
        y[b:b + 600] += burst
    return y


@pytest.mark.parametrize("lag", [17, 21, 25])
def test_click_track_tempo_lag(lag):
    """Clicks every lag*512 samples -> tempogram argmax at that lag -> 2583.984375/lag BPM."""
    y = _clicks(220500, lag * 512) + np.random.default_rng(0).standard_normal(220500).astype(np.float32) * 1e-3
    o = ncref.onset_strength(y, SR, 512)
    bpm, L = ncref.tempo_from_tg(ncref.tempogram_mean(o, 344), SR, 512, 60 * SR / (512 * lag))
    assert L == lag and bpm == 60.0 * SR / (512.0 * lag)


def test_beats_are_evenly_spaced_on_a_click_track():
    y = _clicks(220500, 21 * 512) + np.random.default_rng(1).standard_normal(220500).astype(np.float32) * 1e-3
    o = ncref.onset_strength(y, SR, 512)
    bpm, beats = ncref.beat_track(o, SR, 512, 120.0)
    d = np.diff(beats)
    assert len(beats) >= 15 and set(d.tolist()) <= {20, 21, 22} and np.median(d) == 21


@pytest.mark.parametrize("k", [0, 2, 4, -3])
def test_chroma_lag_of_transposed_chords(k):
    # pitch-shift by an exact number of semitones via resampling the chord part only
    up = 2 ** (k / 12.0)
    t = np.arange(441000) / SR
    rng = np.random.default_rng(3)
    notes = [57, 60, 64]
    src = sum(np.sin(2 * np.pi * 440 * 2 ** ((m - 69) / 12) * t + rng.random()) for m in notes).astype(np.float32) * 0.1
    nc = sum(np.sin(2 * np.pi * 440 * 2 ** ((m - 69) / 12) * up * t + rng.random()) for m in notes).astype(np.float32) * 0.1
    assert refglue.chunk_lag(src, nc) == (k if k <= 6 else k - 12)


def test_trim_boundaries_of_padded_tone():
    t = np.arange(3 * SR) / SR
    tone = (0.3 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    y = np.concatenate([np.zeros(20480, np.float32), tone, np.zeros(30000, np.float32)])
    _, (s, e) = ncref.trim(y, 60)
    # first/last frames whose centred 2048-sample window overlaps the tone (t=39, t=171)
    assert (s, e) == (39 * 512, 172 * 512)


def test_ibi_period_exact_frames():
    y = _clicks(30 * SR, 168 * 64) + np.random.default_rng(2).standard_normal(30 * SR).astype(np.float32) * 1e-3
    ibis = refglue.estimate_ibis_global(y, SR)
    assert ibis is not None and abs(np.median(ibis) * SR / 64 - 168) < 1e-9


def test_halfband_decimator_response():
    h = ncref.halfband_taps()
    assert len(h) == 47 and abs(h.sum() - 1.0) < 1e-15
    n = np.arange(-23, 24)
    assert np.all(h[(n % 2 == 0) & (n != 0)] == 0.0)
    w, H = scipy.signal.freqz(h, worN=8192, fs=1.0)
    assert np.max(np.abs(np.abs(H[w <= 0.11]) - 1.0)) < 1e-4
    assert np.max(20 * np.log10(np.maximum(np.abs(H[w >= 0.33]), 1e-300))) < -100.0


def test_mel_filterbank_slaney_properties():
    W = ncref.mel_filter(22050, 2048, 128)
    assert W.shape == (128, 1025) and W.dtype == np.float32
    # each FFT bin contributes to at most two adjacent bands; every band is non-empty
    assert (np.count_nonzero(W, axis=0) <= 2).all() and (np.count_nonzero(W, axis=1) > 0).all()


def _sliding_tempogram_mean(o, N):
    """The engine's tempogram algorithm (csrc/nc_slide.h) in numpy: five sliding
    f64 sums per lag instead of one FFT autocorrelation per frame."""
    T, p = len(o), N // 2
    x = np.pad(o, (p, p), mode="linear_ramp", end_values=(0, 0)).astype(np.float64)
    w2 = ncref.hann(N).astype(np.float64) ** 2
    ac0 = np.array([np.dot(w2, x[t:t + N] ** 2) for t in range(T)])
    rinv = np.where(ac0 < np.finfo(np.float64).tiny, 1.0, 1.0 / np.where(ac0 == 0, 1, ac0))
    th = 2 * np.pi / N
    k = np.arange(N)
    L = N - k
    c, s = np.cos(th * k), np.sin(th * k)
    A, B, C, D, E = 0.25 + 0.125 * c, -0.25 - 0.25 * c, 0.25 * s, 0.125 * c, -0.125 * s
    j = np.arange(N)[:, None]
    P = x[j] * x[np.minimum(j + k[None, :], len(x) - 1)] * (j < L[None, :])   # p_k[j], masked to j < L
    S0 = P.sum(0)
    Z1 = (np.exp(1j * th * j) * P).sum(0)
    Z2 = (np.exp(2j * th * j) * P).sum(0)
    e1L, e2L = np.exp(-1j * th * k), np.exp(-2j * th * k)
    acc = np.zeros(N)
    for t in range(T):
        ac = A * S0 + B * Z1.real + C * Z1.imag + D * Z2.real + E * Z2.imag
        acc += ac * rinv[t]
        pt = x[t] * x[t + k]
        pl = x[t + L] * x[t + N]
        S0 = S0 - pt + pl
        Z1 = np.exp(-1j * th) * (Z1 - pt + e1L * pl)
        Z2 = np.exp(-2j * th) * (Z2 - pt + e2L * pl)
    return acc / T


@pytest.mark.parametrize("seed", [0, 1])
def test_sliding_tempogram_identity_matches_fft_autocorrelation(seed):
    """w[j]w[j+k] is a degree-2 trigonometric polynomial in j, so the Hann-windowed
    autocorrelation slides in O(1) per frame; agreement is at f64 rounding level."""
    rng = np.random.default_rng(seed)
    o = (rng.random(431) * (rng.random(431) > 0.6)).astype(np.float32)
    ref = ncref.tempogram_mean(o, 344)
    got = _sliding_tempogram_mean(o, 344)
    assert np.max(np.abs(got - ref)) < 1e-12


def _correlation_tempogram_mean(o, N):
    """The engine's window tempogram (csrc/nc_tgcorr.h) in numpy: prefix sums of the frame
    normalisers, six sequences, and per lag three Hankel minus three Toeplitz correlations
    weighted by (1, cos theta k, sin theta k)."""
    T, p = len(o), N // 2
    x = np.pad(o, (p, p), mode="linear_ramp", end_values=(0, 0)).astype(np.float64)
    U = T + N
    x = np.concatenate([x, np.zeros(U - len(x))])
    w2 = ncref.hann(N).astype(np.float64) ** 2
    ac0 = np.array([np.dot(w2, x[t:t + N] ** 2) for t in range(T)])
    r = np.where(ac0 < np.finfo(np.float64).tiny, 1.0, 1.0 / np.where(ac0 == 0, 1, ac0))
    th = 2 * np.pi / N
    t = np.arange(T)
    Q = [np.concatenate([[0.0], np.cumsum(r * f)])
         for f in (np.ones(T), np.cos(th * t), np.sin(th * t), np.cos(2 * th * t), np.sin(2 * th * t))]
    u = np.arange(U)
    cu, su, c2u, s2u = np.cos(th * u), np.sin(th * u), np.cos(2 * th * u), np.sin(2 * th * u)

    def g(at):
        P0, Qc1, Qs1, Qc2, Qs2 = (q[at] for q in Q)
        P1, P2 = cu * Qc1 + su * Qs1, su * Qc1 - cu * Qs1
        P3, P4 = c2u * Qc2 + s2u * Qs2, s2u * Qc2 - c2u * Qs2
        return [(P0 - P1) / 4, P0 / 8 - P1 / 4 + P3 / 8, P2 / 4 - P4 / 8]

    a = [x * v for v in g(np.minimum(T - 1, u) + 1)]
    b = [x * v for v in g(np.maximum(0, u - N + 1))]
    b[2] = -b[2]
    out = np.zeros(N)
    for k in range(N):
        n = U - k
        d = [np.dot(a[i][:n], x[k:]) - np.dot(b[i][k:], x[:n]) for i in range(3)]
        out[k] = d[0] + np.cos(th * k) * d[1] + np.sin(th * k) * d[2]
    return out / T


@pytest.mark.parametrize("quiet", [None, 1e-3, 1e-6])
@pytest.mark.parametrize("seed", [0, 1])
def test_correlation_tempogram_identity_matches_fft_autocorrelation(seed, quiet):
    """The window kernel's six-correlation form agrees with librosa's per-frame FFT
    autocorrelation at f64 rounding level, also when a stretch of the envelope is 1e3 /
    1e6 times quieter than the rest (frame normalisers spanning 12 decades)."""
    rng = np.random.default_rng(seed)
    o = (rng.random(431) * (rng.random(431) > 0.6)).astype(np.float32)
    if quiet is not None:
        o[250:] *= np.float32(quiet)
    ref = ncref.tempogram_mean(o, 344)
    got = _correlation_tempogram_mean(o, 344)
    tol = {None: 1e-13, 1e-3: 1e-12, 1e-6: 1e-9}[quiet]
    assert np.max(np.abs(got - ref)) < tol
