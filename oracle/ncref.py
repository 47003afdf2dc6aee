"""TEST INFRASTRUCTURE ONLY — numpy/scipy restatement of the librosa primitives
that the reference's hot path calls.

librosa is a third-party dependency of the reference (``requirements.txt:22``:
``librosa>=0.10.1``, no exact pin) that is absent from ``/root/reference`` and
from this image.  The semantics restated here are those of librosa **0.11.0**
(identical to 0.10.2 for every function used; 0.10.1's pure-Python beat DP and
``__trim_beats`` differ and are NOT what is restated — see DESIGN.md §Oracle).
Parity of this module with real librosa is *unpinned*: it is pinned by the
known-answer tests in ``tests/test_oracle_known_answers.py`` instead.

One documented deviation: the CQT's octave decimation uses ``decimate2`` (a
47-tap Kaiser half-band FIR, scale sqrt(2)) in place of libsoxr's ``soxr_hq``
(libsoxr is not installed and cannot be bit-matched).

Reference call sites served (file:line under /root/reference/nightcore_analyzer):
  io.py:76           librosa.effects.trim               -> trim()
  tempo.py:44,158    librosa.onset.onset_strength       -> onset_strength()
  tempo.py:45,159    librosa.beat.beat_track            -> beat_track()
  tempo.py:58,63     librosa.feature.tempogram / tempo  -> tempogram_mean(), tempo_from_tg()
  tempo.py:168       librosa.frames_to_time             -> frames_to_time()
  pitch.py:58        librosa.feature.chroma_cqt         -> chroma_cqt()
  spectral.py:54-88  feature.spectral_centroid / spectral_rolloff / rms, stft, fft_frequencies,
                     amplitude_to_db, get_duration     -> spectral_*(), stft_mag(), ...
"""
from __future__ import annotations

import numpy as np
import scipy.signal

TINY32 = np.finfo(np.float32).tiny
TINY64 = np.finfo(np.float64).tiny


# --------------------------------------------------------------------------- windows
def hann(n: int) -> np.ndarray:
    """librosa ``filters.get_window('hann', n, fftbins=True)`` (periodic Hann, f64)."""
    return scipy.signal.get_window("hann", int(n), fftbins=True)


# --------------------------------------------------------------------------- STFT
def _frames(y: np.ndarray, n_fft: int, hop: int, t0: int, t1: int) -> np.ndarray:
    """Frames t0..t1-1 of ``y`` zero-padded by n_fft//2 on both sides (center=True,
    pad_mode='constant', librosa 0.10+ default)."""
    pad = n_fft // 2
    n = len(y)
    starts = np.arange(t0, t1, dtype=np.int64) * hop - pad
    idx = starts[:, None] + np.arange(n_fft, dtype=np.int64)[None, :]
    valid = (idx >= 0) & (idx < n)
    fr = np.zeros(idx.shape, dtype=np.float32)
    fr[valid] = y[idx[valid]]
    return fr


def stft(y, n_fft=2048, hop=512, window="hann", t0=0, t1=None) -> np.ndarray:
    """librosa.stft(center=True, pad_mode='constant') -> complex64 (1+n_fft//2, T).

    librosa multiplies the f32 frames by the f64 window, runs numpy's rfft in
    float64 and stores into a complex64 matrix (util.dtype_r2c(float32)).
    """
    y = np.asarray(y, dtype=np.float32)
    T = 1 + len(y) // hop
    t1 = T if t1 is None else min(t1, T)
    win = hann(n_fft) if window == "hann" else np.ones(n_fft)
    out = np.empty((1 + n_fft // 2, t1 - t0), dtype=np.complex64)
    blk = max(1, (1 << 22) // n_fft)
    for b0 in range(t0, t1, blk):
        b1 = min(t1, b0 + blk)
        fr = _frames(y, n_fft, hop, b0, b1)
        out[:, b0 - t0:b1 - t0] = np.fft.rfft(win[None, :] * fr, axis=-1).T
    return out


# --------------------------------------------------------------------------- mel
def hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        lt = f >= min_log_hz
        mels = np.array(mels)
        mels[lt] = min_log_mel + np.log(f[lt] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    lt = m >= min_log_mel
    freqs[lt] = min_log_hz * np.exp(logstep * (m[lt] - min_log_mel))
    return freqs


def mel_filter(sr=22050, n_fft=2048, n_mels=128, fmin=0.0, fmax=None) -> np.ndarray:
    """librosa.filters.mel(htk=False, norm='slaney', dtype=float32)."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def power_to_db(S, amin=1e-10, top_db=80.0, ref=1.0):
    """librosa.power_to_db (float32 in -> float32 out)."""
    S = np.asarray(S)
    log_spec = 10.0 * np.log10(np.maximum(amin, S))
    log_spec -= 10.0 * np.log10(np.maximum(amin, ref))
    if top_db is not None:
        log_spec = np.maximum(log_spec, log_spec.max() - top_db)
    return log_spec


def mel_db(y, sr=22050, n_fft=2048, hop=512, n_mels=128) -> np.ndarray:
    """power_to_db(melspectrogram(y, fmax=sr/2)) WITHOUT the top_db clamp.

    Returns float32 (n_mels, T).  Computed in frame blocks to bound memory; the
    arithmetic per element is that of librosa (|X|^2 in f32, f32 mel product)."""
    y = np.asarray(y, dtype=np.float32)
    T = 1 + len(y) // hop
    W = mel_filter(sr, n_fft, n_mels, 0.0, sr / 2.0)
    out = np.empty((n_mels, T), dtype=np.float32)
    blk = max(1, (1 << 21) // n_fft)
    for b0 in range(0, T, blk):
        b1 = min(T, b0 + blk)
        P = np.abs(stft(y, n_fft, hop, "hann", b0, b1)) ** 2.0
        M = W @ P                                            # f32 GEMM
        out[:, b0:b1] = 10.0 * np.log10(np.maximum(np.float32(1e-10), M))
    return out


def onset_strength(y, sr=22050, hop=512, n_fft=2048) -> np.ndarray:
    """librosa.onset.onset_strength(y, sr, hop_length) -> float32 (T,).

    mel (128, fmax=sr/2) -> power_to_db(top_db=80 vs the GLOBAL max) ->
    mean over mels of max(0, S[:, t] - S[:, t-1]) -> left pad lag + n_fft//(2 hop)
    -> truncate to T frames."""
    S = mel_db(y, sr, n_fft, hop)
    T = S.shape[1]
    S = np.maximum(S, S.max() - np.float32(80.0))
    d = np.maximum(np.float32(0.0), S[:, 1:] - S[:, :-1])
    od = np.mean(d, axis=0, dtype=np.float32)
    pad = 1 + n_fft // (2 * hop)
    od = np.concatenate([np.zeros(pad, dtype=np.float32), od])[:T]
    return od.astype(np.float32)


# --------------------------------------------------------------------------- tempogram / tempo
def ac_win_length(sr=22050, hop=512, ac_size=8.0) -> int:
    """time_to_frames(ac_size): floor(int(ac_size*sr) // hop)."""
    return int(int(ac_size * sr) // hop)


def tempogram_mean(onset: np.ndarray, win: int, block: int = 4096) -> np.ndarray:
    """mean over frames of librosa.feature.tempogram(onset_envelope, win_length=win).

    linear_ramp pad win//2 (end values 0) -> frames (hop 1) truncated to n ->
    x f64 periodic Hann(win) -> full autocorrelation via FFT (n_pad = 2 win - 1),
    first win lags -> per-frame inf-norm (columns with max < tiny left as is) ->
    mean over frames (float64).  Streamed in blocks of frames (the reference
    materialises the whole (win, n) matrix; the mean is identical up to f64
    summation order)."""
    onset = np.asarray(onset, dtype=np.float32)
    return tempogram_sum(onset, win, 0, onset.shape[-1], block) / onset.shape[-1]


def tempogram_sum(onset: np.ndarray, win: int, f0: int, f1: int, block: int = 4096) -> np.ndarray:
    """Sum over tempogram frames [f0, f1) of the inf-normalised autocorrelation columns
    (the body of tempogram_mean; a frame range lets a fixture script split one long
    signal's tempogram over processes)."""
    onset = np.asarray(onset, dtype=np.float32)
    n = onset.shape[-1]
    p = win // 2
    padded = np.pad(onset, (p, p), mode="linear_ramp", end_values=(0, 0))
    w = hann(win)
    n_pad = 2 * win - 1
    acc = np.zeros(win, dtype=np.float64)
    for b0 in range(f0, f1, block):
        b1 = min(f1, b0 + block)
        idx = np.arange(b0, b1)[:, None] + np.arange(win)[None, :]
        fr = padded[idx] * w[None, :]                       # f64
        ps = np.abs(np.fft.rfft(fr, n=n_pad, axis=-1)) ** 2
        ac = np.fft.irfft(ps, n=n_pad, axis=-1)[:, :win]
        mx = np.max(np.abs(ac), axis=-1, keepdims=True)
        mx[mx < TINY64] = 1.0
        acc += np.sum(ac / mx, axis=0)
    return acc


def tempo_frequencies(n_bins, sr=22050, hop=512) -> np.ndarray:
    f = np.zeros(int(n_bins), dtype=np.float64)
    f[0] = np.inf
    f[1:] = 60.0 * sr / (hop * np.arange(1.0, n_bins))
    return f


def tempo_logprior(win, sr, hop, start_bpm, std_bpm=1.0, max_tempo=320.0) -> np.ndarray:
    bpms = tempo_frequencies(win, sr, hop)
    with np.errstate(invalid="ignore"):
        logprior = -0.5 * ((np.log2(bpms) - np.log2(start_bpm)) / std_bpm) ** 2
    max_idx = int(np.argmax(bpms < max_tempo))
    logprior[:max_idx] = -np.inf
    return logprior


def tempo_from_tg(tg_mean, sr=22050, hop=512, start_bpm=120.0):
    """librosa.feature.tempo tail: argmax(log1p(1e6 tg) + logprior) -> (bpm, lag)."""
    win = len(tg_mean)
    bpms = tempo_frequencies(win, sr, hop)
    score = np.log1p(1e6 * tg_mean) + tempo_logprior(win, sr, hop, start_bpm)
    best = int(np.argmax(score))
    return float(bpms[best]), best


# --------------------------------------------------------------------------- beat tracking
def localmax(x):
    """librosa.util.localmax along the last axis (edge padding)."""
    xp = np.pad(x, (1, 1), mode="edge")
    return (x > xp[:-2]) & (x >= xp[2:])


def normalize_onsets(onset: np.ndarray) -> np.ndarray:
    onset = np.asarray(onset, dtype=np.float32)
    norm = onset.std(ddof=1)
    return onset / (norm + TINY32)


def gaussian_beat_window(P: float) -> np.ndarray:
    return np.exp(-0.5 * (np.arange(-P, P + 1) * 32.0 / P) ** 2)


def beat_local_score(onset_norm: np.ndarray, P: float) -> np.ndarray:
    """Same-mode convolution with the Gaussian beat window (float64), summed in
    ascending window index exactly as librosa's numba kernel does."""
    x = onset_norm.astype(np.float64)
    N = len(x)
    win = gaussian_beat_window(P)
    K = len(win)
    out = np.zeros(N, dtype=np.float64)
    i = np.arange(N)
    for k in range(K):
        j = i + K // 2 - k
        ok = (j >= 0) & (j < N)
        out[ok] += win[k] * x[j[ok]]
    return out


def dp_penalty(P: float, tightness: float = 100.0) -> np.ndarray:
    """pen[d] = tightness*(log(d) - log(P))**2 for d = 0..2P (d=0 unused)."""
    d = np.arange(0, int(2 * P) + 1, dtype=np.float64)
    with np.errstate(divide="ignore"):
        pen = np.float64(np.float32(tightness)) * (np.log(d) - np.log(P)) ** 2
    return pen


def beat_track_dp(localscore: np.ndarray, P: float, tightness: float = 100.0):
    """librosa 0.10.2+ ``__beat_track_dp`` (static tempo).  Returns (backlink, cumscore)."""
    N = len(localscore)
    pen = dp_penalty(P, tightness)
    dmin = int(np.round(P / 2.0))
    dmax = int(2 * P)
    thr = 0.01 * localscore.max()
    backlink = np.full(N, -1, dtype=np.int64)
    cumscore = np.zeros(N, dtype=np.float64)
    first = True
    for i in range(N):
        hi = min(dmax, i)                    # loc = i - d >= 0
        best_loc = -1
        best = -np.inf
        if hi >= dmin:
            d = np.arange(dmin, hi + 1)
            sc = cumscore[i - d] - pen[d]
            j = int(np.argmax(sc))           # first max over d ascending == strict '>' scan
            best = sc[j]
            best_loc = i - int(d[j])
            if not (best > -np.inf):
                best_loc = -1
        cumscore[i] = localscore[i] + best if best_loc >= 0 else localscore[i]
        if first and localscore[i] < thr:
            backlink[i] = -1
        else:
            backlink[i] = best_loc
            first = False
    return backlink, cumscore


def last_beat(cumscore: np.ndarray) -> int:
    mask = localmax(cumscore)
    N = len(cumscore)
    if not mask.any():
        return N - 1
    thr = 0.5 * np.median(cumscore[mask])
    for i in range(N - 1, -1, -1):
        if mask[i] and cumscore[i] >= thr:
            return i
    return N - 1


def trim_beats(localscore: np.ndarray, beats: np.ndarray, trim: bool = True) -> np.ndarray:
    """librosa 0.10.2+ ``__trim_beats``: threshold = 0.5 RMS of the smoothed
    beat-local-score (the numba slice keeps len(localscore)+... elements, i.e.
    n_beats + 2), then clear leading/trailing frames with localscore <= thr."""
    out = beats.copy()
    w = np.hanning(5)
    sm = np.convolve(localscore[beats], w)[len(w) // 2: len(localscore) + len(w) // 2]
    thr = 0.5 * (np.mean(sm ** 2) ** 0.5) if trim else 0.0
    N = len(localscore)
    n = 0
    while n < N and localscore[n] <= thr:
        out[n] = False
        n += 1
    n = N - 1
    while n >= 0 and localscore[n] <= thr:
        out[n] = False
        n -= 1
    return out


def beat_track(onset, sr=22050, hop=512, start_bpm=120.0, tightness=100.0, trim=True,
               tg_mean=None):
    """librosa.beat.beat_track(onset_envelope=...) -> (bpm, beat_frames int64)."""
    onset = np.asarray(onset, dtype=np.float32)
    if not onset.any():
        return 0.0, np.array([], dtype=np.int64)
    if tg_mean is None:
        tg_mean = tempogram_mean(onset, ac_win_length(sr, hop))
    bpm, _ = tempo_from_tg(tg_mean, sr, hop, start_bpm)
    frame_rate = float(sr) / hop
    P = float(np.round(frame_rate * 60.0 / bpm))
    ls = beat_local_score(normalize_onsets(onset), P)
    backlink, cumscore = beat_track_dp(ls, P, tightness)
    tail = last_beat(cumscore)
    beats = np.zeros(len(onset), dtype=bool)
    n = tail
    while n >= 0:
        beats[n] = True
        n = backlink[n]
    beats = trim_beats(ls, beats, trim)
    return bpm, np.flatnonzero(beats).astype(np.int64)


def frames_to_time(frames, sr=22050, hop=512):
    return (np.asanyarray(frames) * hop).astype(int) / float(sr)


# --------------------------------------------------------------------------- rms / trim
def rms_frames(y, frame_length=2048, hop=512) -> np.ndarray:
    """librosa.feature.rms(center=True, pad_mode='constant') -> f32 (T,)."""
    y = np.asarray(y, dtype=np.float32)
    T = 1 + len(y) // hop
    out = np.empty(T, dtype=np.float32)
    blk = 4096
    for b0 in range(0, T, blk):
        b1 = min(T, b0 + blk)
        fr = _frames(y, frame_length, hop, b0, b1)
        out[b0:b1] = np.mean(fr * fr, axis=-1, dtype=np.float32)
    return np.sqrt(out)


def trim(y, top_db=60.0, frame_length=2048, hop=512):
    """librosa.effects.trim -> (y[start:end], (start, end))."""
    y = np.asarray(y, dtype=np.float32)
    rms = rms_frames(y, frame_length, hop)
    ref = np.max(rms)
    power = np.square(rms)
    db = 10.0 * np.log10(np.maximum(np.float32(1e-10), power)) \
        - 10.0 * np.log10(np.maximum(np.float32(1e-10), ref * ref))
    nz = np.flatnonzero(db > -top_db)
    if nz.size:
        start = int(nz[0] * hop)
        end = min(len(y), int((nz[-1] + 1) * hop))
    else:
        start, end = 0, 0
    return y[start:end], (start, end)


# --------------------------------------------------------------------------- spectral features
# spectral.py:52-94 calls these librosa functions on a file at its native rate (sr=None).
def fft_frequencies(sr=22050, n_fft=2048) -> np.ndarray:
    """librosa.fft_frequencies = np.fft.rfftfreq(n_fft, 1/sr) (f64): k * (1 / (n_fft * (1/sr)))."""
    return np.fft.rfftfreq(n=n_fft, d=1.0 / sr)


def stft_mag(y, n_fft=2048, hop=512) -> np.ndarray:
    """np.abs(librosa.stft(y)) -> f32 (1 + n_fft//2, T).  librosa allocates the STFT matrix in
    Fortran order, so reductions over time run frame by frame (kept here for the same
    summation order)."""
    return np.asfortranarray(np.abs(stft(y, n_fft, hop)))


def normalize_l1(S: np.ndarray) -> np.ndarray:
    """librosa.util.normalize(S, norm=1, axis=-2): f64 magnitude sums, columns whose sum is
    below tiny(S) are left unscaled, the result is stored back in S's dtype."""
    length = np.sum(np.abs(S).astype(np.float64), axis=-2, keepdims=True)
    length[length < np.finfo(S.dtype).tiny] = 1.0
    out = np.empty_like(S)
    out[:] = S / length
    return out


def spectral_centroid(y=None, sr=22050, S=None, n_fft=2048, hop=512) -> np.ndarray:
    """librosa.feature.spectral_centroid -> f64 (1, T): sum_k f_k * S_k / sum_k S_k."""
    S = stft_mag(y, n_fft, hop) if S is None else S
    freq = fft_frequencies(sr, n_fft)[:, None]
    return np.sum(freq * normalize_l1(S), axis=-2, keepdims=True)


def spectral_rolloff(y=None, sr=22050, S=None, n_fft=2048, hop=512, roll_percent=0.85) -> np.ndarray:
    """librosa.feature.spectral_rolloff -> f64 (1, T): the lowest bin frequency at which the
    f32 running sum of |S| reaches roll_percent of the frame total."""
    S = stft_mag(y, n_fft, hop) if S is None else S
    freq = fft_frequencies(sr, n_fft)[:, None]
    total = np.cumsum(S, axis=-2)
    thr = np.expand_dims(roll_percent * total[-1, :], axis=-2)
    ind = np.where(total < thr, np.nan, 1)
    return np.nanmin(ind * freq, axis=-2, keepdims=True)


def amplitude_to_db(S, ref=np.max, amin=1e-5, top_db=80.0) -> np.ndarray:
    """librosa.amplitude_to_db = power_to_db(|S|^2, ref=ref(|S|)^2, amin=amin^2, top_db)."""
    mag = np.abs(np.asarray(S))
    ref_value = ref(mag) if callable(ref) else np.abs(ref)
    power = np.square(mag, out=mag)
    return power_to_db(power, amin=amin ** 2, top_db=top_db, ref=ref_value ** 2)


def get_duration(y, sr=22050) -> float:
    """librosa.get_duration(y=y, sr=sr) = samples / sr."""
    return float(np.asarray(y).shape[-1]) / sr


# --------------------------------------------------------------------------- load-time resample
# io.py:54 (librosa.load(sr=22050) -> soxr_hq, absent here): the engine's stand-in is
# scipy.signal.resample_poly; this is its upfirdn sum restated term by term (scipy 1.15
# signal/_upfirdn_apply.pyx _apply_impl), the order the GPU kernel reproduces.
def resample_poly_terms(x, up, down, h, pre_remove, n_out):
    """y[m'] = sum over i = hpp-1..0 of x[x_idx - i] * h[p + i up] for m = m' + pre_remove,
    x_idx = m down // up, p = m down % up (oldest sample first, separate rounding of
    products and sums); left out-of-range taps are skipped while x_idx < len(x), every
    tap (zero samples included) is added once x_idx >= len(x)."""
    x = np.asarray(x, np.float64)
    h = np.asarray(h, np.float64)
    hpp = len(h) // up
    m = np.arange(n_out, dtype=np.int64) + pre_remove
    x_idx = m * down // up
    ph = m * down % up
    flush = x_idx >= len(x)
    acc = np.zeros(n_out)
    xp = np.concatenate([x, [0.0]])
    for i in range(hpp - 1, -1, -1):
        xi = x_idx - i
        inside = (xi >= 0) & (xi < len(x))
        xv = xp[np.where(inside, xi, len(x))]
        take = flush | (xi >= 0)
        acc = np.where(take, acc + xv * h[ph + i * up], acc)
    return acc


# --------------------------------------------------------------------------- CQT chroma
C1_HZ =440.0 * 2.0 ** ((24 - 69) / 12.0)       # note_to_hz('C1')
WINDOW_BANDWIDTH_HANN = 1.50018310546875


def halfband_taps(K: int = 23, beta: float = 11.0) -> np.ndarray:
    """The engine's soxr_hq replacement: h[n] = 0.5 sinc(n/2) kaiser(n), n=-K..K,
    normalised to unit DC gain (f64, 2K+1 taps; even n != 0 are exact zeros)."""
    n = np.arange(-K, K + 1, dtype=np.float64)
    h = 0.5 * np.sinc(n / 2.0) * np.kaiser(2 * K + 1, beta)
    h[(n % 2 == 0) & (n != 0)] = 0.0
    return h / h.sum()


def decimate2(y: np.ndarray, taps: np.ndarray | None = None) -> np.ndarray:
    """librosa.resample(y, orig_sr=2, target_sr=1, res_type='soxr_hq', scale=True)
    restated with ``halfband_taps``: out[m] = sqrt(2) * sum_n h[n] y[2m - n]
    (zero outside), length ceil(len/2), f64 accumulation -> f32."""
    if taps is None:
        taps = halfband_taps()
    K = (len(taps) - 1) // 2
    y = np.asarray(y, dtype=np.float32).astype(np.float64)
    L = len(y)
    M = (L + 1) // 2
    yp = np.pad(y, (K, K + 1))
    out = np.zeros(M, dtype=np.float64)
    for j, n in enumerate(range(-K, K + 1)):
        if taps[j] == 0.0:
            continue
        # y[2m - n] -> yp[2m - n + K]
        out += taps[j] * yp[K - n: K - n + 2 * M: 2][:M]
    return (out * np.sqrt(2.0)).astype(np.float32)


def resample_half(y: np.ndarray, taps: np.ndarray | None = None) -> np.ndarray:
    """librosa.resample(y, orig_sr=2 sr', target_sr=sr', res_type='soxr_hq') with the
    default scale=False, restated with ``halfband_taps`` (decimate2 without the sqrt(2))."""
    if taps is None:
        taps = halfband_taps()
    K = (len(taps) - 1) // 2
    y = np.asarray(y, dtype=np.float32).astype(np.float64)
    M = (len(y) + 1) // 2
    yp = np.pad(y, (K, K + 1))
    out = np.zeros(M, dtype=np.float64)
    for j, n in enumerate(range(-K, K + 1)):
        if taps[j] == 0.0:
            continue
        out += taps[j] * yp[K - n: K - n + 2 * M: 2][:M]
    return out.astype(np.float32)


def interval_frequencies(n_bins, fmin, bins_per_octave):
    ratios = 2.0 ** (np.arange(0, bins_per_octave, dtype=float) / bins_per_octave)
    n_oct = int(np.ceil(n_bins / len(ratios)))
    allr = np.multiply.outer(2.0 ** np.arange(n_oct), ratios).flatten()[:n_bins]
    return np.sort(allr) * fmin


def relative_bandwidth(freqs):
    bpo = np.empty_like(freqs)
    logf = np.log2(freqs)
    bpo[0] = 1 / (logf[1] - logf[0])
    bpo[-1] = 1 / (logf[-1] - logf[-2])
    bpo[1:-1] = 2 / (logf[2:] - logf[:-2])
    return (2.0 ** (2 / bpo) - 1) / (2.0 ** (2 / bpo) + 1)


def wavelet_lengths(freqs, sr, alpha):
    Q = 1.0 / alpha
    f_cutoff = max(freqs * (1 + 0.5 * WINDOW_BANDWIDTH_HANN / Q))
    return Q * sr / freqs, f_cutoff


def _float_window(n):
    n_min, n_max = int(np.floor(n)), int(np.ceil(n))
    w = hann(n_min)
    if len(w) < n_max:
        w = np.pad(w, (0, n_max - len(w)))
    w[n_min:] = 0.0
    return w


def wavelet_basis(freqs, sr, alpha):
    """librosa.filters.wavelet(norm=1, pad_fft=True, window='hann') -> complex64."""
    lengths, _ = wavelet_lengths(freqs, sr, alpha)
    filt = []
    for ilen, f in zip(lengths, freqs):
        ang = np.arange(-ilen // 2, ilen // 2, dtype=float) * 2 * np.pi * f / sr
        sig = np.cos(ang) + 1j * np.sin(ang)
        sig *= _float_window(len(sig))
        sig = sig / np.sum(np.abs(sig))
        filt.append(sig)
    max_len = int(2.0 ** (np.ceil(np.log2(max(lengths)))))
    out = np.zeros((len(filt), max_len), dtype=np.complex64)
    for i, s in enumerate(filt):
        lp = (max_len - len(s)) // 2
        out[i, lp:lp + len(s)] = s
    return out, lengths


def sparsify_rows(x, quantile=0.01):
    """librosa.util.sparsify_rows -> dense complex64 array with dropped entries 0."""
    mags = np.abs(x)
    norms = np.sum(mags, axis=1, keepdims=True)
    mag_sort = np.sort(mags, axis=1)
    cum = np.cumsum(mag_sort / norms, axis=1)
    thr_idx = np.argmin(cum < quantile, axis=1)
    out = np.zeros(x.shape, dtype=np.complex64)
    for i, j in enumerate(thr_idx):
        keep = mags[i] >= mag_sort[i, j]
        out[i, keep] = x[i, keep]
    return out


def vqt_filter_fft(sr, freqs, alpha, sparsity=0.01):
    basis, lengths = wavelet_basis(freqs, sr, alpha)
    n_fft = basis.shape[1]
    basis *= lengths[:, np.newaxis] / float(n_fft)
    fb = np.fft.fft(basis.astype(np.complex128), n=n_fft, axis=1)[:, :(n_fft // 2) + 1]
    return sparsify_rows(fb, sparsity), n_fft


def cqt_mag(y, sr=22050, hop=512, fmin=None, n_bins=252, bins_per_octave=36, tuning=0.0):
    """|librosa.cqt(y, sr, hop, fmin, n_bins, bpo, tuning)| (res_type -> decimate2)."""
    if fmin is None:
        fmin = C1_HZ
    y = np.asarray(y, dtype=np.float32)
    n_oct = int(np.ceil(float(n_bins) / bins_per_octave))
    n_filters = min(bins_per_octave, n_bins)
    fmin = fmin * 2.0 ** (tuning / bins_per_octave)
    freqs = interval_frequencies(n_bins, fmin, bins_per_octave)
    alpha = relative_bandwidth(freqs)
    lengths, _ = wavelet_lengths(freqs, sr, alpha)
    resp = []
    my_y, my_sr, my_hop = y, float(sr), hop
    for i in range(n_oct):
        sl = slice(-n_filters, None) if i == 0 else slice(-n_filters * (i + 1), -n_filters * i)
        fb, n_fft = vqt_filter_fft(my_sr, freqs[sl], alpha[sl])
        fb = (fb * np.sqrt(sr / my_sr)).astype(np.complex64)
        D = stft(my_y, n_fft, my_hop, "ones")
        resp.append((fb @ D).astype(np.complex64))
        if my_hop % 2 == 0:
            my_hop //= 2
            my_sr /= 2.0
            my_y = decimate2(my_y)
    max_col = min(r.shape[-1] for r in resp)
    V = np.empty((n_bins, max_col), dtype=np.complex64)
    end = n_bins
    for r in resp:
        n_o = r.shape[0]
        if end < n_o:
            V[:end] = r[-end:, :max_col]
        else:
            V[end - n_o:end] = r[:, :max_col]
        end -= n_o
    V /= np.sqrt(lengths[:, np.newaxis])
    return np.abs(V).astype(np.float32)


def piptrack(y, sr=22050, n_fft=2048, hop=None, fmin=150.0, fmax=4000.0, threshold=0.1):
    """librosa.piptrack(y=...) -> (pitches f32, mags f32), shape (1+n_fft//2, T)."""
    if hop is None:
        hop = n_fft // 4
    S = np.abs(stft(y, n_fft, hop, "hann"))                          # f32
    fmax = min(fmax, float(sr) / 2)
    fft_freqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    avg = np.gradient(S, axis=0)
    Sd = S.astype(np.float64)
    # numba stencil typing: f32 + f32 -> f32 ; int * f32 -> f64 ; f32 / int -> f64
    a = (S[2:] + S[:-2]).astype(np.float64) - 2 * Sd[1:-1]
    b = (S[2:] - S[:-2]).astype(np.float64) / 2
    with np.errstate(divide="ignore", invalid="ignore"):
        sh = np.where(np.abs(b) >= np.abs(a), 0.0, -b / a)
    shift = np.zeros_like(S)
    shift[1:-1] = sh.astype(np.float32)
    dskew = np.float32(0.5) * avg * shift
    pitches = np.zeros_like(S)
    mags = np.zeros_like(S)
    freq_mask = ((fmin <= fft_freqs) & (fft_freqs < fmax))[:, None]
    ref_value = threshold * np.max(S, axis=0, keepdims=True)
    Z = S * (S > ref_value)
    Zp = np.pad(Z, ((1, 1), (0, 0)), mode="edge")
    lm = (Z > Zp[:-2]) & (Z >= Zp[2:])
    idx = np.nonzero(freq_mask & lm)
    pitches[idx] = (idx[0] + shift[idx]) * float(sr) / n_fft
    mags[idx] = S[idx] + dskew[idx]
    return pitches, mags


def tuning_edges(resolution=0.01):
    return np.linspace(-0.5, 0.5, int(np.ceil(1.0 / resolution)) + 1)


def tuning_counts(freqs, resolution=0.01, bins_per_octave=36):
    """The residual histogram of librosa.pitch_tuning (None when no frequency is > 0)."""
    freqs = np.atleast_1d(freqs)
    freqs = freqs[freqs > 0]
    if not np.any(freqs):
        return None
    octs = np.log2(freqs / (440.0 / 16))
    residual = np.mod(bins_per_octave * octs, 1.0)
    residual[residual >= 0.5] -= 1.0
    counts, _ = np.histogram(residual, tuning_edges(resolution))
    return counts


def pitch_tuning(freqs, resolution=0.01, bins_per_octave=36):
    counts = tuning_counts(freqs, resolution, bins_per_octave)
    if counts is None:
        return 0.0
    return float(tuning_edges(resolution)[np.argmax(counts)])


def estimate_tuning_detail(y, sr=22050, n_fft=2048, bins_per_octave=36):
    """(tuning, bin index, decision margin): estimate_tuning with the histogram's argmax bin
    and its lead over the runner-up bin (test diagnostics; 0 when no peak passes)."""
    pitch, mag = piptrack(y, sr, n_fft)
    pm = pitch > 0
    thr = np.median(mag[pm]) if pm.any() else 0.0
    counts = tuning_counts(pitch[(mag >= thr) & pm], 0.01, bins_per_octave)
    if counts is None:
        return 0.0, 50, 0
    best = int(np.argmax(counts))
    return float(tuning_edges(0.01)[best]), best, int(counts[best] - np.max(np.delete(counts, best)))


def estimate_tuning(y, sr=22050, n_fft=2048, bins_per_octave=36):
    return estimate_tuning_detail(y, sr, n_fft, bins_per_octave)[0]


def cq_to_chroma(n_input=252, bins_per_octave=36, n_chroma=12) -> np.ndarray:
    n_merge = float(bins_per_octave) / n_chroma
    m = np.repeat(np.eye(n_chroma), int(n_merge), axis=1)
    m = np.roll(m, -int(n_merge // 2), axis=1)
    n_oct = np.ceil(float(n_input) / bins_per_octave)
    m = np.tile(m, int(n_oct))[:, :n_input]
    midi0 = np.mod(12 * (np.log2(C1_HZ) - np.log2(440.0)) + 69, 12)
    roll = int(np.round(midi0 * (n_chroma / 12.0)))
    return np.roll(m, roll, axis=0).astype(np.float32)


def chroma_cqt(y, sr=22050, hop=512, bins_per_octave=36, n_octaves=7, tuning=None):
    """librosa.feature.chroma_cqt(y, sr, bins_per_octave=36, hop_length=512) (n_chroma=12)."""
    if tuning is None:
        tuning = estimate_tuning(y, sr, bins_per_octave=bins_per_octave)
    C = cqt_mag(y, sr, hop, None, n_octaves * bins_per_octave, bins_per_octave, tuning)
    chroma = cq_to_chroma(C.shape[0], bins_per_octave, 12) @ C          # f32
    chroma[chroma < 0] = 0.0
    mx = np.max(np.abs(chroma), axis=0, keepdims=True).astype(np.float64)
    mx[mx < TINY32] = 1.0
    return (chroma / mx).astype(np.float32)
