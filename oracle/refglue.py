"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's own glue on the
hot path, on top of ``oracle.ncref``.  Every function cites the reference
file:line (under /root/reference/nightcore_analyzer) it restates.

This is the checker for the MI355X engine and the timed CPU baseline
(``bench.py`` cpu_baseline, kind "port").  It is pinned against golden fixtures
made by running the reference's own modules (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import ncref

SR = 22050
WINDOW_SEC, HOP_SEC = 10.0, 5.0          # io.py:20-21
ENERGY_GATE_DB, SILENCE_STRIP_DB = -40.0, 60.0   # io.py:22-23
HOP_LENGTH = 512                         # tempo.py:24
MIN_BEATS = 4                            # tempo.py:22
AGREEMENT_TOLERANCE = 0.08               # tempo.py:23
IBI_HOP_LENGTH, IBI_MIN_IBIS = 64, 4     # tempo.py:116-117
CHUNK_SEC, MIN_CHUNKS = 20.0, 3          # pitch.py:44-45
REF_HZ = 440.0                           # pitch.py:50
N_BOOTSTRAP, CI_LEVEL, MIN_VALID = 2000, 0.95, 3   # consensus.py:52-55
PURE_NC_TOLERANCE = 0.02                 # consensus.py:54
ALIGN_SR, ALIGN_HOP = 11025, 512         # xcorr.py:45-46
ALIGN_SPEED_LO, ALIGN_SPEED_HI, ALIGN_N_SPEEDS = 1.03, 1.50, 30   # xcorr.py:47-49
ALIGN_MAX_OFFSET, ALIGN_MIN_OFFSET = 120.0, 1.0                  # xcorr.py:50-51


# ------------------------------------------------------------------ io.py
@dataclass
class Window:                             # io.py:27-34 AudioWindow
    audio: np.ndarray
    sample_rate: int
    start_sec: float
    end_sec: float
    energy_db: float


def rms_db(a: np.ndarray) -> float:       # io.py:38-40
    rms = float(np.sqrt(np.mean(a.astype(np.float64) ** 2)))
    return 20.0 * np.log10(max(rms, 1e-10))


def strip_silence(audio, sr=SR, top_db=SILENCE_STRIP_DB):   # io.py:58-79
    trimmed, (start, end) = ncref.trim(audio, top_db=top_db)
    return trimmed, start / sr, (len(audio) - end) / sr


def slice_windows(audio, sr=SR, window_sec=WINDOW_SEC, hop_sec=HOP_SEC):  # io.py:82-112
    win_n, hop_n = int(window_sec * sr), int(hop_sec * sr)
    out, start = [], 0
    while start + win_n <= len(audio):
        chunk = audio[start:start + win_n]
        out.append(Window(chunk, sr, start / sr, (start + win_n) / sr, rms_db(chunk)))
        start += hop_n
    return out


def energy_gate(windows, threshold_db=ENERGY_GATE_DB):   # io.py:115-126
    if not windows:
        return windows
    peak = max(w.energy_db for w in windows)
    return [w for w in windows if w.energy_db >= peak + threshold_db]


# ------------------------------------------------------------------ tempo.py
def estimate_tempo(y, sr=SR, start_bpm=120.0) -> Optional[float]:   # tempo.py:27-77
    onset = ncref.onset_strength(y, sr, HOP_LENGTH)
    tg = ncref.tempogram_mean(onset, ncref.ac_win_length(sr, HOP_LENGTH)) if onset.any() else None
    t_def, beats = ncref.beat_track(onset, sr, HOP_LENGTH, start_bpm, tg_mean=tg)
    t_def = float(np.atleast_1d(t_def)[0])
    if len(beats) < MIN_BEATS:
        return None
    t_tg, _ = ncref.tempo_from_tg(tg, sr, HOP_LENGTH, start_bpm)   # feature.tempo: same tg
    if t_def > 0:
        if abs(t_def - t_tg) / t_def <= AGREEMENT_TOLERANCE:
            return float((t_def + t_tg) / 2.0)
    return t_def if t_def > 0 else (t_tg if t_tg > 0 else None)


def batch_estimate_tempo(windows, start_bpm=120.0):    # tempo.py:80-111
    return [estimate_tempo(w.audio, w.sample_rate, start_bpm) for w in windows]


def estimate_ibis_global(y, sr=SR, hop_length=IBI_HOP_LENGTH, min_ibis=IBI_MIN_IBIS,
                         start_bpm=120.0):               # tempo.py:120-173
    onset = ncref.onset_strength(y, sr, hop_length)
    _, beats = ncref.beat_track(onset, sr, hop_length, start_bpm)
    beats = np.atleast_1d(beats)
    if len(beats) < min_ibis + 1:
        return None
    t = ncref.frames_to_time(beats, sr, hop_length)
    ibis = np.diff(t)
    ibis = ibis[ibis > 0.05]
    if len(ibis) < min_ibis:
        return None
    return ibis


# ------------------------------------------------------------------ pitch.py
def mean_chroma(audio, sr=SR) -> np.ndarray:            # pitch.py:55-64
    return ncref.chroma_cqt(audio, sr, 512, 36).mean(axis=1)


def cyclic_xcorr_peak(src_c, nc_c) -> int:              # pitch.py:67-85
    n = len(src_c)
    xc = np.array([float(np.dot(src_c, np.roll(nc_c, -k))) for k in range(n)])
    lag = int(np.argmax(xc))
    if lag > n // 2:
        lag -= n
    return lag


def chunk_lag(src_chunk, nc_chunk, sr=SR) -> int:       # pitch.py:88-95 (lag; shift = lag/3)
    return cyclic_xcorr_peak(mean_chroma(src_chunk, sr), mean_chroma(nc_chunk, sr))


def chunk_plan(n_src: int, n_nc: int, sr=SR):
    """pitch.py:121-138: list of (src_lo, src_hi, nc_lo, nc_hi)."""
    cn = int(CHUNK_SEC * sr)
    n = min(n_src // cn, n_nc // cn)
    if n < 1:
        return [(0, n_src, 0, n_nc)]
    return [(i * cn, (i + 1) * cn, i * cn, (i + 1) * cn) for i in range(n)]


def estimate_pitch_chroma(src, nc, sr=SR):              # pitch.py:100-173
    plan = chunk_plan(len(src), len(nc), sr)
    lags = [chunk_lag(src[a:b], nc[c:d], sr) for a, b, c, d in plan]
    shifts = np.array([lag / 3.0 for lag in lags])
    n = len(plan)
    point = float(np.median(shifts))
    if n >= MIN_CHUNKS:
        rng = np.random.default_rng(0)
        boots = np.array([float(np.median(rng.choice(shifts, size=n, replace=True)))
                          for _ in range(2000)])
        ci = (float(np.percentile(boots, 2.5)), float(np.percentile(boots, 97.5)))
    else:
        ci = (point, point)
    src_hz = [REF_HZ] * n
    nc_hz = [REF_HZ * (2.0 ** (st / 12.0)) for st in shifts]
    return src_hz, nc_hz, point, ci, n, lags


# ------------------------------------------------------------------ consensus.py
def valid(values) -> np.ndarray:                       # consensus.py:236-240
    return np.array([v for v in values if v is not None and np.isfinite(v) and v > 0],
                    dtype=np.float64)


def bootstrap_ratio(nc_vals, src_vals, n_boot=N_BOOTSTRAP, ci=CI_LEVEL):  # consensus.py:243-267
    rng = np.random.default_rng(seed=42)
    point = float(np.median(nc_vals) / np.median(src_vals))
    boot = np.empty(n_boot)
    for i in range(n_boot):
        a = rng.choice(nc_vals, size=len(nc_vals), replace=True)
        b = rng.choice(src_vals, size=len(src_vals), replace=True)
        boot[i] = np.median(a) / np.median(b)
    alpha = (1.0 - ci) / 2.0
    return point, (float(np.percentile(boot, alpha * 100)),
                   float(np.percentile(boot, (1.0 - alpha) * 100)))


def compute_ibi_ratio(nc_ibis, src_ibis, n_boot=N_BOOTSTRAP, ci=CI_LEVEL):  # consensus.py:270-312
    rng = np.random.default_rng(seed=42)
    point = float(np.median(src_ibis) / np.median(nc_ibis))
    boot = np.empty(n_boot)
    for i in range(n_boot):
        s = rng.choice(src_ibis, size=len(src_ibis), replace=True)
        n = rng.choice(nc_ibis, size=len(nc_ibis), replace=True)
        boot[i] = np.median(s) / np.median(n)
    alpha = (1.0 - ci) / 2.0
    return point, (float(np.percentile(boot, alpha * 100)),
                   float(np.percentile(boot, (1.0 - alpha) * 100)))


def classify(tr, pr, tci, pci, tol=PURE_NC_TOLERANCE) -> str:   # consensus.py:315-336
    d = pr - tr
    overlap = tci[0] <= pci[1] and pci[0] <= tci[1]
    if abs(d) <= tol or (overlap and abs(d) <= 2 * tol):
        return "pure_nightcore"
    if d > tol:
        return "independent_pitch_shift"
    if tr > 1.0 + tol and d < -tol:
        return "time_stretch_only"
    return "ambiguous"


def build_result(src_p, nc_p, src_t, nc_t, nc_duration=None, src_duration=None) -> dict:
    """consensus.py:519-608 (numerical fields only; strings checked via goldens)."""
    sp, npch, st, nt = valid(src_p), valid(nc_p), valid(src_t), valid(nc_t)
    if len(st) < MIN_VALID or len(nt) < MIN_VALID:
        raise ValueError(
            f"Insufficient valid tempo windows (source: {len(st)}, "
            f"nightcore: {len(nt)}).  Need ≥ {MIN_VALID} each.")
    if len(sp) >= MIN_VALID and len(npch) >= MIN_VALID:
        pr, pci = bootstrap_ratio(npch, sp)
        nsp, nnp = len(sp), len(npch)
    else:
        pr, pci, nsp, nnp = 1.0, (1.0, 1.0), 0, 0
    tr, tci = bootstrap_ratio(nt, st)
    corrected = False
    if (nc_duration is not None and src_duration is not None
            and nc_duration < src_duration * 0.99 and tr < 1.0):
        tr = 1.0 / tr
        tci = (1.0 / tci[1], 1.0 / tci[0])
        corrected = True
    return dict(tempo_ratio=tr, pitch_ratio=pr, tempo_ci=tci, pitch_ci=pci,
                classification=classify(tr, pr, tci, pci),
                n_source_pitch_windows=nsp, n_nc_pitch_windows=nnp,
                n_source_tempo_windows=len(st), n_nc_tempo_windows=len(nt),
                nc_median_bpm=float(np.median(nt)), src_median_bpm=float(np.median(st)),
                tempo_was_corrected=corrected)


# ------------------------------------------------------------------ pipeline.py
def run_arrays(nc_audio, src_audio, sr=SR, *, window_sec=WINDOW_SEC, hop_sec=HOP_SEC,
               energy_gate_db=ENERGY_GATE_DB, silence_strip_db=SILENCE_STRIP_DB,
               src_trim_sec=0.0, auto_align=False, compute_pitch=True, compute_ibi=True) -> dict:
    """pipeline.py:23-216 on decoded arrays (load_audio is out of scope)."""
    nc_audio = np.asarray(nc_audio, np.float32)
    src_audio = np.asarray(src_audio, np.float32)
    if silence_strip_db is not None:                                   # :91-104
        nc_audio, _, _ = strip_silence(nc_audio, sr, silence_strip_db)
        src_audio, _, _ = strip_silence(src_audio, sr, silence_strip_db)
    intro = None
    if src_trim_sec > 0.0:                                             # :106-110
        src_audio = src_audio[int(src_trim_sec * sr):]
        intro = src_trim_sec
    elif auto_align:                                                   # :111-125
        raw_offset, _ = find_content_offset(src_audio, nc_audio, sr)
        if raw_offset >= ALIGN_MIN_OFFSET:
            src_audio = src_audio[int(raw_offset * sr):]
            intro = raw_offset
    ncw = energy_gate(slice_windows(nc_audio, sr, window_sec, hop_sec), energy_gate_db)
    srw = energy_gate(slice_windows(src_audio, sr, window_sec, hop_sec), energy_gate_db)
    if not ncw or not srw:                                             # :142-146
        raise RuntimeError("All windows were discarded by the energy gate.  "
                           "Try raising --energy-gate (e.g. --energy-gate -60).")
    lags = []
    if compute_pitch:                                                  # :149-161
        src_p, nc_p, _, _, _, lags = estimate_pitch_chroma(src_audio, nc_audio, sr)
    else:
        src_p, nc_p = [], []
    src_t = batch_estimate_tempo(srw)                                  # :169
    nc_dur, src_dur = len(nc_audio) / sr, len(src_audio) / sr          # :171-172
    prior = 120.0
    vs = [t for t in src_t if t is not None]
    if vs and nc_dur > 0 and src_dur > 0:                              # :175-183
        prior = float(np.median(vs)) * (src_dur / nc_dur)
    nc_t = batch_estimate_tempo(ncw, prior)                            # :186
    res = build_result(src_p, nc_p, src_t, nc_t, nc_duration=nc_dur, src_duration=src_dur)
    res.update(src_tempos=src_t, nc_tempos=nc_t, src_pitches=src_p, nc_pitches=nc_p,
               chunk_lags=lags, nc_start_bpm=prior, nc_duration=nc_dur,
               src_duration=src_dur, intro_offset_sec=intro,
               n_src_windows=len(srw), n_nc_windows=len(ncw))
    if compute_ibi:                                                    # :203-213
        nci = estimate_ibis_global(nc_audio, sr, start_bpm=prior)
        sri = estimate_ibis_global(src_audio, sr)
        res["ibi_ratio"] = res["ibi_ci"] = None
        if nci is not None and len(nci) >= 4 and sri is not None and len(sri) >= 4:
            res["ibi_ratio"], res["ibi_ci"] = compute_ibi_ratio(nci, sri)
    return res


# ------------------------------------------------------------------ xcorr.py
def estimate_speed_xcorr_arrays(ya, yb, sr=SR, n_windows=20, window_sec=3.0,
                                search_range=0.05, skip_edges=0.10):   # xcorr.py:54-162
    ya = np.asarray(ya, np.float32)
    yb = np.asarray(yb, np.float32)
    min_len = min(len(ya), len(yb))
    s, e = int(min_len * skip_edges), int(min_len * (1.0 - skip_edges))
    ya, yb = ya[s:e], yb[s:e]
    win = int(window_sec * sr)
    search = int(search_range * len(yb))
    stride = max(1, win // 4)
    if len(ya) < win or len(yb) < win:
        return 1.0, 0.0
    corr, qual = [], []
    for pa in np.linspace(0, len(ya) - win, n_windows).astype(int):
        wa = ya[pa:pa + win]
        if wa.shape[0] < win or float(np.sqrt(np.mean(wa ** 2))) < 1e-3:
            continue
        exp_pb = int(pa * len(yb) / len(ya))
        lo, hi = max(0, exp_pb - search), min(len(yb) - win, exp_pb + search)
        if lo >= hi:
            continue
        na = float(np.linalg.norm(wa))
        if na < 1e-10:
            continue
        best_c, best_pb = -1.0, exp_pb
        for pb in range(lo, hi, stride):
            wb = yb[pb:pb + win]
            if wb.shape[0] < win:
                continue
            nb = float(np.linalg.norm(wb))
            if nb < 1e-10:
                continue
            c = float(np.dot(wa, wb) / (na * nb))
            if c > best_c:
                best_c, best_pb = c, pb
        if best_c > 0:
            corr.append((pa, best_pb))
            qual.append(best_c)
    if len(corr) < 3:
        return 1.0, 0.0
    a = np.array([c[0] for c in corr], dtype=float)
    b = np.array([c[1] for c in corr], dtype=float)
    return float(np.polyfit(a, b, 1)[0]), float(np.median(qual))


def find_content_offset(src_audio, nc_audio, sr=SR, *, speed_lo=ALIGN_SPEED_LO, speed_hi=ALIGN_SPEED_HI,
                        n_speeds=ALIGN_N_SPEEDS, max_offset_sec=ALIGN_MAX_OFFSET, detail=False):
    """xcorr.py:165-259: RMS-envelope cross-correlation over a grid of nightcore speeds.
    Returns (offset_sec, speed); with detail=True also (peak_idx, speed_idx, score) of the
    winner (speed_idx -1 when no speed is searchable)."""
    if sr != 2 * ALIGN_SR:
        raise NotImplementedError("the restated resampler is 2:1 (sr 22050 -> 11025) only")
    src_env = ncref.rms_frames(ncref.resample_half(src_audio), 2048, ALIGN_HOP).astype(np.float64)  # :205-211
    nc_env = ncref.rms_frames(ncref.resample_half(nc_audio), 2048, ALIGN_HOP).astype(np.float64)
    hop_sec = ALIGN_HOP / ALIGN_SR                                     # :213
    max_offset_frames = int(max_offset_sec / hop_sec)                  # :214
    best_score, best_offset, best_speed = -1.0, 0.0, (speed_lo + speed_hi) / 2.0
    best = (0, -1, -1.0)
    for si, speed in enumerate(np.linspace(speed_lo, speed_hi, n_speeds)):   # :220
        n_st = int(len(nc_env) / speed)
        if n_st < 4 or n_st >= len(src_env):
            continue
        stretched = np.interp(np.linspace(0.0, 1.0, n_st), np.linspace(0.0, 1.0, len(nc_env)), nc_env)
        search_len = min(max_offset_frames, len(src_env) - n_st)       # :237
        if search_len <= 0:
            continue
        corr = np.correlate(src_env[:search_len + n_st], stretched, mode="valid")[:search_len + 1]
        if len(corr) == 0:
            continue
        peak_idx = int(np.argmax(corr))
        peak_val = float(corr[peak_idx])
        win_energy = float(np.sum(src_env[peak_idx:peak_idx + n_st] ** 2))   # :252-254
        query_energy = float(np.sum(stretched ** 2))
        denom = np.sqrt(win_energy * query_energy)
        score = peak_val / denom if denom > 1e-12 else 0.0
        if score > best_score:                                         # :257
            best_score, best_offset, best_speed = score, peak_idx * hop_sec, speed
            best = (peak_idx, si, score)
    if detail:
        return best_offset, float(best_speed), best
    return best_offset, float(best_speed)


def rubberband_pitch_st(pitch_ratio):     # consensus.py:355
    return -12.0 * math.log2(pitch_ratio)


# ------------------------------------------------------------------ spectral.py
SPECTRAL_BANDS = (("sub_bass", 20, 80), ("bass", 80, 250), ("midrange", 250, 2000),   # spectral.py:70-74
                  ("presence", 2000, 6000), ("brilliance", 6000, 20000))


def spectral_analyze(y, sr, detail=False):
    """spectral.py:38-103 on an already-decoded mono f32 signal at its native rate (the
    reference loads with sr=None, :52).  Returns the SpectralStats fields as a dict; with
    detail=True also the per-frame / per-bin intermediates the engine is checked on."""
    y = np.asarray(y, dtype=np.float32)
    S = ncref.stft_mag(y)                                               # :63 (shared by :54-57)
    cen = ncref.spectral_centroid(S=S, sr=sr)[0]                        # :54
    rol = ncref.spectral_rolloff(S=S, sr=sr, roll_percent=0.85)[0]      # :55-57
    rms = ncref.rms_frames(y)                                           # :59 and :76 (same call)
    freqs = ncref.fft_frequencies(sr)                                   # :64
    out = {"centroid": float(np.mean(cen)), "rolloff": float(np.mean(rol)),
           "rms_mean": float(np.mean(rms)), "rms_variance": float(np.var(rms))}
    for name, lo, hi in SPECTRAL_BANDS:                                 # :66-74
        mask = (freqs >= lo) & (freqs < hi)
        out[name] = float(np.mean(S[mask, :])) if mask.any() else 0.0
    loud = rms[rms > np.percentile(rms, 75)]                            # :77-78
    out["decay_rate"] = float(np.mean(np.diff(loud))) if len(loud) > 1 else 0.0
    out["duration"] = ncref.get_duration(y, sr)                         # :80
    db = ncref.amplitude_to_db(S, ref=np.max)                           # :87-94
    favg = np.mean(db, axis=1)
    sig = favg > (np.max(favg) - 60.0)
    out["effective_bandwidth_hz"] = float(freqs[np.where(sig)[0][-1]]) if sig.any() else float(freqs[-1])
    if detail:
        return out, {"centroid": cen, "rolloff": rol, "rms": rms, "bin_db_mean": favg, "S": S}
    return out
