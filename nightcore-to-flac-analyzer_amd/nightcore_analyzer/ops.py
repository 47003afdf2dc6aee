"""Device operations behind the reference's module-level functions (io / tempo /
pitch / xcorr), for callers that use those functions directly instead of
``pipeline.run`` (the reference's workflow does: workflow.py:617, 678, 797).
Every function uploads its arrays once and runs libncgpu kernels; results come
back in the reference's Python types.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .engine import SR, Engine, _Upload, percentile_params, seed_state

HOP = 512


def trim_bounds(eng: Engine, audios: Sequence[np.ndarray], top_db: float) -> List[Tuple[int, int]]:
    """librosa.effects.trim bounds (io.py:76) for each array."""
    sig = eng.upload_signals(audios)
    up = _Upload()
    up.add("off", sig.off, np.int64)
    up.add("len", sig.length, np.int64)
    d = up.commit(eng.dev)
    n = sig.n_files
    tot = int(np.sum(1 + sig.length // 512))
    lens = np.ascontiguousarray(sig.length, np.int64)
    ws = eng.workspace("trim", eng.ctx.lib.nc_trim_workspace_bytes(lens.ctypes.data, n))
    se = torch.empty(2 * n, dtype=torch.int64, device=eng.dev)
    eng.call("nc_trim_bounds", sig.buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(), n, tot,
             float(top_db), se[:n].data_ptr(), se[n:].data_ptr(), ws.data_ptr(), ws.numel(), eng.stream())
    h = se.cpu().numpy()
    return [(int(h[i]), int(h[n + i])) for i in range(n)]


def window_energies(eng: Engine, audio: np.ndarray, starts: np.ndarray, win_len: int) -> np.ndarray:
    """io._rms_db (io.py:38-40) of audio[s:s+win_len] for every start."""
    if len(starts) == 0:
        return np.zeros(0)
    sig = eng.upload_signals([audio])
    off = torch.tensor(np.asarray(starts, np.int64) + sig.off[0], device=eng.dev)
    out = torch.empty(len(starts), dtype=torch.float64, device=eng.dev)
    eng.call("nc_window_energy", sig.buf.data_ptr(), off.data_ptr(), len(starts), int(win_len), out.data_ptr(),
             eng.stream())
    return out.cpu().numpy()


def window_tempos(eng: Engine, audios: Sequence[np.ndarray], start_bpms: Sequence[float],
                  details: Optional[list] = None) -> List[Optional[float]]:
    """tempo.estimate_tempo (tempo.py:27-77) for each window array."""
    res: List[Optional[float]] = [None] * len(audios)
    by_len: dict = {}
    for i, a in enumerate(audios):
        by_len.setdefault(len(a), []).append(i)
    acw = int(int(8.0 * eng.sr) // HOP)     # the tempogram window of the engine's rate
    for L, idx in by_len.items():
        if L == 0:
            continue
        n = len(idx)
        T = 1 + L // HOP
        sig = eng.upload_signals([audios[i] for i in idx])
        up = _Upload()
        up.add("off", sig.off, np.int64)
        up.add("on_off", np.arange(n, dtype=np.int64) * T, np.int64)
        up.add("on_len", np.full(n, T), np.int32)
        up.add("start", [start_bpms[i] for i in idx], np.float64)
        d = up.commit(eng.dev)
        onset = torch.empty(n * T, dtype=torch.float32, device=eng.dev)
        tg = torch.empty(n * acw, dtype=torch.float64, device=eng.dev)
        en = torch.empty(n, dtype=torch.float64, device=eng.dev)
        wsb = eng.ctx.lib.nc_window_stage_workspace_bytes(eng.ctx.h, n, L, HOP)
        ws = eng.workspace("win", wsb)
        st = eng.stream()
        eng.call("nc_window_stage", sig.buf.data_ptr(), d["off"].data_ptr(), None, n, L, HOP, onset.data_ptr(),
                 tg.data_ptr(), en.data_ptr(), ws.data_ptr(), ws.numel(), st)
        bpm = torch.zeros(n, dtype=torch.float64, device=eng.dev)
        lag = torch.zeros(n, dtype=torch.int32, device=eng.dev)
        nb = torch.zeros(n, dtype=torch.int32, device=eng.dev)
        mg = torch.zeros(n, dtype=torch.float64, device=eng.dev)
        wsb2 = eng.ctx.lib.nc_tempo_beats_workspace_bytes(n * T)
        ws2 = eng.workspace("beats", wsb2)
        eng.call("nc_tempo_beats", onset.data_ptr(), d["on_off"].data_ptr(), d["on_len"].data_ptr(), n, T,
                 tg.data_ptr(), acw, d["start"].data_ptr(), None, None, HOP, 1, bpm.data_ptr(), lag.data_ptr(),
                 nb.data_ptr(), mg.data_ptr(), None, n * T, ws2.data_ptr(), ws2.numel(), st)
        b_h, n_h = bpm.cpu().numpy(), nb.cpu().numpy()
        for k, i in enumerate(idx):
            res[i] = float(b_h[k]) if n_h[k] >= 4 else None
        if details is not None:
            details.append(dict(idx=idx, lag=lag.cpu().numpy(), nbeats=n_h, margin=mg.cpu().numpy()))
    return res


def ibis(eng: Engine, ys: Sequence[np.ndarray], start_bpms: Sequence[float], hop: int = 64,
         min_ibis: int = 4) -> List[Optional[np.ndarray]]:
    """tempo.estimate_ibis_global (tempo.py:120-173) for each signal."""
    sig = eng.upload_signals(ys)
    up = _Upload()
    up.add("off", sig.off, np.int64)
    up.add("len", sig.length, np.int64)
    up.add("start", list(start_bpms), np.float64)
    d = up.commit(eng.dev)
    core = eng.ibi_core(sig.buf, d["off"], d["len"], sig.length, d["start"],
                        torch.arange(len(ys), dtype=torch.int32, device=eng.dev), hop=hop, min_ibis=min_ibis)
    vals = core["ibis"].cpu().numpy()
    nibi = core["nibi"].cpu().numpy()
    fb = core["fbase_h"]
    return [vals[fb[i]:fb[i] + nibi[i]].copy() if nibi[i] > 0 else None for i in range(len(ys))]


def chroma_means(eng: Engine, audios: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray, torch.Tensor]:
    """pitch._mean_chroma (pitch.py:55-64) of each array -> ([n,12] f32, tuning[n], device chroma)."""
    sig = eng.upload_signals(audios)
    n = sig.n_files
    up = _Upload()
    up.add("off", sig.off, np.int64)
    up.add("len", sig.length, np.int64)
    d = up.commit(eng.dev)
    out = torch.empty(n * 12, dtype=torch.float32, device=eng.dev)
    tun = torch.empty(n, dtype=torch.float32, device=eng.dev)
    tot = int(sig.length.sum())
    ws = eng.workspace("chroma", eng.ctx.lib.nc_chroma_workspace_bytes(eng.ctx.h, n, tot))
    eng.call("nc_chroma_mean", sig.buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(), n, tot,
             int(sig.length.max()), out.data_ptr(), tun.data_ptr(), None, None, ws.data_ptr(), ws.numel(), eng.stream())
    return out.cpu().numpy().reshape(n, 12), tun.cpu().numpy(), out


def chroma_lags(eng: Engine, chroma_dev: torch.Tensor, src_idx: Sequence[int], nc_idx: Sequence[int]) -> List[int]:
    """pitch._cyclic_xcorr_peak (pitch.py:67-85) for each (src, nc) chroma row pair."""
    n = len(src_idx)
    si = torch.tensor(list(src_idx), dtype=torch.int32, device=eng.dev)
    ni = torch.tensor(list(nc_idx), dtype=torch.int32, device=eng.dev)
    lag = torch.empty(max(1, n), dtype=torch.int32, device=eng.dev)
    eng.call("nc_chroma_lag", chroma_dev.data_ptr(), si.data_ptr(), ni.data_ptr(), n, lag.data_ptr(), eng.stream())
    return lag.cpu().numpy()[:n].astype(int).tolist()


def xcorr_peaks(eng: Engine, src: np.ndarray, nc: np.ndarray) -> List[int]:
    """pitch._cyclic_xcorr_peak (pitch.py:67-85) for rows of [pairs, n] (any n >= 1)."""
    a = np.ascontiguousarray(src, np.float32)
    b = np.ascontiguousarray(nc, np.float32)
    n_pairs, n = a.shape
    d = torch.from_numpy(np.concatenate([a.reshape(-1), b.reshape(-1)])).to(eng.dev)
    lag = torch.empty(max(1, n_pairs), dtype=torch.int32, device=eng.dev)
    eng.call("nc_xcorr_peak", d[:a.size].data_ptr(), d[a.size:].data_ptr(), n, n_pairs, lag.data_ptr(), eng.stream())
    return lag.cpu().numpy()[:n_pairs].astype(int).tolist()


def xcorr_speed(eng: Engine, ya: np.ndarray, yb: np.ndarray, sr: int = SR, n_windows: int = 20,
                window_sec: float = 3.0, search_range: float = 0.05,
                skip_edges: float = 0.10) -> Tuple[float, float]:
    """The search of xcorr.estimate_speed_xcorr (xcorr.py:95-162) on decoded arrays."""
    min_len = min(len(ya), len(yb))
    s, e = int(min_len * skip_edges), int(min_len * (1.0 - skip_edges))
    ya, yb = np.asarray(ya, np.float32)[s:e], np.asarray(yb, np.float32)[s:e]
    win = int(window_sec * sr)
    search = int(search_range * len(yb))
    stride = max(1, win // 4)
    if len(ya) < win or len(yb) < win:
        return 1.0, 0.0
    sig = eng.upload_signals([ya, yb])
    oa, ob = int(sig.off[0]), int(sig.off[1])
    ia, ib, sw, c0, c1, pa_l, pb_l, exp_l = [], [], [], [], [], [], [], []
    for pa in np.linspace(0, len(ya) - win, n_windows).astype(int):
        pa = int(pa)
        exp_pb = int(pa * len(yb) / len(ya))
        lo, hi = max(0, exp_pb - search), min(len(yb) - win, exp_pb + search)
        if lo >= hi:
            continue
        sw.append(len(ia))
        ia.append(oa + pa)
        ib.append(oa + pa)
        pb_l.append(pa)
        c0.append(len(ia))
        for pb in range(lo, hi, stride):
            ia.append(oa + pa)
            ib.append(ob + pb)
            pb_l.append(pb)
        c1.append(len(ia))
        pa_l.append(pa)
        exp_l.append(exp_pb)
    nw = len(sw)
    if nw == 0:
        return 1.0, 0.0
    up = _Upload()
    up.add("ia", ia, np.int64)
    up.add("ib", ib, np.int64)
    up.add("w0", [0], np.int32)
    up.add("w1", [nw], np.int32)
    up.add("sw", sw, np.int32)
    up.add("c0", c0, np.int32)
    up.add("c1", c1, np.int32)
    up.add("pa", pa_l, np.int64)
    up.add("pb", pb_l, np.int64)
    up.add("exp", exp_l, np.int64)
    d = up.commit(eng.dev)
    n_items = len(ia)
    scratch = torch.empty(2 * n_items + 2, dtype=torch.float64, device=eng.dev)
    out = torch.empty(2, dtype=torch.float64, device=eng.dev)
    eng.call("nc_xcorr_search", sig.buf.data_ptr(), d["ia"].data_ptr(), d["ib"].data_ptr(), n_items, win,
             scratch[:n_items].data_ptr(), scratch[n_items:2 * n_items].data_ptr(), d["w0"].data_ptr(),
             d["w1"].data_ptr(), d["sw"].data_ptr(), d["c0"].data_ptr(), d["c1"].data_ptr(), d["pa"].data_ptr(),
             d["pb"].data_ptr(), d["exp"].data_ptr(), 1, out[0:1].data_ptr(), out[1:2].data_ptr(), eng.stream())
    o = out.cpu().numpy()
    return float(o[0]), float(o[1])


def shift_bootstrap(eng: Engine, shifts: np.ndarray) -> Tuple[float, float]:
    """pitch.py:143-150: CI of the median chunk shift, rng = default_rng(0)."""
    (_, ci), = eng.bootstrap([(np.asarray(shifts, np.float64), None)], seed=0)
    return ci


# ------------------------------------------------------------------ load-time resampler
def poly_plan(up: int, down: int, max_in: int):
    """scipy.signal.resample_poly's filter and offsets for ratio up/down (reduced), sized for
    inputs up to max_in samples: (up, down, h padded to a multiple of up (f64), pre_remove).
    Trailing zero taps beyond what a shorter input needs leave every sum unchanged."""
    import math
    from scipy.signal import firwin
    g = math.gcd(int(up), int(down))
    up, down = int(up) // g, int(down) // g
    max_rate = max(up, down)
    half_len = 10 * max_rate
    h = firwin(2 * half_len + 1, 1.0 / max_rate, window=("kaiser", 5.0)) * up
    n_pre_pad = down - half_len % down
    pre_remove = (half_len + n_pre_pad) // down
    n_out = -(-max_in * up // down)

    def out_len(len_h, n_in):        # scipy.signal._upfirdn_apply._output_len
        n = n_in + (len_h + (-len_h % up)) // up - 1
        return -(-n * up // down)
    post = 0
    while out_len(len(h) + n_pre_pad + post, max_in) < n_out + pre_remove:
        post += 1
    h = np.concatenate([np.zeros(n_pre_pad), h, np.zeros(post)])
    h = np.concatenate([h, np.zeros(-len(h) % up)])
    return up, down, h, pre_remove


def resample_poly(eng: Engine, arrays: Sequence[np.ndarray], up: int, down: int) -> List[np.ndarray]:
    """float32(scipy.signal.resample_poly(float64(x), up, down)) for each array, on the GPU
    (nc_resample_poly; bit-identical to scipy).  The load-time resampler of io.load_audio."""
    arrays = [np.asarray(a, np.float32) for a in arrays]
    if not arrays:
        return []
    up, down, h, pre = poly_plan(up, down, max(len(a) for a in arrays))
    if up == down == 1:
        return [a.copy() for a in arrays]
    sig = eng.upload_signals(arrays)
    n_out = np.array([-(-len(a) * up // down) for a in arrays], np.int64)
    o_off = np.zeros(len(arrays), np.int64)
    o_off[1:] = np.cumsum(n_out)[:-1]
    up_ = _Upload()
    up_.add("in_off", sig.off, np.int64)
    up_.add("in_len", sig.length, np.int64)
    up_.add("out_off", o_off, np.int64)
    up_.add("out_len", n_out, np.int64)
    up_.add("h", h, np.float64)
    d = up_.commit(eng.dev)
    y = torch.empty(max(1, int(n_out.sum())), dtype=torch.float32, device=eng.dev)
    eng.call("nc_resample_poly", sig.buf.data_ptr(), d["in_off"].data_ptr(), d["in_len"].data_ptr(), len(arrays),
             y.data_ptr(), d["out_off"].data_ptr(), d["out_len"].data_ptr(), int(n_out.max()), d["h"].data_ptr(),
             len(h), up, down, pre, eng.stream())
    hy = y.cpu().numpy()
    return [hy[o:o + n].copy() for o, n in zip(o_off, n_out)]
