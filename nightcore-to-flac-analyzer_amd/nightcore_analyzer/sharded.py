"""Window-sharded analysis across ranks: one (nightcore, source) pair can span GPUs.

north_star: "the 10 s / 5 s-hop windows over both input files are the natural shard
unit: partition them across the GPUs with an RCCL gather of per-window estimates
over xGMI before consensus".  SURVEY.md §8(e) lays the split out; this module follows
it.  Every rank holds the same decoded pairs and derives the same host plan (silence
trim, windows, 20 s chunk pairs: ``engine.plan_batch``); then

  1. rank r runs the per-window stage (energy, onset, tempogram mean: K1-K5) on its
     contiguous block of windows;                        C1a: all-gather energies
  2. every rank applies the energy gate (io.py:115-126) to the whole batch; rank r
     tracks its source windows with start_bpm 120 (tempo.py:27-77, K6-K8);
                                                         C1b: all-gather window records
  3. every rank forms the nc prior of every pair from the gathered source records
     (median of valid source tempos x duration ratio, pipeline.py:174-183) and tracks
     its nightcore windows with their pair's prior;
     rank r also runs its contiguous block of 20 s chunk pairs (K9-K11, pitch.py:121-138);
                                                         C1c: all-gather window + chunk records
  4. the owner of each pair (pairs are blocked over ranks) runs the bootstraps
     (consensus.py:243-267, pitch.py:143-150), the hop-64 IBI pass of the pair's two
     files (tempo.py:120-173, consensus.py:270-312) and the host assembly (report,
     warnings, logs), then the finished results are gathered to every rank.

The records are fixed-size f64 rows (``all_gather_into_tensor``: RCCL over xGMI with the
"nccl" backend, CPU tensors with gloo); shards of unequal size are padded to the
largest one, and every gathered block carries its rank's error flag, so a failure on
one rank raises on every rank instead of leaving the others blocked in a collective.

The device work is behind a small stage interface (``DeviceStages``: libncgpu on this
rank's GPU).  The same orchestration runs over any object with that interface; the
multi-process CPU tests drive it with the oracle, so the exchange, the prior and the
consensus placement are tested without a GPU.  Every result equals the single-rank
``Engine.analyze`` result of the same batch.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import consensus as C
from .distributed import shard_range
from .engine import (ALIGN_MIN_OFFSET, CHUNK_SEC, HOP_LENGTH, IBI_HOP, MIN_BEATS, MIN_CHUNKS, REF_HZ, SR,
                     DeviceSignals, Engine, PairOutcome, Params, _Upload, assemble_pair, plan_batch)

# per-window record: energy_db, bpm, nbeats, tempo lag, decision margin
W_ENERGY, W_BPM, W_NBEATS, W_LAG, W_MARGIN = range(5)
W_FIELDS = 5
# per-chunk-pair record: lag, tuning (src, nc), mean chroma (src 12, nc 12), lag margin
CP_FIELDS = 3 + 24 + 1


class ShardError(RuntimeError):
    """Another rank of a window-sharded run failed (its own exception is raised there)."""


# ------------------------------------------------------------------------------ exchange
class Exchange:
    """Fixed-size f64 record gathers over the default (or given) process group."""

    def __init__(self, group=None):
        self.group = group
        self.on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        backend = dist.get_backend(group) if self.on else "gloo"
        self.dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    def gather_rows(self, local: np.ndarray, n_total: int, failed: Optional[BaseException]) -> np.ndarray:
        """Rank r contributes rows [lo_r, hi_r) of an n_total x k table (lo/hi from
        shard_range); returns the whole table on every rank.  One all_gather_into_tensor of
        (largest shard + 1 flag row) x k f64 per rank."""
        k = local.shape[1]
        if not self.on or self.world == 1:
            if failed is not None:
                raise failed
            return np.ascontiguousarray(local, np.float64)
        S = -(-n_total // self.world)
        mine = np.zeros((S + 1, k), np.float64)
        mine[:local.shape[0]] = local
        mine[S, 0] = 1.0 if failed is not None else 0.0
        t = torch.from_numpy(mine).to(self.dev)
        out = torch.empty((self.world * (S + 1), k), dtype=torch.float64, device=self.dev)
        dist.all_gather_into_tensor(out, t, group=self.group)
        allr = out.cpu().numpy().reshape(self.world, S + 1, k)
        bad = [r for r in range(self.world) if allr[r, S, 0] != 0.0]
        if failed is not None:
            raise failed
        if bad:
            raise ShardError(f"window-sharded analysis failed on rank(s) {bad}")
        rows = []
        for r in range(self.world):
            lo, hi = shard_range(n_total, self.world, r)
            rows.append(allr[r, :hi - lo])
        return np.concatenate(rows, axis=0) if rows else np.zeros((0, k))

    def gather_objects(self, local: list) -> list:
        if not self.on or self.world == 1:
            return list(local)
        buf: List[Optional[list]] = [None] * self.world
        dist.all_gather_object(buf, local, group=self.group)
        out: list = []
        for part in buf:
            out.extend(part)
        return out


def _try(fn, *args):
    try:
        return fn(*args), None
    except BaseException as exc:       # noqa: BLE001 - re-raised after the collective
        return None, exc


# ------------------------------------------------------------------------------ device stages
class DeviceStages:
    """The stage operations of one rank on its GPU (libncgpu), over signals resident in
    HBM: files nc_0, src_0, nc_1, src_1, ... in one buffer."""

    def __init__(self, eng: Engine, signals: DeviceSignals):
        self.eng = eng
        self.sig = signals
        self.off = signals.off
        self.length = signals.length
        self._win = None

    def trim(self, p: Params) -> Tuple[np.ndarray, np.ndarray]:
        return self.eng._trim_all(self.sig, p)

    def align(self, start: np.ndarray, end: np.ndarray) -> List[Tuple[float, float]]:
        o, s = self.sig.off, start
        return self.eng.align_offsets(self.sig.buf, o[1::2] + s[1::2], end[1::2] - s[1::2], o[0::2] + s[0::2],
                                      end[0::2] - s[0::2])

    def windows(self, win_abs: np.ndarray, win_n: int) -> np.ndarray:
        """Per-window stage (nc_window_stage: energy, onset, tempogram mean) -> energies."""
        eng, n = self.eng, len(win_abs)
        if n == 0:
            self._win = None
            return np.zeros(0)
        T = 1 + win_n // HOP_LENGTH
        acw = int(int(8.0 * SR) // HOP_LENGTH)
        off = torch.from_numpy(np.ascontiguousarray(win_abs, np.int64)).to(eng.dev)
        onset = torch.empty(n * T, dtype=torch.float32, device=eng.dev)
        tg = torch.empty(n * acw, dtype=torch.float64, device=eng.dev)
        en = torch.empty(n, dtype=torch.float64, device=eng.dev)
        ws = eng.workspace("win", eng.ctx.lib.nc_window_stage_workspace_bytes(eng.ctx.h, n, win_n, HOP_LENGTH))
        eng.call("nc_window_stage", self.sig.buf.data_ptr(), off.data_ptr(), None, n, win_n, HOP_LENGTH,
                 onset.data_ptr(), tg.data_ptr(), en.data_ptr(), ws.data_ptr(), ws.numel(), eng.stream())
        self._win = dict(onset=onset, tg=tg, T=T, acw=acw)
        return en.cpu().numpy()

    def tempo(self, sel: np.ndarray, start_bpm: np.ndarray) -> np.ndarray:
        """beat_track of the selected local windows (indices into the last windows() call)
        with per-window start_bpm -> [n_sel, (bpm, nbeats, lag, margin)]."""
        eng, n = self.eng, len(sel)
        out = np.zeros((n, 4), np.float64)
        if n == 0:
            return out
        w = self._win
        T, acw = w["T"], w["acw"]
        up = _Upload()
        up.add("on_off", np.asarray(sel, np.int64) * T, np.int64)
        up.add("on_len", np.full(n, T), np.int32)
        up.add("start", start_bpm, np.float64)
        d = up.commit(eng.dev)
        tg = w["tg"].view(-1, acw)[torch.from_numpy(np.asarray(sel, np.int64)).to(eng.dev)].contiguous()
        bpm = torch.zeros(n, dtype=torch.float64, device=eng.dev)
        lag = torch.zeros(n, dtype=torch.int32, device=eng.dev)
        nb = torch.zeros(n, dtype=torch.int32, device=eng.dev)
        mg = torch.zeros(n, dtype=torch.float64, device=eng.dev)
        ws = eng.workspace("beats", eng.ctx.lib.nc_tempo_beats_workspace_bytes(n * T))   # any window length
        eng.call("nc_tempo_beats", w["onset"].data_ptr(), d["on_off"].data_ptr(), d["on_len"].data_ptr(), n, T,
                 tg.data_ptr(), acw, d["start"].data_ptr(), None, None, HOP_LENGTH, 1, bpm.data_ptr(),
                 lag.data_ptr(), nb.data_ptr(), mg.data_ptr(), None, n * T, ws.data_ptr(), ws.numel(), eng.stream())
        out[:, 0] = bpm.cpu().numpy()
        out[:, 1] = nb.cpu().numpy()
        out[:, 2] = lag.cpu().numpy()
        out[:, 3] = mg.cpu().numpy()
        return out

    def chunks(self, chunk_off: Sequence[int], chunk_len: Sequence[int]) -> np.ndarray:
        """Mean chroma of every chunk (files interleaved src, nc per chunk pair) and the
        pair lags -> [n_pairs, CP_FIELDS]."""
        eng, n = self.eng, len(chunk_off)
        out = np.zeros((n // 2, CP_FIELDS), np.float64)
        if n == 0:
            return out
        up = _Upload()
        up.add("off", chunk_off, np.int64)
        up.add("len", chunk_len, np.int64)
        up.add("si", np.arange(0, n, 2), np.int32)
        up.add("ni", np.arange(1, n, 2), np.int32)
        d = up.commit(eng.dev)
        chroma = torch.empty(n * 12, dtype=torch.float32, device=eng.dev)
        tun = torch.empty(n, dtype=torch.float32, device=eng.dev)
        lag = torch.empty(n // 2, dtype=torch.int32, device=eng.dev)
        tot = int(np.sum(chunk_len))
        ws = eng.workspace("chroma", eng.ctx.lib.nc_chroma_workspace_bytes(eng.ctx.h, n, tot))
        eng.call("nc_chroma_mean", self.sig.buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(), n, tot,
                 int(max(chunk_len)), chroma.data_ptr(), tun.data_ptr(), None, ws.data_ptr(), ws.numel(),
                 eng.stream())
        mg = torch.empty(n // 2, dtype=torch.float64, device=eng.dev)
        eng.call("nc_chroma_lag_margin", chroma.data_ptr(), d["si"].data_ptr(), d["ni"].data_ptr(), n // 2,
                 lag.data_ptr(), mg.data_ptr(), eng.stream())
        out[:, 0] = lag.cpu().numpy()
        t = tun.cpu().numpy().reshape(-1, 2)
        out[:, 1:3] = t
        out[:, 3:27] = chroma.cpu().numpy().reshape(-1, 24)
        out[:, 27] = mg.cpu().numpy()
        return out

    def bootstrap(self, jobs, seed: int):
        return self.eng.bootstrap(jobs, seed=seed) if jobs else []

    def ibi(self, f_off: np.ndarray, f_len: np.ndarray, start_bpm: np.ndarray):
        """estimate_ibis_global of each file span -> (ibis (array, or None under 4), IBI
        counts, beat counts, tempo lags)."""
        eng, n = self.eng, len(f_off)
        if n == 0:
            z = np.zeros(0, np.int64)
            return [], z, z, z
        up = _Upload()
        up.add("off", f_off, np.int64)
        up.add("len", f_len, np.int64)
        up.add("start", start_bpm, np.float64)
        d = up.commit(eng.dev)
        core = eng.ibi_core(self.sig.buf, d["off"], d["len"], np.asarray(f_len, np.int64), d["start"],
                            torch.arange(n, dtype=torch.int32, device=eng.dev))
        vals, nibi = core["ibis"].cpu().numpy(), core["nibi"].cpu().numpy()
        fb = core["fbase_h"]
        ibis = [vals[fb[i]:fb[i] + nibi[i]].copy() if nibi[i] >= 4 else None for i in range(n)]
        return ibis, nibi, core["nbeats"].cpu().numpy(), core["lag"].cpu().numpy()


# ------------------------------------------------------------------------------ orchestration
def _gate(energy: np.ndarray, w0, w1, threshold_db: float) -> np.ndarray:
    """io.energy_gate (io.py:115-126) for every file: keep energy >= file max + threshold."""
    act = np.zeros(len(energy), bool)
    for a, b in zip(w0, w1):
        if b > a:
            e = energy[a:b]
            act[a:b] = e >= e.max() + threshold_db
    return act


def analyze_sharded(stages, p: Optional[Params] = None, group=None) -> List[PairOutcome]:
    """pipeline.run's analysis of every pair held by ``stages`` with the windows and chunk
    pairs split over the ranks of ``group``; every rank returns all outcomes in pair
    order (module docstring)."""
    p = p or Params()
    ex = Exchange(group)
    rank, world = ex.rank, ex.world
    start, end = stages.trim(p) if p.silence_strip_db is not None else \
        (np.zeros(len(stages.off), np.int64), np.asarray(stages.length, np.int64).copy())
    align = stages.align(start, end) if (p.auto_align and p.src_trim_sec == 0.0) else None
    pl = plan_batch(stages.off, stages.length, start, end, p, align)
    B, n_win, n_src_w = pl.B, pl.n_win, pl.n_src_w
    w0, w1 = pl.w0, pl.w1
    pair_of = np.zeros(max(1, n_win), np.int64)            # pair of each window
    for b in range(B):
        pair_of[w0[2 * b]:w1[2 * b]] = b
        pair_of[w0[2 * b + 1]:w1[2 * b + 1]] = b

    # 1. per-window stage on this rank's block; C1a
    lo, hi = shard_range(n_win, world, rank)
    rec = np.zeros((hi - lo, W_FIELDS), np.float64)
    e_loc, err = _try(stages.windows, pl.win_abs[lo:hi], pl.win_n)
    if err is None:
        rec[:, W_ENERGY] = e_loc
    energy = ex.gather_rows(rec[:, :1], n_win, err)[:, 0]
    active = _gate(energy, w0, w1, p.energy_gate_db)

    # 2. source windows with start_bpm 120; C1b
    src_sel = np.array([i - lo for i in range(lo, min(hi, n_src_w)) if active[i]], np.int64)
    r, err = _try(stages.tempo, src_sel, np.full(len(src_sel), 120.0))
    if err is None and len(src_sel):
        rec[src_sel, W_BPM:] = r
    table = ex.gather_rows(rec, n_win, err)

    # 3. nc prior of every pair (pipeline.py:174-183), nightcore windows; chunk pairs; C1c
    prior = np.full(B, 120.0)
    for b in range(B):
        valid = [table[w, W_BPM] for w in range(w0[2 * b + 1], w1[2 * b + 1])
                 if active[w] and table[w, W_NBEATS] >= MIN_BEATS]
        nc_dur, src_dur = pl.f_len[2 * b] / SR, pl.f_len[2 * b + 1] / SR
        if valid and nc_dur > 0 and src_dur > 0:
            prior[b] = C._median(valid) * (src_dur / nc_dur)
    nc_sel = np.array([i - lo for i in range(max(lo, n_src_w), hi) if active[i]], np.int64)
    r, err = _try(stages.tempo, nc_sel, prior[pair_of[nc_sel + lo]] if len(nc_sel) else np.zeros(0))
    if err is None and len(nc_sel):
        rec[nc_sel, W_BPM:] = r
    table = ex.gather_rows(rec, n_win, err)
    clo, chi = shard_range(pl.n_cp, world, rank)
    cp, err = _try(stages.chunks, pl.chunk_off[2 * clo:2 * chi], pl.chunk_len[2 * clo:2 * chi])
    cps = ex.gather_rows(cp if err is None else np.zeros((chi - clo, CP_FIELDS)), pl.n_cp, err)

    # 4. consensus on the owner of each pair
    plo, phi = shard_range(B, world, rank)
    outs, err = _try(_consensus, stages, p, pl, align, active, energy, table, prior, cps, plo, phi)
    ex.gather_rows(np.zeros((phi - plo, 1)), B, err)     # fail together before the result gather
    for o in outs:
        o.logs                          # render the deferred log lines (plain strings travel)
    return ex.gather_objects(outs)


def _consensus(stages, p: Params, pl, align, active, energy, table, prior, cps, plo: int, phi: int) -> list:
    """Bootstraps, IBI pass and host assembly of pairs [plo, phi) (this rank's)."""
    B, n_cp = pl.B, pl.n_cp
    w0, w1 = pl.w0, pl.w1
    lags = [int(v) for v in cps[:, 0]] if n_cp else []
    shifts = np.array([l / 3.0 for l in lags], np.float64)                       # pitch.py:95
    nc_hz = np.array([REF_HZ * (2.0 ** (s / 12.0)) for s in shifts], np.float64)  # pitch.py:161-164
    src_hz = np.full(n_cp, REF_HZ)
    n_pj = len(pl.pair_chunks)
    nj = B + n_pj
    bout = np.full(3 * nj, np.nan)
    sout = np.full(3 * max(1, n_pj), np.nan)
    bpm, nbeats = table[:, W_BPM], table[:, W_NBEATS]

    def valid_tempos(f):
        return [bpm[w] for w in range(w0[f], w1[f]) if active[w] and nbeats[w] >= MIN_BEATS and bpm[w] > 0
                and math.isfinite(bpm[w])]

    tempo_jobs, pitch_jobs, shift_jobs = [], [], []
    for b in range(plo, phi):
        nt, st = valid_tempos(2 * b), valid_tempos(2 * b + 1)
        if len(nt) >= C.MIN_VALID and len(st) >= C.MIN_VALID:
            tempo_jobs.append((b, (np.array(nt), np.array(st))))
        if n_pj:
            c0, c1 = pl.pair_chunks[b]
            if c1 - c0 >= C.MIN_VALID:
                pitch_jobs.append((B + b, (nc_hz[c0:c1], src_hz[c0:c1])))
            if c1 - c0 >= MIN_CHUNKS:
                shift_jobs.append((b, (shifts[c0:c1], None)))
    for jobs, out, n, seed in ((tempo_jobs + pitch_jobs, bout, nj, 42), (shift_jobs, sout, max(1, n_pj), 0)):
        res = stages.bootstrap([j for _, j in jobs], seed)
        for (i, _), (pt, (lo_, hi_)) in zip(jobs, res):
            out[i], out[n + i], out[2 * n + i] = pt, lo_, hi_

    ibi = None
    if p.compute_ibi:
        # hop-64 pass of the owned pairs' files (nc with the pair prior, src with 120)
        files = [f for b in range(plo, phi) for f in (2 * b, 2 * b + 1)]
        sb = np.array([prior[f // 2] if f % 2 == 0 else 120.0 for f in files])
        ibis, nibi, nb, lg = stages.ibi(pl.f_off[files], pl.f_len[files], sb)
        nF = 2 * B
        ibi = dict(nibi=np.zeros(nF, np.int64), nbeats=np.zeros(nF, np.int64), lag=np.zeros(nF, np.int64),
                   out=np.full(3 * B, np.nan))
        for k, f in enumerate(files):
            ibi["nibi"][f] = nibi[k]
            ibi["nbeats"][f], ibi["lag"][f] = nb[k], lg[k]
        jobs = [(b, (ibis[2 * (b - plo) + 1], ibis[2 * (b - plo)])) for b in range(plo, phi)
                if ibis[2 * (b - plo)] is not None and ibis[2 * (b - plo) + 1] is not None]
        for (b, _), (pt, (lo_, hi_)) in zip(jobs, stages.bootstrap([j for _, j in jobs], 42)):
            ibi["out"][b], ibi["out"][B + b], ibi["out"][2 * B + b] = pt, lo_, hi_

    pvals = np.concatenate([shifts, nc_hz, src_hz]) if n_cp else np.zeros(3)
    tun = cps[:, 1:3].reshape(-1).astype(np.float32) if n_cp else np.zeros(0, np.float32)
    chroma = cps[:, 3:27].reshape(-1).astype(np.float32) if n_cp else np.zeros(0, np.float32)
    h = {"active_l": active.tolist(), "energy": energy, "clag_l": lags, "pvals": pvals, "pvals_l": pvals.tolist(),
         "sout_l": sout.tolist(), "bout_l": bout.tolist(), "tuning": tun, "chroma": chroma,
         "cmargin": cps[:, 27].copy() if n_cp else np.zeros(0),
         "bpm_l": bpm.tolist(), "nbeats_l": [int(v) for v in nbeats], "prior_l": prior.tolist(),
         "margin": table[:, W_MARGIN]}
    starts_l = [s.tolist() for s in pl.starts]
    w0l, w1l = [int(v) for v in w0], [int(v) for v in w1]
    return [assemble_pair(b, p, h, ibi, starts_l, w0l, w1l, pl.f_len, pl.strip_len, pl.lead, pl.trail,
                          pl.intro[b], pl.win_n, pl.pair_chunks, n_cp, nj, n_pj, align[b] if align else None)
            for b in range(plo, phi)]


def run_window_sharded(pairs: Sequence[Tuple[np.ndarray, np.ndarray]], p: Optional[Params] = None,
                       group=None, device: Optional[int] = None) -> List[PairOutcome]:
    """Upload every (nc, src) pair to this rank's GPU and run ``analyze_sharded``."""
    from .engine import get_engine
    eng = get_engine(device)
    flat = []
    for nc, src in pairs:
        flat += [np.asarray(nc, np.float32), np.asarray(src, np.float32)]
    return analyze_sharded(DeviceStages(eng, eng.upload_signals(flat)), p, group)
