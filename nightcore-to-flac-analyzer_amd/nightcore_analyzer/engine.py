"""The MI355X engine: batched, stream-ordered execution of ``pipeline.run`` for
many (nightcore, source) pairs at once on one GPU.

Flow for a batch of B pairs (2B files), everything between the two host
synchronisations running on one HIP stream:

  H2D signals (one buffer) -> nc_trim_bounds ............................ sync 1
  host plan: src trim, windows (io.slice_windows), 20 s chunks (pitch.py:121-138)
  H2D plan (one buffer)
  nc_window_stage (all windows: energy, onset, tempogram mean)
  nc_energy_gate -> nc_tempo_beats(src, prior 120) -> nc_tempo_prior
  -> nc_tempo_beats(nc, per-pair prior) -> nc_collect_valid
  nc_chroma_mean -> nc_chroma_lag -> nc_pitch_hz            (compute_pitch)
  nc_bootstrap_ratio (tempo + pitch, seed 42; chunk shifts, seed 0)
  nc_ibi_onset -> nc_ibi_tempogram -> nc_tempo_beats(hop 64) -> nc_ibi_from_beats
  -> nc_bootstrap_ratio (IBI)                                (compute_ibi)
  D2H results ............................................................ sync 2
  host: AnalysisResult assembly (classification, Rubber Band, warnings, logs)

The host never touches audio samples after the upload; there is no CPU path.
"""
from __future__ import annotations

import gc
import logging
import math
import os
import threading
import time
import weakref
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native
from . import consensus as C

SR = 22050
HOP_LENGTH = 512
IBI_HOP = 64
MIN_BEATS = 4
CHUNK_SEC = 20.0
MIN_CHUNKS = 3
REF_HZ = 440.0
ALIGN_SR, ALIGN_HOP = 11025, 512                                   # xcorr.py:45-46
ALIGN_SPEED_LO, ALIGN_SPEED_HI, ALIGN_N_SPEEDS = 1.03, 1.50, 30    # xcorr.py:47-49
ALIGN_MAX_OFFSET, ALIGN_MIN_OFFSET = 120.0, 1.0                   # xcorr.py:50-51
_ALIGN = 64


# ------------------------------------------------------------------------------ helpers
def seed_state(seed: int) -> List[int]:
    """PCG64 state of np.random.default_rng(seed) as 4 uint64 (state hi/lo, inc hi/lo)."""
    st = np.random.PCG64(seed).state["state"]
    s, inc = int(st["state"]), int(st["inc"])
    m = (1 << 64) - 1
    return [(s >> 64) & m, s & m, (inc >> 64) & m, inc & m]


def h2d(arr, dtype, dev: torch.device) -> torch.Tensor:
    """Small host array -> device tensor through pinned memory, without a host sync."""
    a = np.ascontiguousarray(np.asarray(arr, dtype=dtype).reshape(-1))
    return torch.from_numpy(a).pin_memory().to(dev, non_blocking=True)


def percentile_params(n_boot: int, ci: float) -> Tuple[float, float, float, float]:
    """(virtual index, gamma) of np.percentile(.., alpha*100) and (1-alpha)*100, 'linear'."""
    alpha = (1.0 - ci) / 2.0
    out = []
    for q in (alpha * 100, (1.0 - alpha) * 100):
        quant = np.true_divide(np.float64(q), 100)
        virt = np.float64(n_boot - 1) * quant
        prev = np.floor(virt)
        out += [float(prev), float(virt - prev)]
    return tuple(out)


PEAK_SLOTS = 192   # piptrack peak slots per tuning frame (csrc/nc_piptrack.h kPeakSlots)
NEAR_TIE = 1e-3    # chroma-lag decisions closer than this (relative xcorr gap) are reported
TUNING_NEAR_TIE = 1  # tuning decisions whose histogram argmax leads by at most this many residuals
_logger = logging.getLogger("nightcore_analyzer")


class _GcPaused:
    """Python's cyclic collector paused for a host-heavy call (restored on exit): a generation-2
    pass over a long-lived process's objects costs milliseconds and lands at random inside it;
    the calls that use this create no reference cycles."""

    def __enter__(self):
        self.was = gc.isenabled()
        gc.disable()

    def __exit__(self, *exc):
        if self.was:
            gc.enable()


class _DevSpan:
    """A typed span of a device byte buffer as the native entry points take it: an address
    and a length.  Carving the pipeline's ~50 plan and result arrays as torch views costs a
    few microseconds of host time each (one group's launch spent ~0.25 ms there); a span is
    a plain address, sliced like a 1-D tensor, and becomes a tensor only on request (``t``)."""
    __slots__ = ("base", "addr", "n", "dtype", "isz")

    def __init__(self, base: torch.Tensor, addr: int, n: int, dtype: torch.dtype, isz: int):
        self.base, self.addr, self.n, self.dtype, self.isz = base, addr, n, dtype, isz

    def data_ptr(self) -> int:
        return self.addr

    def numel(self) -> int:
        return self.n

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, sl: slice) -> "_DevSpan":
        a, b, step = sl.indices(self.n)
        if step != 1:
            raise ValueError("a device span slices contiguously")
        return _DevSpan(self.base, self.addr + a * self.isz, max(0, b - a), self.dtype, self.isz)

    @property
    def t(self) -> torch.Tensor:
        o = self.addr - self.base.data_ptr()
        return self.base[o:o + self.n * self.isz].view(self.dtype)

    def fill_(self, v) -> None:
        self.t.fill_(v)


def _tensor(x):
    return x.t if isinstance(x, _DevSpan) else x


class _Upload:
    """Packs many small host arrays into one H2D copy; returns device views (torch views,
    or ``_DevSpan`` address spans with ``spans=True``)."""

    def __init__(self):
        self.parts: List[Tuple[str, np.ndarray]] = []

    def add(self, name: str, arr, dtype):
        a = np.ascontiguousarray(np.asarray(arr, dtype=dtype).reshape(-1))
        self.parts.append((name, a))

    def commit(self, dev: torch.device, spans: bool = False) -> Dict[str, torch.Tensor]:
        offs, total = [], 0
        for _, a in self.parts:
            total = (total + 15) & ~15
            offs.append(total)
            total += a.nbytes
        host = np.zeros(max(16, total), dtype=np.uint8)
        for (_, a), o in zip(self.parts, offs):
            host[o:o + a.nbytes] = a.view(np.uint8)
        # pinned staging + async copy: never waits for work already queued on the stream
        d = torch.from_numpy(host).pin_memory().to(dev, non_blocking=True)
        if spans:
            p0 = d.data_ptr()
            return {name: _DevSpan(d, p0 + o, max(1, a.size), _TORCH_DTYPE[a.dtype.str], a.itemsize)
                    for (name, a), o in zip(self.parts, offs)}
        out = {}
        for (name, a), o in zip(self.parts, offs):
            t = d[o:o + max(a.nbytes, a.itemsize)].view(_TORCH_DTYPE[a.dtype.str])
            out[name] = t[:max(1, a.size)]
        return out


_TORCH_DTYPE = {np.dtype(np.float64).str: torch.float64, np.dtype(np.float32).str: torch.float32,
                np.dtype(np.int64).str: torch.int64, np.dtype(np.int32).str: torch.int32,
                np.dtype(np.uint8).str: torch.uint8, np.dtype(np.uint64).str: torch.uint64}


class _Arena:
    """Many small device outputs carved from one byte buffer: one zero-fill on the
    stream instead of one per tensor, and one D2H copy into one pinned buffer."""

    def __init__(self):
        self.parts: List[Tuple[str, np.dtype, int]] = []
        self.host: Optional[torch.Tensor] = None

    def add(self, name: str, n: int, dtype) -> None:
        self.parts.append((name, np.dtype(dtype), max(1, int(n))))

    def commit(self, dev: torch.device, spans: bool = False) -> Dict[str, torch.Tensor]:
        self.offs, total = [], 0
        for _, dt, n in self.parts:
            total = (total + 15) & ~15
            self.offs.append(total)
            total += n * dt.itemsize
        self.nbytes = max(16, total)
        self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=dev)
        if spans:
            p0 = self.buf.data_ptr()
            return {name: _DevSpan(self.buf, p0 + o, n, _TORCH_DTYPE[dt.str], dt.itemsize)
                    for (name, dt, n), o in zip(self.parts, self.offs)}
        return {name: self.buf[o:o + n * dt.itemsize].view(_TORCH_DTYPE[dt.str])
                for (name, dt, n), o in zip(self.parts, self.offs)}

    def alloc_host(self) -> None:
        """Allocate the pinned host mirror now (before partial copies)."""
        if getattr(self, "host", None) is None:
            self.host = torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=True)

    def copy_parts(self, parts) -> None:
        """Queue D2H copies of some parts on the current stream, into the same places of the
        host mirror that to_host() fills: [name] or (name, first element, end element)."""
        self.alloc_host()
        idx = {name: i for i, (name, _, _) in enumerate(self.parts)}
        for part in parts:
            name, a, b = (part, 0, None) if isinstance(part, str) else part
            _, dt, n = self.parts[idx[name]]
            b = n if b is None else b
            o = self.offs[idx[name]]
            lo, hi = o + a * dt.itemsize, o + b * dt.itemsize
            if hi > lo:
                self.host[lo:hi].copy_(self.buf[lo:hi], non_blocking=True)

    def to_host(self) -> Tuple[torch.Tensor, Dict[str, np.ndarray]]:
        """Queue the D2H copy; the numpy views are valid once the stream reaches it."""
        self.alloc_host()
        host = self.host
        host.copy_(self.buf, non_blocking=True)
        hb = host.numpy()
        views = {name: hb[o:o + n * dt.itemsize].view(dt) for (name, dt, n), o in zip(self.parts, self.offs)}
        self.host_layout = (hb, {name: (views[name], o) for (name, _, _), o in zip(self.parts, self.offs)})
        return host, views


@dataclass
class DeviceSignals:
    """Signals resident in HBM: one f32 buffer, per-file offset/length (samples)."""
    buf: torch.Tensor
    off: np.ndarray
    length: np.ndarray

    @property
    def n_files(self) -> int:
        return len(self.off)


@dataclass
class PairOutcome:
    """One pair's result (or the exception run() raises) and its log lines.  Lines are
    recorded as strings or zero-argument callables and rendered on first access of
    ``logs`` (same text, formatted only if somebody reads it)."""
    result: Optional[C.AnalysisResult] = None
    error: Optional[BaseException] = None
    _log_ops: list = field(default_factory=list)
    detail: dict = field(default_factory=dict)
    # (AsmContext, pair index in it): the inputs assemble_pair read, kept for the window-sharded
    # result gather (sharded.GatheredOutcomes), which sends them as plain arrays and re-runs
    # assemble_pair on the receiving rank; the MELODIA hook's (pick, lines) when it ran
    _asm: Optional[tuple] = field(default=None, repr=False, compare=False)
    _melodia: Optional[tuple] = field(default=None, repr=False, compare=False)

    @property
    def logs(self) -> List[str]:
        if any(not isinstance(x, str) for x in self._log_ops):
            lines: List[str] = []
            for x in self._log_ops:
                if isinstance(x, str):
                    lines.append(x)
                else:
                    r = x()
                    lines.extend(r) if isinstance(r, list) else lines.append(r)
            self._log_ops[:] = lines        # in place: assemble_pair keeps appending to this list
        return self._log_ops


def cu_masks(spec: str, num_cu: int) -> Tuple[List[int], List[int]]:
    """(window-chain mask, chroma-chain mask) as 32-bit words for NC_CU_SPLIT=k[:form]: "even"
    (default) gives the window chain k / words CUs of every 32-CU word, "low" the first k CUs."""
    k, form = (spec.split(":") + ["even"])[:2]
    k, words = int(k), (num_cu + 31) // 32
    if form == "low":
        bits = [min(32, max(0, k - 32 * i)) for i in range(words)]
    else:
        bits = [k // words + (1 if i < k % words else 0) for i in range(words)]
    full = (1 << 32) - 1
    win = [((1 << b) - 1) & full for b in bits]
    return win, [full ^ m for m in win]


def _cu_masked_streams(spec: str, num_cu: int, dev: torch.device):
    """Two HIP streams restricted to complementary CU sets (hipExtStreamCreateWithCUMask of the
    HIP runtime torch loaded), wrapped as torch streams."""
    import ctypes as _C
    lib = _C.CDLL("libamdhip64.so")
    fn = lib.hipExtStreamCreateWithCUMask
    fn.restype = _C.c_int
    fn.argtypes = [_C.POINTER(_C.c_void_p), _C.c_uint32, _C.POINTER(_C.c_uint32)]
    out = []
    for m in cu_masks(spec, num_cu):
        h = _C.c_void_p()
        arr = (_C.c_uint32 * len(m))(*m)
        with torch.cuda.device(dev):
            rc = fn(_C.byref(h), len(m), arr)
        if rc != 0:
            raise _native.NativeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
        out.append(torch.cuda.ExternalStream(h.value, device=dev))
    return out


@dataclass(eq=False)
class _TrimBlocks:
    """A finished (or queued) nc_trim_bounds call: its workspace (the f64 512-sample block sums
    of files [f0, f1) of the batch), the device offsets of those files and the trim's event."""
    ws: torch.Tensor
    off: "_DevSpan"
    f0: int
    f1: int
    event: Optional[torch.cuda.Event]


@dataclass(eq=False)
class AsmContext:
    """What ``assemble_pair`` reads for the pairs of one group: the group's host result arrays
    (``h``: the device arena's views, or the split-pair path's record columns), the hop-64 IBI
    results, and the host plan.  Every outcome keeps a reference to its group's context, so the
    window-sharded gather can send the context as plain arrays and the receiving rank rebuilds
    the outcome with the same ``assemble_pair`` call (sharded.GatheredOutcomes)."""
    h: dict
    ibi: Optional[dict]
    starts: list
    w0: list
    w1: list
    f_len: np.ndarray
    strip_len: np.ndarray
    lead: np.ndarray
    trail: np.ndarray
    intro: list
    win_n: int
    pair_chunks: list
    n_cp: int
    nj: int
    n_pitch_jobs: int
    align: Optional[list]
    # the pinned host arena the views of ``h`` were carved from (engine._Arena.to_host: the
    # bytes and {name: (view, byte offset)}): the record gather sends it as one array
    arena: Optional[tuple] = None
    starts_a: Optional[list] = None     # ``starts`` as the plan's int arrays (the record gather's form)

    def assemble(self, b: int, p: "Params", out: Optional["PairOutcome"] = None, wait=None, span=None) -> "PairOutcome":
        o = assemble_pair(b, p, self.h, self.ibi, self.starts, self.w0, self.w1, self.f_len, self.strip_len,
                          self.lead, self.trail, self.intro[b], self.win_n, self.pair_chunks, self.n_cp, self.nj,
                          self.n_pitch_jobs, self.align[b] if self.align else None, out=out, wait=wait, span=span)
        o._asm = (self, b)
        return o


@dataclass
class Params:
    window_sec: float = 10.0
    hop_sec: float = 5.0
    energy_gate_db: float = -40.0
    silence_strip_db: Optional[float] = 60.0
    src_trim_sec: float = 0.0
    auto_align: bool = False
    compute_pitch: bool = True
    compute_ibi: bool = True
    ibi_beats: bool = False      # also copy the hop-64 beat frames back (detail["ibi_beats"]: (nc, src))
    # MELODIA refinement (pitch.py:246-291) where essentia is installed: melodia(pair, chroma
    # shift, log) -> (src Hz, nc Hz) when accepted, else None (pipeline.run sets it; it runs
    # essentia on the host arrays, as the reference does)
    melodia: Optional[Callable] = None


def _group_bounds(B: int, group_pairs, ) -> List[Tuple[int, int]]:
    """Pair groups of about group_pairs; the last one is halved so that the host
    assembly left exposed after the final device work stays short.  A list of sizes
    gives the schedule explicitly (repeated from its start if it does not cover B)."""
    if isinstance(group_pairs, (list, tuple)):
        sizes, left, i = [], B, 0
        while left > 0:
            n = min(left, max(1, int(group_pairs[i % len(group_pairs)])))
            sizes.append(n)
            left -= n
            i += 1
    elif group_pairs is None:
        # default: groups of 32 pairs, the last two evened out when 32 does not divide the batch
        # (no group under 16 pairs once B > 32).  Round 5, with the oldest group assembled as soon
        # as it completes (Engine.EAGER_FINISH): 4 x 16 ran the 64-pair step 4-5 % faster than the
        # earlier 6/26/26/6 (profiles/r5_group_schedule.txt).  Round 6, after the STFT frame queue
        # made each group's device work shorter against its fixed tail (two bootstraps, the chroma
        # plan and tail, six small launches per group): 2 x 32 7.96-8.59 against 4 x 16
        # 8.44-9.32 ms per step in alternating bench runs, device idle 2.6-3.0 against 4.8 %
        # (profiles/r6_group_schedule.txt; 21/21/22 and 64 no better).  NC_GROUP_PAIRS=G: A/B knob
        G = max(1, int(os.environ.get("NC_GROUP_PAIRS", "32")))
        q, r = divmod(B, G)
        if B <= G:
            sizes = [B] if B else []
        elif r == 0 or r >= G // 2:
            sizes = [G] * q + ([r] if r else [])
        else:
            sizes = [G] * (q - 1) + [(G + r + 1) // 2, (G + r) // 2]
    else:
        gp = max(1, int(group_pairs))
        sizes = [gp] * (B // gp) + ([B % gp] if B % gp else [])
        if len(sizes) > 1 and sizes[-1] >= 8:
            last = sizes.pop()
            sizes += [last - last // 2, last // 2]
    out, g0 = [], 0
    for n in sizes:
        out.append((g0, g0 + n))
        g0 += n
    return out


@dataclass
class BatchPlan:
    """Host plan of one batch of pairs (files nc_0, src_0, nc_1, src_1, ...): the trimmed
    file spans, the 10 s windows and the 20 s chunk pairs, as the reference derives them
    (io.py:58-112, pipeline.py:91-136, pitch.py:121-138).  Window order: every source
    window (pair-major), then every nightcore window; w0[f]..w1[f] are file f's windows."""
    nF: int
    B: int
    f_off: np.ndarray
    f_len: np.ndarray
    strip_len: np.ndarray
    lead: np.ndarray
    trail: np.ndarray
    intro: list
    win_n: int
    hop_n: int
    starts: list
    w0: np.ndarray
    w1: np.ndarray
    win_abs: np.ndarray
    n_win: int
    n_src_w: int
    chunk_off: list
    chunk_len: list
    pair_chunks: list
    n_chunks: int
    n_cp: int


def beat_needs_workspace(T: int, acw: int) -> bool:
    """nc_tempo_beats runs a T-frame sequence in LDS up to 64 KB (csrc/beat.hip
    launch_tempo_beats), longer ones through a global workspace."""
    tab = ((2 * (acw - 1) + 2) * 8 + 15) // 16 * 16
    return tab + T * 21 + 16 > 64 * 1024


# the longest window the per-window stage runs: window_tg_slide_kernel's LDS image of
# 2 T + 3 acw doubles within kWinTgLdsCap = 160 KiB - 1 KiB (csrc/window_stage.hip
# wtg_slide_lds_doubles): T <= 9660 frames, ~224 s at hop 512
MAX_WINDOW_FRAMES = ((160 * 1024 - 1024) // 8 - 3 * 344) // 2


def plan_batch(off: np.ndarray, length: np.ndarray, start: np.ndarray, end: np.ndarray, p: "Params",
               align: Optional[List[Tuple[float, float]]] = None) -> BatchPlan:
    """Silence-trim bounds [start, end) of every file -> BatchPlan (host only, deterministic:
    every rank of a sharded run derives the same plan)."""
    if 1 + int(p.window_sec * SR) // HOP_LENGTH > MAX_WINDOW_FRAMES:
        raise ValueError(f"window_sec={p.window_sec} is longer than the engine's per-window stage supports "
                         f"({(MAX_WINDOW_FRAMES - 1) * HOP_LENGTH / SR:.0f} s)")
    nF = len(off)
    B = nF // 2
    f_off = np.asarray(off, np.int64) + start
    f_len = end - start
    strip_len = f_len.copy()
    lead = start / SR
    trail = (np.asarray(length, np.int64) - end) / SR
    intro = [None] * B
    if p.src_trim_sec > 0.0:
        k = int(p.src_trim_sec * SR)
        for b in range(B):
            f = 2 * b + 1
            cut = min(k, int(f_len[f]))
            f_off[f] += cut
            f_len[f] -= cut
            intro[b] = p.src_trim_sec
    elif align is not None:
        for b, (raw, _) in enumerate(align):
            if raw >= ALIGN_MIN_OFFSET:                  # pipeline.py:114-116
                f = 2 * b + 1
                cut = min(int(raw * SR), int(f_len[f]))
                f_off[f] += cut
                f_len[f] -= cut
                intro[b] = raw

    win_n, hop_n = int(p.window_sec * SR), int(p.hop_sec * SR)
    starts = []
    for f in range(nF):
        L = int(f_len[f])
        s = np.arange(0, max(0, L - win_n) + 1, hop_n, dtype=np.int64) if L >= win_n and hop_n > 0 \
            else np.zeros(0, np.int64)
        starts.append(s)
    # window order: all source windows (pair-major), then all nightcore windows
    order = [2 * b + 1 for b in range(B)] + [2 * b for b in range(B)]
    w0 = np.zeros(nF, np.int64)
    w1 = np.zeros(nF, np.int64)
    win_abs, pos = [], 0
    for f in order:
        w0[f] = pos
        win_abs.append(f_off[f] + starts[f])
        pos += len(starts[f])
        w1[f] = pos
    n_win = pos
    n_src_w = int(sum(len(starts[2 * b + 1]) for b in range(B)))
    win_abs = np.concatenate(win_abs) if win_abs else np.zeros(0, np.int64)

    chunk_off, chunk_len, pair_chunks = [], [], []
    if p.compute_pitch:
        cn = int(CHUNK_SEC * SR)
        for b in range(B):
            ns, nn = int(f_len[2 * b + 1]), int(f_len[2 * b])
            n = min(ns // cn, nn // cn)
            first = len(chunk_off) // 2
            if n < 1:
                chunk_off += [f_off[2 * b + 1], f_off[2 * b]]
                chunk_len += [ns, nn]
                n = 1
            else:
                for i in range(n):
                    chunk_off += [f_off[2 * b + 1] + i * cn, f_off[2 * b] + i * cn]
                    chunk_len += [cn, cn]
            pair_chunks.append((first, first + n))
    n_chunks = len(chunk_off)
    n_cp = n_chunks // 2
    return BatchPlan(nF, B, f_off, f_len, strip_len, lead, trail, intro, win_n, hop_n, starts, w0, w1, win_abs, n_win,
                     n_src_w, chunk_off, chunk_len, pair_chunks, n_chunks, n_cp)


def shared_tuning_map(pl: BatchPlan, tp: int, win_chunk: np.ndarray, tf_skip: np.ndarray) -> None:
    """Chunks whose first ``tp`` tuning frames are a window's leading STFT frames: a standard
    20 s chunk (chunk i of file f starts at i * CHUNK) that starts where a window of the same
    file starts.  Sets win_chunk[window] = chunk and tf_skip[chunk] = tp for each such pair
    (vectorised over the batch's chunks; a per-chunk loop cost ~0.5 ms of host time per
    26-pair group)."""
    n_chunks, hop_n = pl.n_chunks, pl.hop_n
    if n_chunks == 0 or hop_n <= 0:
        return
    cn = int(CHUNK_SEC * SR)
    cl = np.asarray(pl.chunk_len, np.int64)
    per = np.array([c1 - c0 for c0, c1 in pl.pair_chunks], np.int64)
    first = np.array([c0 for c0, _ in pl.pair_chunks], np.int64)
    pc = np.arange(n_chunks) >> 1                      # chunk pair of chunk c (src, nc interleaved)
    side = np.arange(n_chunks) & 1                     # 0: source (file 2b + 1), 1: nightcore (2b)
    b = np.repeat(np.arange(len(per)), per)[pc]
    i = pc - np.repeat(first, per)[pc]                 # chunk index within its pair
    f = 2 * b + 1 - side
    pos = i * cn                                       # the chunk's start inside its file
    k = pos // hop_n                                   # the window that would start there
    w0, w1 = np.asarray(pl.w0, np.int64), np.asarray(pl.w1, np.int64)
    ok = (cl == cn) & (pos % hop_n == 0) & (k < w1[f] - w0[f])
    c = np.flatnonzero(ok)
    wk = w0[f[c]] + k[c]
    hit = np.asarray(pl.win_abs, np.int64)[wk] - np.asarray(pl.f_off, np.int64)[f[c]] == pos[c]
    win_chunk[wk[hit]] = c[hit]
    tf_skip[c[hit]] = tp


class _HostViews(dict):
    """A group's host result views, plus python-list forms ("bpm_l", ...) made on first
    access for the scalar lookups of the assembly loops (dropped by ``refresh`` when a
    later stage's copy has landed)."""

    def __missing__(self, key):
        if key.endswith("_l") and key[:-2] in self:
            v = self[key[:-2]].tolist()
            self[key] = v
            return v
        raise KeyError(key)

    def refresh(self) -> None:
        for k in [k for k in self if k.endswith("_l")]:
            del self[k]


class _StageWaiter:
    """wait(stage) for assemble_pair when lines are streamed: emit the pair's lines so far,
    then wait for that stage's results (engine._launch_group stage_copy)."""

    def __init__(self, out: PairOutcome, g: dict, h: _HostViews, emit):
        self.out, self.g, self.h, self.emit = out, g, h, emit
        self.done = 0

    def flush(self) -> None:
        lines = self.out.logs                       # renders the deferred lines
        for line in lines[self.done:]:
            self.emit(line)
        self.done = len(lines)

    def __call__(self, stage: str) -> None:
        self.flush()
        ev = self.g["stage_ev"].get(stage) if stage != "final" else None
        (ev or self.g["event"]).synchronize()
        self.h.refresh()


# ------------------------------------------------------------------------------ engine
class Engine:
    def __init__(self, device: int = 0, sr: int = SR):
        """``sr`` (round 6): an engine whose context's rate-dependent tables (mel bank,
        tempogram windows) are built for that sample rate serves the tempo seams at it
        (tempo.py:27-173 pass sr through to librosa); the batched pipeline, the chroma and the
        tuning need the default 22 050 Hz."""
        if not torch.cuda.is_available():
            raise _native.NativeUnavailable("no HIP device visible to torch (ROCm); the engine has no CPU path")
        self.device_index = device
        self.dev = torch.device("cuda", device)
        self.sr = int(sr)
        self.ctx = _native.Context(device, self.sr)
        self._ws: Dict[str, torch.Tensor] = {}
        self.num_cu = self.ctx.lib.nc_num_cu(self.ctx.h)
        self.timers: Optional[Dict[str, list]] = None
        self.host_stats: Optional[Dict[str, float]] = None  # {phase: seconds} when enabled
        self._jb_memo: Dict[Tuple[int, int], int] = {}
        self.host_trace: Optional[list] = None   # [(perf_counter, label)] of the pipelined loop when enabled
        # the chroma chain runs on its own stream, concurrently with the window/tempo chain
        # (NC_SERIAL_STREAMS=1 queues it on the launch stream instead: isolated per-kernel timings)
        # NC_STREAM_PRIO="chroma,tail" sets the two side streams' priorities (torch: lower = more
        # urgent; the launch stream stays at 0).  Round 1 measured -1,-1 against 0,0 at 14.20
        # against 14.26 ms per step: within box-to-box spread, so the default is arbitrary
        prio = [int(v) for v in os.environ.get("NC_STREAM_PRIO", "-1,-1").replace(":", ",").split(",")]
        self.chroma_stream = torch.cuda.current_stream(self.dev) if os.environ.get("NC_SERIAL_STREAMS") == "1" \
            else torch.cuda.Stream(self.dev, priority=prio[0])
        # consensus tail (bootstraps + D2H of a group) on a third stream: the window chain of the
        # next group starts as soon as this group's window chain is done, instead of queueing
        # behind a bootstrap that waits for this group's (longer) chroma chain
        self.tail_stream = torch.cuda.current_stream(self.dev) if os.environ.get("NC_SERIAL_STREAMS") == "1" \
            else torch.cuda.Stream(self.dev, priority=prio[1])
        # the silence trims of the next batch of analyze_batches, queued while the current
        # batch's last groups run (not behind their bootstraps on the tail stream)
        self.trim_stream = torch.cuda.current_stream(self.dev) if os.environ.get("NC_SERIAL_STREAMS") == "1" \
            else torch.cuda.Stream(self.dev)
        # leading tuning frames of a chunk computed inside the window STFT (nc_window_stage_tuning);
        # NC_SHARE_TUNING=0 runs every tuning frame in the chroma chain instead (same results)
        self.share_tuning = os.environ.get("NC_SHARE_TUNING", "1") != "0"
        # NC_CU_SPLIT=k[:form] (measurement): the window chain on a stream of k
        # CUs and the chroma chain on a stream of the others (hipExtStreamCreateWithCUMask), the
        # persistent STFT / tuning grids sized to them (NC_STFT_CUS / NC_CHROMA_CUS, set by the caller
        # before the context is created).  The masked window stream becomes torch's current stream
        split = os.environ.get("NC_CU_SPLIT")
        if split:
            w, c = _cu_masked_streams(split, self.num_cu, self.dev)
            torch.cuda.set_stream(w)
            self.chroma_stream = c

    def close(self) -> None:
        """Wait for this engine's streams, then drop its workspaces and its context (tables)."""
        if getattr(self, "ctx", None) is None:
            return
        for s_ in {self.chroma_stream, self.tail_stream, self.trim_stream}:
            s_.synchronize()
        torch.cuda.current_stream(self.dev).synchronize()
        self._ws.clear()
        self.ctx.close()
        self.ctx = None

    def set_serial(self, on: bool) -> None:
        """Queue the chroma chain and the consensus tail on the launch stream too (on=True):
        every kernel then runs alone, so per-kernel timers measure its isolated speed rather
        than its share of a concurrently loaded chip.  Measurement only (bench.py)."""
        if on:
            self._streams = (self.chroma_stream, self.tail_stream, self.trim_stream)
            self.chroma_stream = self.tail_stream = self.trim_stream = torch.cuda.current_stream(self.dev)
        elif getattr(self, "_streams", None):
            self.chroma_stream, self.tail_stream, self.trim_stream = self._streams
            self._streams = None

    # -------------------------------------------------------------- plumbing
    def _job_bytes(self, cap: int, n_boot: int) -> int:
        """nc_bootstrap_job_bytes, memoised (a group asks for ~80 jobs' sizes, most of them equal)."""
        key = (cap, n_boot)
        v = self._jb_memo.get(key)
        if v is None:
            v = self._jb_memo[key] = int(self.ctx.lib.nc_bootstrap_job_bytes(cap, n_boot))
        return v

    def stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    def workspace(self, name: str, nbytes: int) -> torch.Tensor:
        t = self._ws.get(name)
        if t is None or t.numel() < nbytes:
            t = torch.empty(int(max(256, nbytes * 1.1)), dtype=torch.uint8, device=self.dev)
            self._ws[name] = t
        return t

    def call(self, name: str, *args):
        if self.timers is None:
            self.ctx.call(name, *args)
            return
        s = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        self.ctx.call(name, *args)
        e1.record(s)
        self.timers.setdefault(name, []).append((e0, e1))

    def start_timers(self):
        """Record a HIP event pair around every entry-point launch (on the launch stream)."""
        self.timers = {}

    def stop_timers(self) -> Dict[str, Tuple[float, int]]:
        """{entry point: (total ms, launches)}; synchronises."""
        torch.cuda.synchronize(self.dev)
        out = {k: (sum(a.elapsed_time(b) for a, b in v), len(v)) for k, v in (self.timers or {}).items()}
        self.timers = None
        return out

    GROUPS_IN_FLIGHT = 3    # pair groups queued ahead of the host's oldest wait (EAGER_FINISH off)
    # Round 5: the host assembles a group only once its results are on the host (or when
    # MAX_GROUPS_IN_FLIGHT are queued) and launches the next group meanwhile; untraced device
    # idle over 10 pipelined steps 4.6-4.9 % -> 4.2-4.7 % (tools/idle_probe.py), the step the same
    EAGER_FINISH = True
    MAX_GROUPS_IN_FLIGHT = 5

    KERNEL_TAGS = ("stft_mel", "window_tg", "tuning_peaks", "decimate", "cqt_low", "cqt_high", "trim_blocks", "tempo_beat",
                   "tg_slide", "spectral_frames", "spectral_bins")

    def kernel_profile(self, on) -> None:
        """The library's per-kernel timers (nc_profile_enable): False/0 off, True/1 HIP events
        around each launch plus the kernels' own execution spans, 2 spans only (cheap enough
        to leave on in a timed region), 3 events around the roofline kernels only plus spans,
        4 those events alone, 5 spans plus marker spans around the small entry points (timeline
        diagnosis: tools/concurrency_spans.py --marks)."""
        self.ctx.call("nc_profile_enable", int(on))

    def _profile_read(self, fn: str) -> Dict[str, Tuple[float, int]]:
        import ctypes as C
        out = {}
        for tag in self.KERNEL_TAGS:
            ms, n = C.c_double(0.0), C.c_int(0)
            self.ctx.call(fn, tag.encode(), C.byref(ms), C.byref(n))
            if n.value:
                out[tag] = (ms.value, n.value)
        if "cqt_low" in out and "cqt_high" in out:
            # the CQT unit of the roofline (7 octaves of every chunk of a chroma call): the two
            # kernels' times summed, as rocprofv3 --stats lists them (two rows)
            out["cqt_chroma"] = (out["cqt_low"][0] + out["cqt_high"][0], out["cqt_low"][1])
        return out

    def kernel_times(self) -> Dict[str, Tuple[float, int]]:
        """{kernel tag: (total ms, launches)} of the HIP-event brackets since the last read
        (nc_profile_read); waits for them."""
        return self._profile_read("nc_profile_read")

    def kernel_spans(self) -> Dict[str, Tuple[float, int]]:
        """{kernel tag: (total ms, launches)} of the kernels' execution spans since the last
        read (nc_profile_read_span: first wave start .. last wave end, rocprofv3's kernel
        duration); waits for them."""
        return self._profile_read("nc_profile_read_span")

    def device_busy(self) -> Tuple[float, float, int]:
        """(busy ms, extent ms, launches) over every kernel span recorded since the last read
        (nc_profile_read_busy: union of the execution spans of all tags; profile modes 1-3);
        waits for the device and clears the spans."""
        import ctypes as C
        b, e, n = C.c_double(0.0), C.c_double(0.0), C.c_int(0)
        self.ctx.call("nc_profile_read_busy", C.byref(b), C.byref(e), C.byref(n))
        return b.value, e.value, n.value

    def device_spans(self, cap: int = 1 << 16) -> List[Tuple[str, float, float]]:
        """[(tag, start ms, end ms)] of every kernel span recorded since the last read, in launch
        order (nc_profile_dump_spans; profile modes 1-3); waits for the device, clears the spans."""
        import ctypes as C
        tags = C.create_string_buffer(1 << 14)
        idx = np.zeros(cap, np.int32)
        st, en = np.zeros(cap), np.zeros(cap)
        n = C.c_int(0)
        self.ctx.call("nc_profile_dump_spans", C.addressof(tags), len(tags), idx.ctypes.data, st.ctypes.data,
                      en.ctypes.data, cap, C.byref(n))
        names = tags.value.decode().split("\n")
        return [(names[idx[i]], float(st[i]), float(en[i])) for i in range(n.value)]

    def upload_signals(self, arrays: Sequence[np.ndarray]) -> DeviceSignals:
        """The files into one f32 HBM buffer (64-sample aligned offsets).  When every file is
        16-bit PCM as stored (``io.Pcm16``) the 2-byte samples are uploaded and widened on the
        device (``nc_pcm16_to_f32``, k / 32768 exactly): half the host -> HBM bytes."""
        from .io import Pcm16, as_f32
        lens = np.array([len(a) for a in arrays], dtype=np.int64)
        offs = np.zeros(len(arrays), dtype=np.int64)
        tot = 0
        for i, n in enumerate(lens):
            offs[i] = tot
            tot += (int(n) + _ALIGN - 1) // _ALIGN * _ALIGN
        pcm = bool(arrays) and all(isinstance(a, Pcm16) for a in arrays)
        host = torch.zeros(max(_ALIGN, tot), dtype=torch.int16 if pcm else torch.float32, pin_memory=True)
        hv = host.numpy()
        for a, o in zip(arrays, offs):
            hv[o:o + len(a)] = a.view(np.ndarray) if pcm else as_f32(a)
        if not pcm:
            return DeviceSignals(host.to(self.dev, non_blocking=True), offs, lens)
        raw = host.to(self.dev, non_blocking=True)
        buf = torch.empty(raw.numel(), dtype=torch.float32, device=self.dev)
        self.call("nc_pcm16_to_f32", raw.data_ptr(), raw.numel(), buf.data_ptr(), self.stream())
        return DeviceSignals(buf, offs, lens)

    # -------------------------------------------------------------- bootstrap (generic)
    def bootstrap(self, jobs: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]], seed: int,
                  n_boot: int = C.N_BOOTSTRAP, ci: float = C.CI_LEVEL, ws_tag: str = ""):
        """[(A, B|None)] -> [(point, (lo, hi))] with numpy default_rng(seed) semantics.
        ``ws_tag`` prefixes the workspace name (work queued beside the pipelined groups)."""
        dev = self.dev
        vals, a_off, a_n, b_off, b_n, caps = [], [], [], [], [], []
        pos = 0
        has_b = jobs[0][1] is not None
        for A, B in jobs:
            A = np.asarray(A, np.float64)
            a_off.append(pos)
            a_n.append(len(A))
            vals.append(A)
            pos += len(A)
            if has_b:
                B = np.asarray(B, np.float64)
                b_off.append(pos)
                b_n.append(len(B))
                vals.append(B)
                pos += len(B)
            caps.append(len(A) + (len(B) if has_b else 0))
        wsoff, tot = [], 0
        for c in caps:
            wsoff.append(tot)
            tot += self.ctx.lib.nc_bootstrap_job_bytes(int(c), int(n_boot))
        up = _Upload()
        up.add("vals", np.concatenate(vals) if vals else np.zeros(1), np.float64)
        up.add("a_off", a_off, np.int64)
        up.add("a_n", a_n, np.int32)
        up.add("b_off", b_off or [0], np.int64)
        up.add("b_n", b_n or [0], np.int32)
        up.add("seed", seed_state(seed) * len(jobs), np.uint64)
        up.add("wsoff", wsoff, np.int64)
        up.add("cap", caps, np.int32)
        d = up.commit(dev)
        n = len(jobs)
        out = torch.empty(3 * n, dtype=torch.float64, device=dev)
        ws = self.workspace(ws_tag + "boot", tot)
        il, gl, ih, gh = percentile_params(n_boot, ci)
        self.call("nc_bootstrap_ratio", d["vals"].data_ptr(), d["a_off"].data_ptr(), d["a_n"].data_ptr(),
                  d["b_off"].data_ptr() if has_b else None, d["b_n"].data_ptr() if has_b else None, n,
                  n_boot, d["seed"].data_ptr(), il, gl, ih, gh, 1, out[0:n].data_ptr(),
                  out[n:2 * n].data_ptr(), out[2 * n:3 * n].data_ptr(), None, d["wsoff"].data_ptr(),
                  d["cap"].data_ptr(), ws.data_ptr(), ws.numel(), self.stream())
        o = out.cpu().numpy()
        return [(float(o[i]), (float(o[n + i]), float(o[2 * n + i]))) for i in range(n)]

    # -------------------------------------------------------------- auto-align (xcorr.py:165-259)
    def align_offsets(self, buf: torch.Tensor, src_off, src_len, nc_off, nc_len, sr: int = SR,
                      speed_lo: float = ALIGN_SPEED_LO, speed_hi: float = ALIGN_SPEED_HI,
                      n_speeds: int = ALIGN_N_SPEEDS, max_offset_sec: float = ALIGN_MAX_OFFSET):
        """xcorr.find_content_offset for every (src, nc) pair of signals already in ``buf``
        (sample offsets / lengths): [(offset_sec, speed_est)] (one host sync)."""
        if sr != 2 * ALIGN_SR:
            raise NotImplementedError("the device resampler is 2:1 (sr 22050 -> 11025) only")
        n = len(src_off)
        if n == 0:
            return []
        speeds = np.linspace(speed_lo, speed_hi, n_speeds)            # xcorr.py:220
        hop_sec = ALIGN_HOP / ALIGN_SR                                   # xcorr.py:213
        max_frames = int(max_offset_sec / hop_sec)                       # xcorr.py:214
        lens = np.concatenate([np.asarray(src_len, np.int64), np.asarray(nc_len, np.int64)])
        up = _Upload()
        up.add("src_off", src_off, np.int64)
        up.add("src_len", src_len, np.int64)
        up.add("nc_off", nc_off, np.int64)
        up.add("nc_len", nc_len, np.int64)
        up.add("speeds", speeds, np.float64)
        d = up.commit(self.dev)
        ar = _Arena()
        ar.add("peak", n, np.int32)
        ar.add("speed", n, np.int32)
        ar.add("score", n, np.float64)
        o = ar.commit(self.dev)
        tot, mx = int(lens.sum()), int(max(1, lens.max()))
        ws = self.workspace("align", self.ctx.lib.nc_align_workspace_bytes(self.ctx.h, n, n_speeds, tot, mx,
                                                                           max_frames))
        self.call("nc_align_offsets", buf.data_ptr(), d["src_off"].data_ptr(), d["src_len"].data_ptr(),
                  d["nc_off"].data_ptr(), d["nc_len"].data_ptr(), n, d["speeds"].data_ptr(), n_speeds, max_frames,
                  tot, mx, o["peak"].data_ptr(), o["speed"].data_ptr(), o["score"].data_ptr(), ws.data_ptr(),
                  ws.numel(), self.stream())
        hbuf, h = ar.to_host()
        torch.cuda.current_stream(self.dev).synchronize()
        out = []
        for p_, s_ in zip(h["peak"].tolist(), h["speed"].tolist()):
            if s_ < 0:
                out.append((0.0, (speed_lo + speed_hi) / 2.0))
            else:
                out.append((p_ * hop_sec, float(speeds[s_])))
        return out

    # -------------------------------------------------------------- batched pipeline
    # -------------------------------------------------------------- spectral (spectral.py:38-103)
    SPECTRAL_BANDS = ((20, 80), (80, 250), (250, 2000), (2000, 6000), (6000, 20000))   # spectral.py:70-74

    def spectral_frames(self, buf: torch.Tensor, off, length, srs, roll_percent: float = 0.85,
                        frame_rms: bool = False):
        """nc_spectral_stats over signals already in ``buf`` (sample offsets / lengths, each at
        its own rate srs[f]).  Queues the launch and the D2H copy of the per-file sums (and,
        with frame_rms, of the frame RMS); returns (event, host views, keep-alive).
        ``spectral_finish`` turns the views into per-file statistics."""
        with _GcPaused():
            return self._spectral_frames(buf, off, length, srs, roll_percent, frame_rms)

    def _spectral_frames(self, buf, off, length, srs, roll_percent, frame_rms):
        off = np.asarray(off, np.int64)
        length = np.asarray(length, np.int64)
        n = len(off)
        T = 1 + length // 512                                              # centred frames
        base = np.zeros(n + 1, np.int64)
        base[1:] = np.cumsum(T)
        # bin spacing and band bins once per distinct rate (a per-file loop of rfftfreq and band
        # masks cost ~4 ms per 128 files, as much as the device work)
        rates, inv = np.unique(np.asarray(srs, np.float64), return_inverse=True)
        rb = np.zeros((len(rates), len(self.SPECTRAL_BANDS), 2), np.int32)
        rhz = np.zeros(len(rates), np.float64)
        for u, sr in enumerate(rates):
            freqs = np.fft.rfftfreq(2048, 1.0 / sr)                        # librosa.fft_frequencies
            rhz[u] = freqs[1]
            for b, (lo, hi) in enumerate(self.SPECTRAL_BANDS):
                idx = np.flatnonzero((freqs >= lo) & (freqs < hi))
                if idx.size:
                    rb[u, b] = (idx[0], idx[-1] + 1)
        bands = np.ascontiguousarray(rb[inv])
        hz = np.ascontiguousarray(rhz[inv])
        up = _Upload()
        up.add("off", off, np.int64)
        up.add("len", length, np.int64)
        up.add("base", base, np.int64)
        up.add("hz", hz, np.float64)
        up.add("bands", bands, np.int32)
        d = up.commit(self.dev, spans=True)
        ar = _Arena()
        ar.add("stats", 12 * n, np.float64)
        ar.add("bins", 1025 * n, np.float64)
        o = ar.commit(self.dev, spans=True)
        rms = torch.empty(int(base[-1]), dtype=torch.float32, device=self.dev)
        tot, mx = int(base[-1]), int(T.max())
        ws = self.workspace("spectral", self.ctx.lib.nc_spectral_workspace_bytes(tot, n, mx))
        self.call("nc_spectral_stats", buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(),
                  d["base"].data_ptr(), d["hz"].data_ptr(), d["bands"].data_ptr(), n, tot, mx,
                  float(roll_percent), rms.data_ptr(), o["stats"].data_ptr(), o["bins"].data_ptr(),
                  ws.data_ptr(), ws.numel(), self.stream())
        hbuf, h = ar.to_host()
        if frame_rms:
            hr = torch.empty(rms.numel(), dtype=torch.float32, pin_memory=True)
            hr.copy_(rms, non_blocking=True)
            h["rms"] = hr.numpy()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        h.update(base=base, T=T, bands=bands, hz=hz, length=length, srs=list(srs))
        return ev, h, (d, o, hbuf, rms)

    @staticmethod
    def spectral_finish(h) -> List[dict]:
        """Per-file SpectralStats fields from the device sums (spectral.py:54-94): means over
        the T_f frames and band bins, the effective bandwidth from the per-bin dB means."""
        with _GcPaused():
            return Engine._spectral_finish(h)

    @staticmethod
    def _spectral_finish(h) -> List[dict]:
        n = len(h["srs"])
        st = h["stats"].reshape(n, 12)
        T = h["T"].astype(np.float64)
        nb = (h["bands"][:, :, 1] - h["bands"][:, :, 0]).astype(np.float64)
        band = np.where(nb > 0, st[:, 2:7] / (np.maximum(nb, 1.0) * T[:, None]), 0.0)
        favg = h["bins"].reshape(n, 1025) / T[:, None]
        sig = favg > favg.max(axis=1, keepdims=True) - 60.0
        last = np.where(sig.any(axis=1), 1024 - np.argmax(sig[:, ::-1], axis=1), 1024)
        names = ("sub_bass", "bass", "midrange", "presence", "brilliance")
        out = []
        for f in range(n):
            r = {"centroid": float(st[f, 0] / T[f]), "rolloff": float(st[f, 1] / T[f]),
                 "rms_mean": float(st[f, 8]), "rms_variance": float(st[f, 9])}
            r.update({name: float(band[f, b]) for b, name in enumerate(names)})
            r["decay_rate"] = float(st[f, 11])
            r["duration"] = float(h["length"][f]) / h["srs"][f]            # librosa.get_duration
            r["effective_bandwidth_hz"] = float(int(last[f]) * h["hz"][f])
            out.append(r)
        return out

    def spectral(self, signals: Sequence[Tuple[np.ndarray, int]]) -> List[dict]:
        """spectral.analyze statistics for decoded (signal, native rate) pairs, one batch."""
        if not signals:
            return []
        sig = self.upload_signals([np.asarray(y, np.float32) for y, _ in signals])
        ev, h, keep = self.spectral_frames(sig.buf, sig.off, sig.length, [int(sr) for _, sr in signals])
        ev.synchronize()
        return self.spectral_finish(h)

    def analyze(self, pairs: Optional[Sequence[Tuple[np.ndarray, np.ndarray]]] = None, params: Params = None,
                signals: Optional[DeviceSignals] = None, group_pairs=None,
                log: Optional[Callable[[int, str], None]] = None) -> List[PairOutcome]:
        """Run pipeline.run's analysis for every (nc, src) pair.  ``signals``
        (files ordered nc_0, src_0, nc_1, src_1, ...) may be passed already
        resident in HBM; otherwise ``pairs`` are uploaded.

        After one trim pass over all files (the only blocking read-back), pairs
        are processed in groups of ``group_pairs``: the whole device pipeline of
        up to GROUPS_IN_FLIGHT groups is queued (plans uploaded through pinned memory,
        results copied back asynchronously) before the host assembles the results of
        the oldest, so host assembly overlaps the device work of the later groups.

        Python's cyclic garbage collector is paused for the call: a generation-2 pass
        over the host's live objects costs ~10 ms, as long as several groups of device
        work, and lands at a random point of the pipeline.  The call creates no reference
        cycles (everything it allocates is freed by reference counting), and the
        collector's previous state is restored on return.

        ``log(pair index, line)``, when given, receives each pair's log lines while the
        pipeline runs, in the reference's order (pipeline.py:77-215): the device copies
        each stage's results back as the stage completes (energy gate, pitch, source
        tempo, nightcore tempo, consensus), and a pair's lines up to a stage are emitted
        as soon as that stage's results are on the host."""
        gc_was_enabled = gc.isenabled()
        gc.disable()
        try:
            return self._analyze(pairs, params, signals, group_pairs, log)
        finally:
            if gc_was_enabled:
                gc.enable()

    def analyze_batches(self, batches: Sequence[DeviceSignals], params: Params = None,
                        group_pairs=None) -> List[List[PairOutcome]]:
        """``analyze`` of several resident batches back to back, pipelined: the silence trims
        of batch k + 1 are queued (on their own stream) as soon as batch k's last group is
        launched, and batch k + 1's first groups are launched while batch k's last groups
        still run, so the device does not idle through a batch's start-up (trim read-back,
        host plan of the first group).  Every batch is analysed completely and independently;
        the results equal one ``analyze`` call per batch."""
        gc_was_enabled = gc.isenabled()
        gc.disable()
        try:
            return self._analyze_many(list(batches), params or Params(), group_pairs, None)
        finally:
            if gc_was_enabled:
                gc.enable()

    def _analyze(self, pairs, params, signals, group_pairs, log=None) -> List[PairOutcome]:
        p = params or Params()
        if signals is None:
            flat = []
            for nc, src in pairs:
                flat += [nc, src]
            signals = self.upload_signals(flat)
        return self._analyze_many([signals], p, group_pairs, log)[0]

    def _split_trim(self, signals: DeviceSignals, p: Params, groups) -> bool:
        return p.silence_strip_db is not None and len(groups) > 1 and not (p.auto_align and p.src_trim_sec == 0.0)

    def _analyze_many(self, batches: List[DeviceSignals], p: Params, group_pairs, log=None) -> List[List[PairOutcome]]:
        gen = self._analyze_gen(batches, p, group_pairs, log)
        while True:
            try:
                next(gen)
            except StopIteration as stop:
                return stop.value

    def _analyze_gen(self, batches: List[DeviceSignals], p: Params, group_pairs, log=None, on_group=None):
        """The body of ``_analyze_many`` as a generator that yields after each pair group is
        launched (the host is then free until the next ``next``): a caller can interleave
        other host work — the window-sharded record exchanges — with the pipelined groups
        while up to GROUPS_IN_FLIGHT of them keep the device busy.  ``on_group(batch, first
        pair, outcomes)`` runs as each group is assembled, while the later groups are still on
        the device (the sharded result gather packs its records there).  Returns the results."""
        hs = self.host_stats
        launch = torch.cuda.current_stream(self.dev)
        # the signals are complete on the launch stream here; trims of later batches wait for
        # this point only, not for the groups queued on the launch stream after it
        ev_sig = torch.cuda.Event()
        ev_sig.record(launch)
        results: List[List[PairOutcome]] = [[] for _ in batches]
        # up to GROUPS_IN_FLIGHT groups (of any batch) are queued before the host waits for the
        # oldest: the window stream never idles behind the host assembly of an earlier group,
        # the assembly of group g overlaps the device work of the groups after it, and the depth
        # of the device queues (and the memory held by queued groups) stays bounded
        pending: List[dict] = []

        def trim_begin(bi: int, ahead: bool) -> dict:
            """io.strip_silence bounds of batch bi: two launches when the batch has several
            groups (the first group's files, then the rest), read back when needed."""
            signals = batches[bi]
            groups = _group_bounds(signals.n_files // 2, group_pairs)
            if not self._split_trim(signals, p, groups):
                return dict(groups=groups, split=False)
            nF, f1 = signals.n_files, 2 * groups[0][1]
            st0 = self.trim_stream if ahead else launch
            first = self._trim_launch(signals, 0, f1, p, st0, "trim0", ev_sig)
            rest = self._trim_launch(signals, f1, nF, p, self.trim_stream if ahead else self.tail_stream, "trim1",
                                     ev_sig)
            return dict(groups=groups, split=True, first=first, rest=rest, f1=f1)

        trace = self.host_trace

        def mark(label):
            if trace is not None:
                trace.append((time.perf_counter(), label))

        def finish(g):
            mark(f"finish b{g['bi']} g{g['g0']}")
            outs = self._finish_group(g, log)
            results[g["bi"]] += outs
            if on_group is not None:
                on_group(g["bi"], g["g0"], outs)

        nxt = None
        for bi, signals in enumerate(batches):
            t0 = time.perf_counter()
            mark(f"b{bi} trim")
            tr = nxt if nxt is not None else trim_begin(bi, False)
            nxt = None
            groups = tr["groups"]
            align = None
            if tr["split"]:
                nF, f1 = signals.n_files, tr["f1"]
                start = np.zeros(nF, np.int64)
                end = np.zeros(nF, np.int64)
                start[:f1], end[:f1] = self._trim_wait(tr["first"])
                blocks = [tr["first"][3], tr["rest"][3]]
            else:
                start, end, tb = self._trim_all(signals, p)
                blocks = [tb] if tb is not None else []
                if p.auto_align and p.src_trim_sec == 0.0:  # pipeline.py:111-125 (manual trim has priority)
                    align = self.align_offsets(signals.buf, signals.off[1::2] + start[1::2], end[1::2] - start[1::2],
                                               signals.off[0::2] + start[0::2], end[0::2] - start[0::2])
            if hs is not None:
                hs["trim"] = hs.get("trim", 0.0) + time.perf_counter() - t0
            for gi, (g0, g1) in enumerate(groups):
                if gi == 1 and tr["split"]:
                    f1 = tr["f1"]
                    start[f1:], end[f1:] = self._trim_wait(tr["rest"])
                sl = slice(2 * g0, 2 * g1)
                sub = DeviceSignals(signals.buf, signals.off[sl], signals.length[sl])
                t0 = time.perf_counter()
                mark(f"b{bi} g{gi} launch")
                # NC_BLOCK_ENERGY=0 (A/B measurement only): the round-5 per-frame energies in the STFT
                tb = next((b for b in blocks if b.f0 <= 2 * g0 and 2 * g1 <= b.f1), None) \
                    if os.environ.get("NC_BLOCK_ENERGY", "1") != "0" else None
                g = self._launch_group(sub, p, start[sl].copy(), end[sl].copy(),
                                       align[g0:g1] if align is not None else None, log is not None,
                                       blocks=(tb, 2 * g0 - tb.f0) if tb is not None else None)
                g["g0"], g["bi"] = g0, bi
                pending.append(g)
                if gi == len(groups) - 1 and bi + 1 < len(batches):
                    mark(f"b{bi + 1} trim_begin")
                    nxt = trim_begin(bi + 1, True)
                if hs is not None:
                    hs["launch"] = hs.get("launch", 0.0) + time.perf_counter() - t0
                if self.EAGER_FINISH:
                    # launch ahead while the oldest group still runs: assemble it only once it
                    # is complete (or the in-flight cap is reached), so the host's assembly never
                    # leaves the device with just a small group queued
                    while pending and (len(pending) > self.MAX_GROUPS_IN_FLIGHT or
                                       (len(pending) > 1 and pending[0]["event"].query())):
                        finish(pending.pop(0))
                elif len(pending) > self.GROUPS_IN_FLIGHT:
                    finish(pending.pop(0))
                mark("yield")
                yield
        for g in pending:
            finish(g)
        mark("end")
        return results

    def _trim_launch(self, signals: DeviceSignals, f0: int, f1: int, p: Params, stream, ws_name: str,
                     ev_sig: Optional[torch.cuda.Event] = None):
        """Queue nc_trim_bounds for files [f0, f1) on `stream` and the async copy of the bounds
        into pinned memory; returns (event, pinned bounds, keep-alive).  On a side stream the
        trim first waits for ev_sig (the signals complete on the launch stream)."""
        dev = self.dev
        off, length = signals.off[f0:f1], signals.length[f0:f1]
        n = f1 - f0
        lens = np.ascontiguousarray(length, np.int64)
        launch = torch.cuda.current_stream(dev)
        if stream != launch:          # the signals may still be in flight on the launch stream
            if ev_sig is None:
                ev_sig = torch.cuda.Event()
                ev_sig.record(launch)
            stream.wait_event(ev_sig)
        with torch.cuda.stream(stream):
            up = _Upload()
            up.add("off", off, np.int64)
            up.add("len", lens, np.int64)
            d0 = up.commit(dev, spans=True)
            wsb = self.ctx.lib.nc_trim_workspace_bytes(lens.ctypes.data, n)
            # a fresh workspace per launch (not a named one): its 512-sample block sums give the
            # batch's window energies later (nc_window_energy_blocks), while the next batch's trim
            # already runs ahead on the trim stream
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            se = torch.empty(2 * n, dtype=torch.int64, device=dev)
            self.call("nc_trim_bounds", signals.buf.data_ptr(), d0["off"].data_ptr(), d0["len"].data_ptr(), n,
                      int(np.sum(1 + lens // 512)), float(p.silence_strip_db), se[:n].data_ptr(),
                      se[n:].data_ptr(), ws.data_ptr(), ws.numel(), stream.cuda_stream)
            host = torch.empty(2 * n, dtype=torch.int64, pin_memory=True)
            host.copy_(se, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        return ev, host, (d0, se), _TrimBlocks(ws, d0["off"], f0, f1, ev)

    @staticmethod
    def _trim_wait(launched) -> Tuple[np.ndarray, np.ndarray]:
        ev, host, _, _ = launched
        ev.synchronize()
        h = host.numpy()
        n = len(h) // 2
        return h[:n].copy(), h[n:].copy()

    def _trim_all(self, signals: DeviceSignals, p: Params):
        """io.strip_silence bounds of every file (sync 1), and the trim's block sums
        (_TrimBlocks; None without a silence trim)."""
        nF = signals.n_files
        if p.silence_strip_db is None:
            return np.zeros(nF, np.int64), signals.length.copy(), None
        dev, st = self.dev, self.stream()
        up = _Upload()
        up.add("off", signals.off, np.int64)
        up.add("len", signals.length, np.int64)
        d0 = up.commit(dev)
        tot_frames = int(np.sum(1 + signals.length // 512))
        lens = np.ascontiguousarray(signals.length, np.int64)
        # a plain address (ndarray.ctypes.data_as would build a ctypes.cast reference cycle)
        wsb = self.ctx.lib.nc_trim_workspace_bytes(lens.ctypes.data, nF)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)     # fresh: its block sums outlive the call
        se = torch.empty(2 * nF, dtype=torch.int64, device=dev)
        self.call("nc_trim_bounds", signals.buf.data_ptr(), d0["off"].data_ptr(), d0["len"].data_ptr(), nF,
                  tot_frames, float(p.silence_strip_db), se[:nF].data_ptr(), se[nF:].data_ptr(),
                  ws.data_ptr(), ws.numel(), st)
        se_h = se.cpu().numpy()
        return se_h[:nF].copy(), se_h[nF:].copy(), _TrimBlocks(ws, d0["off"], 0, nF, None)

    def _launch_group(self, signals: DeviceSignals, p: Params, start: np.ndarray, end: np.ndarray,
                      align: Optional[List[Tuple[float, float]]] = None, stream_logs: bool = False,
                      blocks: Optional[Tuple["_TrimBlocks", int]] = None) -> dict:
        """Queue the whole device pipeline of one group of pairs; returns the pending group.
        ``blocks``: the silence trim holding this group's files and the index of its first file
        there; the window energies then come from the trim's block sums, not from the STFT."""
        dev, st = self.dev, self.stream()
        pl = plan_batch(signals.off, signals.length, start, end, p, align)
        nF, B = pl.nF, pl.B
        f_off, f_len, strip_len, lead, trail, intro = pl.f_off, pl.f_len, pl.strip_len, pl.lead, pl.trail, pl.intro
        win_n, hop_n, starts, w0, w1 = pl.win_n, pl.hop_n, pl.starts, pl.w0, pl.w1
        win_abs, n_win, n_src_w = pl.win_abs, pl.n_win, pl.n_src_w
        chunk_off, chunk_len, pair_chunks, n_chunks, n_cp = pl.chunk_off, pl.chunk_len, pl.pair_chunks, \
            pl.n_chunks, pl.n_cp
        T = 1 + win_n // HOP_LENGTH
        acw = int(int(8.0 * SR) // HOP_LENGTH)

        # shared tuning frames: a standard 20 s chunk that starts where a window of the same file
        # starts has its first tp tuning frames in that window's STFT (nc_window_stage_tuning)
        tp = (win_n - 1024) // HOP_LENGTH + 1 if win_n >= 1024 else 0
        share = tp > 0 and n_win > 0 and n_chunks > 0 and self.share_tuning
        win_chunk = np.full(max(1, n_win), -1, np.int32)
        tf_skip = np.zeros(max(1, n_chunks), np.int32)
        if share:
            shared_tuning_map(pl, tp, win_chunk, tf_skip)
            share = bool(tf_skip.any())
        chunk_tf_base = np.zeros(max(1, n_chunks) + 1, np.int64)
        if n_chunks:
            chunk_tf_base[1:n_chunks + 1] = np.cumsum(1 + np.asarray(chunk_len, np.int64) // HOP_LENGTH)

        # bootstrap jobs (tempo: A = nc valid, B = src valid; pitch: A = nc_hz, B = src_hz; shift)
        n_pitch_jobs = len(pair_chunks)
        nj = B + n_pitch_jobs
        TV, PV = max(1, n_win), max(1, 3 * n_cp)   # vals = [tempo values at the window index | shift, nc_hz, src_hz]
        jobs_a_off = [w0[2 * b] for b in range(B)] + [TV + n_cp + c0 for c0, _ in pair_chunks]
        jobs_b_off = [w0[2 * b + 1] for b in range(B)] + [TV + 2 * n_cp + c0 for c0, _ in pair_chunks]
        caps = [max(1, (w1[2 * b] - w0[2 * b]) + (w1[2 * b + 1] - w0[2 * b + 1])) for b in range(B)] + \
               [2 * (c1 - c0) for c0, c1 in pair_chunks]
        p_n = [c1 - c0 for c0, c1 in pair_chunks]
        jb = self._job_bytes
        wsoff, tot = [], 0
        for c in caps:
            wsoff.append(tot)
            tot += jb(int(c), C.N_BOOTSTRAP)
        s_wsoff, s_tot = [], 0
        for n in p_n:
            s_wsoff.append(s_tot)
            s_tot += jb(int(n), C.N_BOOTSTRAP)

        # one H2D copy: plan + bootstrap jobs.  a_n / b_n = [valid counts (written on the
        # device by nc_collect_valid) | chunk counts of the pitch jobs]
        up = _Upload()
        up.add("win_off", win_abs if n_win else [0], np.int64)
        if blocks is not None and n_win:
            # each window's file as an index into the trim call that holds the group's files
            w0a, w1a = np.asarray(w0, np.int64), np.asarray(w1, np.int64)
            order = np.argsort(w0a, kind="stable")
            up.add("win_file", np.repeat(order, (w1a - w0a)[order]) + blocks[1], np.int32)
        up.add("w0", w0, np.int32)
        up.add("w1", w1, np.int32)
        up.add("nc_w0", [w0[2 * b] for b in range(B)], np.int32)
        up.add("nc_w1", [w1[2 * b] for b in range(B)], np.int32)
        up.add("on_off", np.arange(n_win, dtype=np.int64) * T if n_win else [0], np.int64)
        up.add("on_len", np.full(max(1, n_win), T), np.int32)
        up.add("src_w0", [w0[2 * b + 1] for b in range(B)], np.int32)
        up.add("src_w1", [w1[2 * b + 1] for b in range(B)], np.int32)
        up.add("src_len", [f_len[2 * b + 1] for b in range(B)], np.int64)
        up.add("nc_len", [f_len[2 * b] for b in range(B)], np.int64)
        nc_pair = np.concatenate([np.full(len(starts[2 * b]), b, np.int32) for b in range(B)]) \
            if n_win - n_src_w else np.zeros(1, np.int32)
        up.add("nc_pair", nc_pair, np.int32)
        up.add("src_pair", np.zeros(max(1, n_src_w), np.int32), np.int32)
        up.add("start120", [120.0], np.float64)
        up.add("chunk_off", chunk_off or [0], np.int64)
        up.add("chunk_len", chunk_len or [0], np.int64)
        up.add("lag_src", np.arange(0, n_chunks, 2), np.int32)
        up.add("lag_nc", np.arange(1, n_chunks, 2), np.int32)
        up.add("f_off", f_off, np.int64)
        up.add("f_len", f_len, np.int64)
        up.add("a_off", jobs_a_off, np.int64)
        up.add("b_off", jobs_b_off, np.int64)
        up.add("a_n", [0] * B + p_n, np.int32)
        up.add("b_n", [0] * B + p_n, np.int32)
        up.add("seed", seed_state(42) * nj, np.uint64)
        up.add("wsoff", wsoff, np.int64)
        up.add("cap", caps, np.int32)
        up.add("s_off", [TV + c0 for c0, _ in pair_chunks] or [0], np.int64)
        up.add("s_n", p_n or [0], np.int32)
        up.add("s_seed", seed_state(0) * max(1, n_pitch_jobs), np.uint64)
        up.add("s_wsoff", s_wsoff or [0], np.int64)
        up.add("s_cap", p_n or [1], np.int32)
        up.add("win_chunk", win_chunk, np.int32)
        up.add("tf_skip", tf_skip, np.int32)
        up.add("tf_base", chunk_tf_base, np.int64)
        d = up.commit(dev, spans=True)

        # one zero-filled output arena, copied back in one D2H
        ar = _Arena()
        for name, n, dt in (("chroma", n_chunks * 12, np.float32), ("tuning", n_chunks, np.float32),
                            ("tmargin", n_chunks, np.int32),
                            ("clag", n_cp, np.int32), ("cmargin", n_cp, np.float64), ("vals", TV + PV, np.float64), ("energy", n_win, np.float64),
                            ("active", n_win, np.uint8), ("bpm", n_win, np.float64), ("lag", n_win, np.int32),
                            ("nbeats", n_win, np.int32), ("margin", n_win, np.float64), ("prior", B, np.float64),
                            ("bout", 3 * nj, np.float64), ("sout", 3 * max(1, n_pitch_jobs), np.float64),
                            ("npk", n_chunks, np.int32)):
            ar.add(name, n, dt)
        o = ar.commit(dev, spans=True)
        tvals, pvals = o["vals"][:TV], o["vals"][TV:]

        # ---------------------------------------------------------------- 3. plan ready -> stream 2
        # the chroma chain runs on stream 2, concurrently with the window/tempo chain; the
        # consensus tail joins them.  With shared tuning frames the window stage appends the
        # leading frames' piptrack peaks to this group's peak lists (its own, zeroed in the
        # arena) and the chroma chain waits for them before the tuning select.
        s1, s2 = torch.cuda.current_stream(dev), self.chroma_stream
        stage_ev: Dict[str, torch.cuda.Event] = {}

        def stage_copy(stage: str, stream, parts) -> None:
            """With streamed logs: copy a stage's results back as soon as it completes (into
            the places of the pinned mirror the final copy also fills, before the final
            copy's stream waits on this one)."""
            if stream_logs:
                with torch.cuda.stream(stream):
                    ar.copy_parts(parts)
                    e = torch.cuda.Event()
                    e.record(stream)
                    stage_ev[stage] = e
        peaks = None
        ev_stft = None
        if share:
            # peak lists from a ring of GROUPS_IN_FLIGHT + 1 workspaces: a slot comes back only
            # after the host has waited for the group that used it (analyze's in-flight bound),
            # so no large per-group allocation reaches the caching allocator
            n_slots = int(chunk_tf_base[n_chunks]) * PEAK_SLOTS
            ring = max(self.GROUPS_IN_FLIGHT, self.MAX_GROUPS_IN_FLIGHT) + 1
            self._peak_ring = (getattr(self, "_peak_ring", -1) + 1) % ring
            pk = self.workspace(f"peaks{self._peak_ring}", 8 * n_slots)
            for s_ in (s1, self.chroma_stream):
                pk.record_stream(s_)
            peaks = (pk[:4 * n_slots].view(torch.float32), pk[4 * n_slots:8 * n_slots].view(torch.float32))
            ev_stft = torch.cuda.Event()
            ev_stft.record(s1)          # creates the event; the window stage re-records it after the STFT
        ev_plan = torch.cuda.Event()
        ev_plan.record(s1)
        s2.wait_event(ev_plan)
        st2 = s2.cuda_stream

        # ---------------------------------------------------------------- 4. per-window stage
        bpm, lag, nbeats, margin, prior = o["bpm"], o["lag"], o["nbeats"], o["margin"], o["prior"]
        energy, active = o["energy"], o["active"]
        if n_win:
            onset = torch.empty(n_win * T, dtype=torch.float32, device=dev)
            tg = torch.empty(n_win * acw, dtype=torch.float64, device=dev)
            wsb = self.ctx.lib.nc_window_stage_workspace_bytes(self.ctx.h, n_win, win_n, HOP_LENGTH)
            ws = self.workspace("win", wsb)
            # window energies (io._rms_db): from the silence trim's f64 block sums when the batch
            # was trimmed (the STFT then skips its per-frame energy), else fused into the STFT
            en_ptr = energy.data_ptr()
            if blocks is not None:
                tb = blocks[0]
                self.call("nc_window_energy_blocks", signals.buf.data_ptr(), tb.ws.data_ptr(), tb.f1 - tb.f0,
                          tb.off.data_ptr(), d["win_off"].data_ptr(), d["win_file"].data_ptr(), n_win, win_n,
                          en_ptr, st)
                tb.ws.record_stream(torch.cuda.current_stream(dev))
                en_ptr = None
            if share:
                self.call("nc_window_stage_tuning", signals.buf.data_ptr(), d["win_off"].data_ptr(), None, n_win,
                          win_n, HOP_LENGTH, onset.data_ptr(), tg.data_ptr(), en_ptr,
                          d["win_chunk"].data_ptr(), d["tf_base"].data_ptr(), tp, peaks[0].data_ptr(),
                          peaks[1].data_ptr(), o["npk"].data_ptr(), ev_stft.cuda_event, ws.data_ptr(), ws.numel(), st)
            else:
                self.call("nc_window_stage", signals.buf.data_ptr(), d["win_off"].data_ptr(), None, n_win, win_n,
                          HOP_LENGTH, onset.data_ptr(), tg.data_ptr(), en_ptr, ws.data_ptr(), ws.numel(),
                          st)

        # ---------------------------------------------------------------- 3b. chroma (stream 2)
        if n_chunks:
            tot_len = int(np.sum(chunk_len))
            wsb = self.ctx.lib.nc_chroma_workspace_bytes(self.ctx.h, n_chunks, tot_len)
            ws_c = self.workspace("chroma", wsb)
            ws_c.record_stream(s2)  # used on stream 2: not reusable until that work is done
            if share:
                self.call("nc_chroma_mean_shared", signals.buf.data_ptr(), d["chunk_off"].data_ptr(),
                          d["chunk_len"].data_ptr(), n_chunks, tot_len, int(max(chunk_len)), o["chroma"].data_ptr(),
                          o["tuning"].data_ptr(), None, o["tmargin"].data_ptr(), d["tf_skip"].data_ptr(),
                          int(tf_skip.sum()),
                          peaks[0].data_ptr(), peaks[1].data_ptr(), o["npk"].data_ptr(), ev_stft.cuda_event,
                          ws_c.data_ptr(), ws_c.numel(), st2)
            else:
                self.call("nc_chroma_mean", signals.buf.data_ptr(), d["chunk_off"].data_ptr(),
                          d["chunk_len"].data_ptr(), n_chunks, tot_len, int(max(chunk_len)), o["chroma"].data_ptr(),
                          o["tuning"].data_ptr(), None, o["tmargin"].data_ptr(), ws_c.data_ptr(), ws_c.numel(), st2)
            self.call("nc_chroma_lag_margin", o["chroma"].data_ptr(), d["lag_src"].data_ptr(),
                      d["lag_nc"].data_ptr(), n_cp, o["clag"].data_ptr(), o["cmargin"].data_ptr(), st2)
            self.call("nc_pitch_hz", o["clag"].data_ptr(), n_cp, pvals[0:n_cp].data_ptr(),
                      pvals[n_cp:2 * n_cp].data_ptr(), pvals[2 * n_cp:3 * n_cp].data_ptr(), st2)
        n_boot = C.N_BOOTSTRAP
        il, gl, ih, gh = percentile_params(n_boot, C.CI_LEVEL)
        bout, sout = o["bout"], o["sout"]
        if n_pitch_jobs:
            # chunk-shift bootstrap (pitch.py:143-150, seed 0): needs only the chroma chain
            ws2 = self.workspace("boot_s", s_tot)
            ws2.record_stream(s2)
            self.call("nc_bootstrap_ratio", o["vals"].data_ptr(), d["s_off"].data_ptr(), d["s_n"].data_ptr(), None,
                      None, n_pitch_jobs, n_boot, d["s_seed"].data_ptr(), il, gl, ih, gh, MIN_CHUNKS,
                      sout[0:n_pitch_jobs].data_ptr(), sout[n_pitch_jobs:2 * n_pitch_jobs].data_ptr(),
                      sout[2 * n_pitch_jobs:3 * n_pitch_jobs].data_ptr(), None, d["s_wsoff"].data_ptr(),
                      d["s_cap"].data_ptr(), ws2.data_ptr(), ws2.numel(), st2)
        stage_copy("pitch", s2, ["clag", "cmargin", ("vals", TV, TV + PV), "sout", "chroma", "tuning", "tmargin"])
        ev_chroma = torch.cuda.Event()
        ev_chroma.record(s2)

        # ---------------------------------------------------------------- 4b. tempo (window stream)
        # windows longer than ~66 s do not fit the beat tracker's LDS path: global workspace
        bws, bws_n, btot = None, 0, 0
        if n_win and beat_needs_workspace(T, acw):
            wsb = self.workspace("beats", self.ctx.lib.nc_tempo_beats_workspace_bytes(n_win * T))
            bws, bws_n, btot = wsb.data_ptr(), wsb.numel(), n_win * T
        if n_win:
            self.call("nc_energy_gate", energy.data_ptr(), d["w0"].data_ptr(), d["w1"].data_ptr(), nF,
                      float(p.energy_gate_db), active.data_ptr(), st)
            stage_copy("gate", s1, ["energy", "active"])
            if n_src_w:
                self.call("nc_tempo_beats", onset.data_ptr(), d["on_off"].data_ptr(), d["on_len"].data_ptr(),
                          n_src_w, T, tg.data_ptr(), acw, d["start120"].data_ptr(), d["src_pair"].data_ptr(),
                          active.data_ptr(), HOP_LENGTH, 1, bpm.data_ptr(), lag.data_ptr(), nbeats.data_ptr(),
                          margin.data_ptr(), None, btot, bws, bws_n, st)
            self.call("nc_tempo_prior", bpm.data_ptr(), nbeats.data_ptr(), active.data_ptr(),
                      d["src_w0"].data_ptr(), d["src_w1"].data_ptr(), d["src_len"].data_ptr(),
                      d["nc_len"].data_ptr(), B, prior.data_ptr(), st)
            stage_copy("src", s1, [("bpm", 0, n_src_w), ("nbeats", 0, n_src_w), ("margin", 0, n_src_w), "prior"])
            n_nc_w = n_win - n_src_w
            if n_nc_w:
                self.call("nc_tempo_beats", onset.data_ptr(),
                          d["on_off"][n_src_w:].data_ptr(), d["on_len"][n_src_w:].data_ptr(), n_nc_w, T,
                          tg[n_src_w * acw:].data_ptr(), acw, prior.data_ptr(), d["nc_pair"].data_ptr(),
                          active[n_src_w:].data_ptr(), HOP_LENGTH, 1, bpm[n_src_w:].data_ptr(),
                          lag[n_src_w:].data_ptr(), nbeats[n_src_w:].data_ptr(), margin[n_src_w:].data_ptr(),
                          None, btot, bws, bws_n, st)
            stage_copy("nc", s1, [("bpm", n_src_w, n_win), ("nbeats", n_src_w, n_win), ("margin", n_src_w, n_win)])
            # valid-tempo compaction per side: the counts land in the bootstrap jobs' a_n / b_n
            for side, cnt in (("nc", d["a_n"]), ("src", d["b_n"])):
                self.call("nc_collect_valid", bpm.data_ptr(), nbeats.data_ptr(), active.data_ptr(),
                          d[side + "_w0"].data_ptr(), d[side + "_w1"].data_ptr(), B, MIN_BEATS, tvals.data_ptr(),
                          cnt.data_ptr(), st)
        else:
            prior.fill_(120.0)
            stage_copy("gate", s1, ["prior"])

        # ---------------------------------------------------------------- 5. IBI pass (window stream)
        ibi = None
        if p.compute_ibi:
            ibi = self._ibi_pass(signals, d["f_off"], d["f_len"], f_len, prior, B, p.ibi_beats)
        ev_window = torch.cuda.Event()
        ev_window.record(s1)

        # ---------------------------------------------------------------- 6. bootstraps (tempo + pitch, seed 42)
        # on the tail stream once both chains of this group are done; the window stream is free
        # for the next group's window chain meanwhile
        s3 = self.tail_stream
        s3.wait_event(ev_window)
        s3.wait_event(ev_chroma)
        st3 = s3.cuda_stream
        ws = self.workspace("boot", tot)
        ws.record_stream(s3)
        self.call("nc_bootstrap_ratio", o["vals"].data_ptr(), d["a_off"].data_ptr(), d["a_n"].data_ptr(),
                  d["b_off"].data_ptr(), d["b_n"].data_ptr(), nj, n_boot, d["seed"].data_ptr(), il, gl, ih, gh,
                  C.MIN_VALID, bout[0:nj].data_ptr(), bout[nj:2 * nj].data_ptr(), bout[2 * nj:].data_ptr(), None,
                  d["wsoff"].data_ptr(), d["cap"].data_ptr(), ws.data_ptr(), ws.numel(), st3)

        # ---------------------------------------------------------------- 7. async D2H into pinned buffers
        with torch.cuda.stream(s3):
            hbuf, host = ar.to_host()
            host["pvals"] = host["vals"][TV:]
            pinned = [hbuf]
            if ibi is not None:
                for k, v in ibi.items():
                    if isinstance(v, torch.Tensor):
                        h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
                        h.copy_(v, non_blocking=True)
                        pinned.append(h)
                        host["ibi_" + k] = h.numpy()
                    else:
                        host["ibi_" + k] = v
            ev = torch.cuda.Event()
            ev.record(s3)
        return dict(p=p, host=host, arena=ar.host_layout, pinned=pinned, event=ev, stage_ev=stage_ev,
                    keep=(d, o, ar, ibi, peaks),
                    has_ibi=ibi is not None,
                    align=align,
                    starts=starts, w0=w0, w1=w1, f_len=f_len,
                    strip_len=strip_len, lead=lead, trail=trail, intro=intro, win_n=win_n,
                    pair_chunks=pair_chunks, n_cp=n_cp, nj=nj, n_pitch_jobs=n_pitch_jobs, B=B,
                    spans=[((int(f_off[2 * b + 1] - signals.off[2 * b + 1]), int(f_len[2 * b + 1])),
                            (int(f_off[2 * b] - signals.off[2 * b]), int(f_len[2 * b]))) for b in range(B)]
                    if p.melodia is not None else None)

    def _finish_group(self, g: dict, log=None) -> List[PairOutcome]:
        """Wait for one group's results (sync 2 of that group) and assemble them on the host.
        With ``log``, each pair's lines go out stage by stage as the stages' results land."""
        hs = self.host_stats
        t0 = time.perf_counter()
        if log is None:
            g["event"].synchronize()
        t1 = time.perf_counter()
        if self.host_trace is not None:
            self.host_trace.append((t1, "synced"))
        h = _HostViews(g["host"])
        if log is None:
            # group-wide screens (every result is on the host): a pair's own near-tie and beat
            # capacity checks run only when some pair of the group can trip them
            h["any_nb_neg"] = bool((h["nbeats"] < 0).any())
            h["any_cm_tie"] = bool((h["cmargin"] < NEAR_TIE).any())
            h["any_tm_tie"] = bool((h["tmargin"] <= TUNING_NEAR_TIE).any())
        g["starts_l"] = [x.tolist() for x in g["starts"]]
        g["w0"], g["w1"] = g["w0"].tolist(), g["w1"].tolist()
        ibi = {k[4:]: v for k, v in g["host"].items() if k.startswith("ibi_")} if g["has_ibi"] else None
        ctx = AsmContext(h, ibi, g["starts_l"], g["w0"], g["w1"], g["f_len"], g["strip_len"], g["lead"], g["trail"],
                         g["intro"], g["win_n"], g["pair_chunks"], g["n_cp"], g["nj"], g["n_pitch_jobs"], g["align"],
                         g.get("arena"), g["starts"])
        out = []
        for b in range(g["B"]):
            o = PairOutcome()
            wait = None
            if log is not None:
                wait = _StageWaiter(o, g, h, lambda line, i=g["g0"] + b: log(i, line))
            ctx.assemble(b, g["p"], out=o, wait=wait,
                         span=(g["g0"] + b, g["spans"][b]) if g.get("spans") else None)
            if wait is not None:
                wait.flush()
            out.append(o)
        if hs is not None:
            hs["wait"] = hs.get("wait", 0.0) + t1 - t0
            hs["assemble"] = hs.get("assemble", 0.0) + time.perf_counter() - t1
        return out

    # -------------------------------------------------------------- IBI pass (tempo.py:120-173)
    def ibi_core(self, buf, d_off, d_len, f_len, start_vals, pidx, hop: int = IBI_HOP, min_ibis: int = 4,
                 ws_tag: str = ""):
        """onset(hop) -> streamed tempogram mean -> beat_track -> IBIs for every
        file (tempo.py:158-172); start bpm of file f = start_vals[pidx[f]]."""
        dev, st = self.dev, self.stream()
        nF = len(f_len)
        frames = 1 + np.asarray(f_len, np.int64) // hop
        total = int(frames.sum())
        onset = torch.empty(max(1, total), dtype=torch.float32, device=dev)
        fbase = torch.empty(nF + 1, dtype=torch.int64, device=dev)
        wsb = self.ctx.lib.nc_ibi_onset_workspace_bytes(self.ctx.h, nF, total)
        ws = self.workspace(ws_tag + "ibi_on", wsb)
        self.call("nc_ibi_onset", buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), nF, total, hop,
                  onset.data_ptr(), fbase.data_ptr(), ws.data_ptr(), ws.numel(), st)
        acw = int(int(8.0 * self.sr) // hop)
        tg = torch.empty(nF * acw, dtype=torch.float64, device=dev)
        fmax = int(frames.max())
        wsb = self.ctx.lib.nc_ibi_tempogram_workspace_bytes(self.ctx.h, nF, total, fmax, hop)
        ws = self.workspace(ws_tag + "ibi_tg", wsb)
        self.call("nc_ibi_tempogram", onset.data_ptr(), fbase.data_ptr(), nF, total, fmax, hop, tg.data_ptr(),
                  ws.data_ptr(), ws.numel(), st)
        lens = h2d(frames, np.int32, dev)
        bpm = torch.zeros(nF, dtype=torch.float64, device=dev)
        lag = torch.zeros(nF, dtype=torch.int32, device=dev)
        nb = torch.zeros(nF, dtype=torch.int32, device=dev)
        mg = torch.zeros(nF, dtype=torch.float64, device=dev)
        beats = torch.empty(max(1, total), dtype=torch.int32, device=dev)
        wsb = self.ctx.lib.nc_tempo_beats_workspace_bytes(total)
        ws = self.workspace(ws_tag + "ibi_beats", wsb)
        self.call("nc_tempo_beats", onset.data_ptr(), fbase.data_ptr(), lens.data_ptr(), nF, int(frames.max()),
                  tg.data_ptr(), acw, start_vals.data_ptr(), pidx.data_ptr(), None, hop, 1, bpm.data_ptr(),
                  lag.data_ptr(), nb.data_ptr(), mg.data_ptr(), beats.data_ptr(), total, ws.data_ptr(), ws.numel(),
                  st)
        ibis = torch.empty(max(1, total), dtype=torch.float64, device=dev)
        nibi = torch.zeros(nF, dtype=torch.int32, device=dev)
        self.call("nc_ibi_from_beats", beats.data_ptr(), fbase.data_ptr(), nb.data_ptr(), nF, hop, min_ibis,
                  ibis.data_ptr(), nibi.data_ptr(), st)
        fb_h = np.concatenate([[0], np.cumsum(frames)]).astype(np.int64)
        return dict(onset=onset, fbase=fbase, fbase_h=fb_h, frames=frames, tg=tg, bpm=bpm, lag=lag, nbeats=nb,
                    margin=mg, beats=beats, ibis=ibis, nibi=nibi)

    def _ibi_pass(self, signals, d_off, d_len, f_len, prior, B, keep_beats=False):
        dev, st = self.dev, self.stream()
        nF = 2 * B
        starts = torch.cat([_tensor(prior)[:B], torch.full((1,), 120.0, dtype=torch.float64, device=dev)])
        pidx = h2d([f // 2 if f % 2 == 0 else B for f in range(nF)], np.int32, dev)
        core = self.ibi_core(signals.buf, d_off, d_len, f_len, starts, pidx)
        frames, fb_h, ibis, nibi = core["frames"], core["fbase_h"], core["ibis"], core["nibi"]
        nb, bpm, lag, mg = core["nbeats"], core["bpm"], core["lag"], core["margin"]
        # bootstrap: A = src ibis, B = nc ibis (consensus.py:303-307), seed 42, need >= 4 each
        caps = [int(frames[2 * b] // 32 + frames[2 * b + 1] // 32 + 4) for b in range(B)]
        wsoff, tot = [], 0
        for c in caps:
            wsoff.append(tot)
            tot += self.ctx.lib.nc_bootstrap_job_bytes(c, C.N_BOOTSTRAP)
        up = _Upload()
        up.add("a_off", [fb_h[2 * b + 1] for b in range(B)], np.int64)
        up.add("b_off", [fb_h[2 * b] for b in range(B)], np.int64)
        up.add("seed", seed_state(42) * B, np.uint64)
        up.add("wsoff", wsoff, np.int64)
        up.add("cap", caps, np.int32)
        dd = up.commit(dev)
        src_i = torch.arange(1, nF, 2, device=dev)
        nc_i = torch.arange(0, nF, 2, device=dev)
        a_n = nibi[src_i].contiguous()
        b_n = nibi[nc_i].contiguous()
        out = torch.full((3 * B,), float("nan"), dtype=torch.float64, device=dev)
        ws = self.workspace("boot_ibi", tot)
        il, gl, ih, gh = percentile_params(C.N_BOOTSTRAP, C.CI_LEVEL)
        self.call("nc_bootstrap_ratio", ibis.data_ptr(), dd["a_off"].data_ptr(), a_n.data_ptr(),
                  dd["b_off"].data_ptr(), b_n.data_ptr(), B, C.N_BOOTSTRAP, dd["seed"].data_ptr(), il, gl, ih, gh,
                  4, out[0:B].data_ptr(), out[B:2 * B].data_ptr(), out[2 * B:].data_ptr(), None,
                  dd["wsoff"].data_ptr(), dd["cap"].data_ptr(), ws.data_ptr(), ws.numel(), st)
        res = dict(out=out, nibi=nibi, nbeats=nb, bpm=bpm, lag=lag, margin=mg)
        if keep_beats:
            res.update(beats=core["beats"], fbase=fb_h)
        return res

# ------------------------------------------------------------------------------ host assembly + logs
class _Lines:
    """A deferred log entry: ``fn(*args)`` renders the line (or lines) when the outcome's logs
    are first read.  ``fn`` is a module-level function and ``args`` plain values, so an
    unrendered outcome pickles (the window-sharded gather sends outcomes to other ranks without
    formatting ~130 lines per pair; sharded.GatheredOutcomes)."""
    __slots__ = ("fn", "args")

    def __init__(self, fn, *args):
        self.fn, self.args = fn, args

    def __call__(self):
        return self.fn(*self.args)

    def __reduce__(self):
        return (_Lines, (self.fn,) + tuple(self.args))


# the deferred lines of assemble_pair (pipeline.py:77-215's text)
def _log_strip(top_db, lead_n, trail_n, len_n, lead_s, trail_s, len_s):
    return [f"Stripping silence (top_db={top_db} dB)…",
            f"  nightcore: −{lead_n:.2f}s leading, −{trail_n:.2f}s trailing  →  {len_n / SR:.1f} s",
            f"  source:    −{lead_s:.2f}s leading, −{trail_s:.2f}s trailing  →  {len_s / SR:.1f} s"]


def _log_slicing(window_sec, hop_sec, n_nc, n_src, gate_db):
    return [f"Slicing into {window_sec:.0f} s windows (hop {hop_sec:.0f} s)…",
            f"  nightcore: {n_nc} windows  |  source: {n_src} windows",
            f"Energy gating (threshold {gate_db} dB below peak)…"]


def _log_gated(n_nc, n_src):
    return f"  after gating — nightcore: {n_nc} windows  |  source: {n_src} windows"


def _log_chroma(point_st, lo_st, hi_st, n):
    return (f"    Chroma xcorr: {point_st:+.3f} st  95% CI [{lo_st:+.3f}, {hi_st:+.3f}] st"
            f"  ({n} chunk{'s' if n != 1 else ''})")


def _log_tempo_windows(starts, win_n):
    """``starts``: the sample offsets of the pair's gated windows of one file, in order."""
    n = len(starts)
    return [f"    tempo window {i + 1}/{n}  [{s / SR:.1f}–{(s + win_n) / SR:.1f} s]"
            for i, s in enumerate(starts.tolist())]


def _log_confident(n_conf, n):
    return f"    {n_conf}/{n} windows yielded a confident tempo estimate"


def _log_prior(prior, med, ratio):
    return f"  NC tempo prior: {prior:.1f} BPM  (src median {med:.1f} BPM × dur ratio {ratio:.4f})"


def _log_ibi(r, lo, hi):
    return f"  IBI ratio: {r:.6f}×  95% CI [{lo:.6f}, {hi:.6f}]"


def assemble_pair(b, p: Params, h, ibi, starts, w0, w1, f_len, strip_len, lead, trail, intro,
                  win_n, pair_chunks, n_cp, nj, n_pitch_jobs, align=None, out: Optional[PairOutcome] = None,
                  wait=None, span=None) -> PairOutcome:
    """One pair's AnalysisResult (or run()'s exception) and its log lines, in the order of
    pipeline.py:77-215, from the host views of its group.  ``wait(stage)`` ("gate",
    "pitch", "src", "nc", "final") is called before the lines that need a stage's
    results (streamed logs); without it every result is already on the host."""
    out = out if out is not None else PairOutcome()
    wait = wait or (lambda stage: None)
    L = out._log_ops.append   # str, or a callable rendering the line(s) when logs are read
    fn, fs = 2 * b, 2 * b + 1
    nc_len, src_len = int(f_len[fn]), int(f_len[fs])
    if p.silence_strip_db is not None:
        L(_Lines(_log_strip, p.silence_strip_db, float(lead[fn]), float(trail[fn]), float(strip_len[fn]),
                 float(lead[fs]), float(trail[fs]), float(strip_len[fs])))
    if p.src_trim_sec > 0.0:
        L(f"Manual source trim: skipping {p.src_trim_sec:.2f}s from source start")
    elif align is not None:                              # pipeline.py:111-125
        raw, spd = align
        L("Detecting intro offset (RMS envelope alignment)…")
        if raw >= ALIGN_MIN_OFFSET:
            L(f"  Intro detected — trimming {raw:.2f}s from source start  (speed hint: {spd:.4f}×)")
        else:
            L(f"  No significant intro offset detected  (raw: {raw:.2f}s < {ALIGN_MIN_OFFSET:.1f}s threshold)")
    L(_Lines(_log_slicing, p.window_sec, p.hop_sec, len(starts[fn]), len(starts[fs]), p.energy_gate_db))
    wait("gate")
    act = h["active_l"]
    src_w = [w for w in range(w0[fs], w1[fs]) if act[w]]
    nc_w = [w for w in range(w0[fn], w1[fn]) if act[w]]
    L(_Lines(_log_gated, len(nc_w), len(src_w)))
    out.detail.update(energy_src=h["energy"][w0[fs]:w1[fs]].copy(), energy_nc=h["energy"][w0[fn]:w1[fn]].copy(),
                      n_src_windows=len(src_w), n_nc_windows=len(nc_w),
                      nc_duration=nc_len / SR, src_duration=src_len / SR)
    if not nc_w or not src_w:
        out.error = RuntimeError("All windows were discarded by the energy gate.  "
                                 "Try raising --energy-gate (e.g. --energy-gate -60).")
        return out

    # pitch
    pitch_boot = None
    if p.compute_pitch:
        L("Estimating pitch (chromagram cross-correlation)…")
        c0, c1 = pair_chunks[b]
        n = c1 - c0
        wait("pitch")
        lags = h["clag_l"][c0:c1]
        pv = h["pvals_l"]
        src_p = pv[2 * n_cp + c0:2 * n_cp + c1]
        nc_p = pv[n_cp + c0:n_cp + c1]
        point_st = C._median(pv[c0:c1])          # the shifts, as python floats
        if n >= MIN_CHUNKS:
            j = b
            lo_st, hi_st = h["sout_l"][n_pitch_jobs + j], h["sout_l"][2 * n_pitch_jobs + j]
        else:
            lo_st = hi_st = point_st
            L(f"    Only {n} chunk(s) available (need ≥ {MIN_CHUNKS}) — "
              "pitch CI is degenerate; estimate may be less reliable.")
        L(_Lines(_log_chroma, point_st, lo_st, hi_st, n))
        pick = None
        if p.melodia is None or span is None:
            L("    essentia not available — skipping MELODIA refinement")
        else:
            lines: List[str] = []
            pick = p.melodia(span[0], point_st, lines.append, span[1])   # batch pair index, trimmed spans
            out._melodia = (pick, list(lines), None)
            for x in lines:
                L(x)
        method = "chroma+melodia" if pick is not None else "chroma_xcorr"
        if pick is not None:
            src_p, nc_p = pick
        L(f"  Pitch method: {method}")
        margins = h["cmargin"][c0:c1].copy()
        tmargins = h["tmargin"][2 * c0:2 * c1].copy() if "tmargin" in h else None
        out.detail.update(chunk_lags=lags, chunk_lag_margin=margins, tuning=h["tuning"][2 * c0:2 * c1].copy(),
                          chroma=h["chroma"][24 * c0:24 * c1].reshape(-1, 12).copy(), tuning_margin=tmargins)
        if h.get("any_cm_tie", True) and len(margins) and margins.min() < NEAR_TIE:
            # not in the reference's log stream (kept identical); Python logging only
            _logger.info("chroma lag near-tie in pair %d: chunk(s) %s, relative margin %s", b,
                         np.flatnonzero(margins < NEAR_TIE).tolist(), np.round(margins[margins < NEAR_TIE], 6).tolist())
        if h.get("any_tm_tie", True) and tmargins is not None and len(tmargins) and tmargins.min() <= TUNING_NEAR_TIE:
            # a tuning histogram whose best bin leads by <= 1 residual: one peak decides the
            # CQT's fmin shift, so an f32 / f64 difference in a single peak could flip it
            _logger.info("tuning near-tie in pair %d: chunk(s) %s (src, nc interleaved), count margin %s", b,
                         np.flatnonzero(tmargins <= TUNING_NEAR_TIE).tolist(),
                         tmargins[tmargins <= TUNING_NEAR_TIE].tolist())
    else:
        L("Skipping pitch estimation.")
        src_p, nc_p, method = [], [], None

    # tempo
    L("Estimating tempo (librosa)…")
    tempos = {}
    for side, ws_ in (("src", src_w), ("nc", nc_w)):
        if side == "src":
            L("  ← source →")
        vals = []
        f = fs if side == "src" else fn
        st_f, base = starts[f], w0[f]
        nws = len(ws_)
        L(_Lines(_log_tempo_windows, np.asarray(st_f)[np.asarray(ws_, np.int64) - base], win_n))
        wait(side)
        bpm_l, nb_l = h["bpm_l"], h["nbeats_l"]
        if h.get("any_nb_neg", True) and any(nb_l[w] < 0 for w in ws_):
            # the device beat list overflowed its capacity: an engine limit, not "no tempo"
            out.error = _native.NativeError(f"beat tracker capacity exceeded in a {side} window of pair {b}")
            return out
        vals = [bpm_l[w] if nb_l[w] >= MIN_BEATS else None for w in ws_]
        L(_Lines(_log_confident, sum(1 for v in vals if v is not None), nws))
        tempos[side] = vals
        if side == "src":
            valid_src = [t for t in vals if t is not None]
            nc_dur, src_dur = nc_len / SR, src_len / SR
            if valid_src and nc_dur > 0 and src_dur > 0:
                med = C._median(valid_src)
                pr_ = h['prior_l'][b]
                L(_Lines(_log_prior, pr_, med, src_dur / nc_dur))
            L("  ← nightcore →")
    out.detail.update(src_tempos=tempos["src"], nc_tempos=tempos["nc"], nc_start_bpm=h["prior_l"][b],
                      tempo_margin_src=h["margin"][src_w].copy(), tempo_margin_nc=h["margin"][nc_w].copy())
    L("Computing consensus…")
    wait("final")
    if p.compute_pitch and method == "chroma+melodia":
        vs, vn = C._valid(src_p), C._valid(nc_p)
        if len(vs) >= C.MIN_VALID and len(vn) >= C.MIN_VALID:
            # consensus.py:550-553 on the MELODIA lists (a gathered outcome rebuilt on another
            # rank replays the owner's answer: sharded._MelodiaReplay)
            pitch_boot = getattr(p.melodia, "pitch_boot", None) or C._bootstrap_ratio(vn, vs)
            out._melodia = out._melodia[:2] + (pitch_boot,)
    elif p.compute_pitch:
        pj = len(w0) // 2 + b     # pitch job index: after the B tempo jobs
        bo = h["bout_l"]
        pitch_boot = (bo[pj], (bo[nj + pj], bo[2 * nj + pj]))
    try:
        bo = h["bout_l"]
        tempo_boot = (bo[b], (bo[nj + b], bo[2 * nj + b]))
        res = C.assemble(src_p, nc_p, tempos["src"], tempos["nc"], nc_duration=nc_len / SR,
                         src_duration=src_len / SR, pitch_boot=pitch_boot, tempo_boot=tempo_boot)
    except ValueError as exc:
        out.error = exc
        return out
    res.intro_offset_sec = intro
    res.pitch_method = method
    if ibi is not None:
        L("Computing IBI ratio (high-precision beat timestamps, hop=64)…")
        nb_ = ibi["nibi"]
        Bn = len(nb_) // 2
        if nb_[2 * b] >= 4 and nb_[2 * b + 1] >= 4:
            o = ibi["out"]
            res.ibi_ratio = float(o[b])
            res.ibi_ci = (float(o[Bn + b]), float(o[2 * Bn + b]))
            L(_Lines(_log_ibi, res.ibi_ratio, res.ibi_ci[0], res.ibi_ci[1]))
        else:
            L("  IBI ratio: insufficient beats — skipped")
        out.detail.update(ibi_nbeats=(int(ibi["nbeats"][2 * b]), int(ibi["nbeats"][2 * b + 1])),
                          ibi_n=(int(nb_[2 * b]), int(nb_[2 * b + 1])),
                          ibi_lag=(int(ibi["lag"][2 * b]), int(ibi["lag"][2 * b + 1])))
        if "beats" in ibi:
            fb, bt, nbt = ibi["fbase"], ibi["beats"], ibi["nbeats"]
            out.detail["ibi_beats"] = tuple(bt[fb[f]:fb[f] + max(0, int(nbt[f]))].copy() for f in (fn, fs))
    L("Done.")
    out.result = res
    return out


_tls = threading.local()
_live: "weakref.WeakSet[Engine]" = weakref.WeakSet()     # engines not yet collected (tests, diagnostics)


def get_engine(device: Optional[int] = None, sr: int = SR) -> Engine:
    """This thread's engine for ``device`` — contexts are not shared across threads.  The
    engine lives in thread-local storage, so it (its context, streams and HBM workspaces) is
    released when the thread ends: the reference's GUI starts a fresh QThread per analysis
    (gui/worker.py:16-56), and a long session must not keep one engine per finished thread.
    ``release_engine`` frees it earlier.  ``sr``: an engine whose tables are built for that
    sample rate (the tempo seams at other rates), kept beside the 22 050 Hz one."""
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    engines = getattr(_tls, "engines", None)
    if engines is None:
        engines = _tls.engines = {}
    key = device if int(sr) == SR else (device, int(sr))
    e = engines.get(key)
    if e is None:
        e = engines[key] = Engine(device, int(sr))
        _live.add(e)
    return e


def release_engine(device: Optional[int] = None) -> None:
    """Close this thread's engine for ``device`` (every device when None) after its queued
    work: the next get_engine on this thread builds a new one."""
    engines = getattr(_tls, "engines", None) or {}
    for d in [d for d in engines if device is None or (d[0] if isinstance(d, tuple) else d) == device]:
        engines.pop(d).close()


def live_engines() -> int:
    """Engines still alive in this process (every thread's)."""
    gc.collect()
    return len(_live)
