"""Window-sharded analysis across ranks: the items of a batch of (nightcore, source)
pairs — 10 s windows and 20 s chunk pairs — are split over the GPUs of a node, so one
pair can span GPUs.

north_star: "the 10 s / 5 s-hop windows over both input files are the natural shard
unit: partition them across the GPUs with an RCCL gather of per-window estimates over
xGMI before consensus".  SURVEY.md §8(e) lays the split out and this module follows it:

* **Item plan** (``shard_plan``, host, identical on every rank, from the untrimmed file
  lengths alone).  Every pair contributes, in pair-major order, its source window slots,
  its nightcore window slots and its chunk-pair slots (a chunk pair weighs CP_COST
  windows: its CQT chain costs about that much device time).  Slot counts come from the
  untrimmed lengths; silence trimming only shortens a file, so a slot past the trimmed
  count is simply empty.  The weighted item line is cut into one contiguous block per
  rank.  A pair belongs to the rank holding its first item (its *owner*: consensus, IBI,
  report).  Most pairs lie inside one block (*interior*); only the pairs a block boundary
  cuts (*split pairs*, at most world - 1 of them when there are more pairs than ranks)
  need an exchange.
* **Rank r loads, uploads and trims only the pairs it touches.**
* **Interior pairs** run through the pipelined single-GPU engine (``Engine._analyze_gen``:
  pair groups on three HIP streams, up to three in flight), with no collective at all.
* **Split pairs** run stage by stage on a fourth stream, interleaved with the interior
  groups (the host advances the engine's group pipeline between stages, so the device
  always has queued work while the host waits on an exchange):
    1. windows of this rank's slots: energy, onset, tempogram mean (K1-K5), and the tempo
       of its source windows at start_bpm 120 (tempo.py:27-77, K6-K8);
                                           C1a: all-gather of the split pairs' window records
    2. energy gate of each file over its gathered energies (io.py:115-126); nc prior of
       each pair from its gathered source records (pipeline.py:174-183); tempo of this
       rank's nightcore windows with their pair's prior; this rank's chunk pairs
       (tuning, CQT chroma, lag: K9-K11, pitch.py:121-138);
                                           C1b: all-gather of window + chunk-pair records
    3. the owner runs the bootstraps (consensus.py:243-312, pitch.py:143-150), the hop-64
       IBI pass (tempo.py:120-173) and the host assembly (report, warnings, logs).
* The results of every pair are gathered to every rank (``gather=True``, the API
  default) as record tables, no pickle: per pair a fixed-size result row and, per assembly
  group, the inputs ``assemble_pair`` read (``pack_outcomes``).  One all-gather moves every
  rank's bytes to every rank (device tensors over RCCL); a rank reads all result rows as one
  table (``GatheredOutcomes.table``) and rebuilds another rank's whole outcome (report,
  logs, detail) with the same ``assemble_pair`` call on first access.  The benchmark's N > 1
  headline times the gather and the table read of every step.

The records are fixed-size f64 rows.  They are assembled on the host from the stage
results (a few hundred bytes per window), copied to the exchange device on the split-pair
stream and gathered with ``all_gather_into_tensor`` (device tensors over RCCL with the
"nccl" backend, CPU tensors with gloo), then read back.  Blocks of unequal size are padded
to the largest.  When no pair is split (equal pairs, B divisible by the world size:
BASELINE config 4) the plan has no exchange on the data path.

**Fail together.**  Every rank runs the same sequence of collectives, fixed by the plan
alone.  A local exception is never raised where it happens: it is held and carried, as
the rank's error flag, into the next collective, and every collective either returns on
every rank or raises on every rank (the failing rank's own exception there, ``ShardError``
on the others).  With ``steps`` > 1 an error after a step's last collective rides into the
next step's first gather; the interior pipeline's errors are held by the pump and raised
after the last split-pair collective, before the final flag check.

The split-pair stages run over a small stage interface: ``DeviceStages`` (libncgpu on
this rank's GPU) or, in the multi-process CPU tests, the oracle
(``tests/sharded_oracle.OracleStages``), so the plan, the exchange, the prior and the
consensus placement are tested without a GPU.  Every result equals the single-rank
``Engine.analyze`` result of the same batch.
"""
from __future__ import annotations

import collections.abc
import contextlib
import dataclasses
import gc
import json
import math
import operator
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import consensus as C
from .distributed import shard_range
from .engine import (CHUNK_SEC, HOP_LENGTH, IBI_HOP, MIN_BEATS, MIN_CHUNKS, REF_HZ, SR, AsmContext, DeviceSignals,
                     Engine, PairOutcome, Params, _HostViews, _TrimBlocks, _Upload, plan_batch)

# exchanged window record: exists, energy_db, bpm, nbeats, tempo lag, decision margin
R_EXISTS, R_ENERGY, R_BPM, R_NBEATS, R_LAG, R_MARGIN = range(6)
W_FIELDS = 6
# chunk-pair record: exists, lag, tuning (src, nc), mean chroma (src 12, nc 12), lag margin,
# tuning decision margins (src, nc)
CP_FIELDS = 1 + 3 + 24 + 1 + 2
CP_COST = 8          # a chunk pair's weight in the item line, in windows
IBI_TILE = 2048      # frames per tempogram tile (csrc/ibi.hip TG_TB): the IBI frame split's unit
IBI_PAD = 1 + 1024 // IBI_HOP   # onset_strength's lag + n_fft // (2 hop) left pad at hop 64


class ShardError(RuntimeError):
    """Another rank of a window-sharded run failed (its own exception is raised there)."""


# ------------------------------------------------------------------------------ item plan
def n_window_slots(L: int, win_n: int, hop_n: int) -> int:
    """io.slice_windows' count for a file of L samples (io.py:82-112)."""
    return (L - win_n) // hop_n + 1 if L >= win_n and hop_n > 0 else 0


@dataclass
class ShardPlan:
    """Item blocks of every rank (see the module docstring).  rng[b, s, r] = slot range
    [lo, hi) of segment s (0 source windows, 1 nightcore windows, 2 chunk pairs) of pair b
    on rank r."""
    world: int
    B: int
    slots: np.ndarray          # [B, 3]
    rng: np.ndarray            # [B, 3, world, 2]
    owner: np.ndarray          # [B]
    split: np.ndarray          # [B] bool
    wrow: np.ndarray           # [B] first exchange-table window row of a split pair (-1 otherwise)
    crow: np.ndarray           # [B] first exchange-table chunk row of a split pair (-1 otherwise)
    n_wrows: int
    n_crows: int

    def on_rank(self, b: int, r: int) -> bool:
        return bool(np.any(self.rng[b, :, r, 1] > self.rng[b, :, r, 0]))

    def _present(self) -> np.ndarray:
        """[B, world] bool: pair b has items on rank r."""
        return np.any(self.rng[:, :, :, 1] > self.rng[:, :, :, 0], axis=1)

    def touched(self, r: int) -> List[int]:
        return np.flatnonzero((self.owner == r) | self._present()[:, r]).tolist()

    def needed(self, r: int, ibi: bool) -> List[int]:
        """Pairs rank r must hold: the ones it touches, and with the hop-64 IBI pass every
        split pair (the pass of a split pair's files is split over all ranks, C2-C4)."""
        m = (self.owner == r) | self._present()[:, r]
        return np.flatnonzero(m | (self.split if ibi else False)).tolist()

    def owned(self, r: int) -> List[int]:
        return np.flatnonzero(self.owner == r).tolist()

    def window_row(self, b: int, side: int, k: int) -> int:
        return int(self.wrow[b] + (k if side == 0 else self.slots[b, 0] + k))

    def contrib_w(self, r: int) -> np.ndarray:
        """Exchange-table window rows rank r computes (split pairs, ascending)."""
        rows = []
        for b in np.flatnonzero(self.split):
            for side in (0, 1):
                lo, hi = self.rng[b, side, r]
                rows += [self.window_row(b, side, k) for k in range(lo, hi)]
        return np.asarray(rows, np.int64)

    def contrib_c(self, r: int) -> np.ndarray:
        rows = []
        for b in np.flatnonzero(self.split):
            lo, hi = self.rng[b, 2, r]
            rows += [int(self.crow[b] + k) for k in range(lo, hi)]
        return np.asarray(rows, np.int64)


def shard_plan(lengths: Sequence[int], p: Params, world: int, split_offset: float = 0.0) -> ShardPlan:
    """The item blocks of a batch whose files (nc_0, src_0, nc_1, src_1, ...) have the given
    untrimmed lengths.  ``split_offset`` moves every inner block boundary by that fraction
    of a mean pair (0: plain equal blocks; 0.5 cuts every boundary through a pair's middle,
    which is how the exchange is measured on batches whose blocks would otherwise align)."""
    L = np.asarray(lengths, np.int64)
    B = len(L) // 2
    win_n, hop_n = int(p.window_sec * SR), int(p.hop_sec * SR)
    cn = int(CHUNK_SEC * SR)
    ln, ls = L[0::2], L[1::2]

    def n_slots(x):  # n_window_slots, vectorised
        return np.where((x >= win_n) & (hop_n > 0), (x - win_n) // max(hop_n, 1) + 1, 0)

    slots = np.stack([n_slots(ls), n_slots(ln),
                      np.maximum(1, np.minimum(ls // cn, ln // cn)) if p.compute_pitch else np.zeros(B, np.int64)],
                     axis=1).astype(np.int64).reshape(B, 3)
    cost = slots[:, 0] + slots[:, 1] + CP_COST * slots[:, 2]
    base = np.concatenate([[0], np.cumsum(cost)]).astype(np.int64)
    T = int(base[-1])
    bounds = np.array([T * r // world for r in range(world + 1)], np.int64)
    if split_offset and B:
        shift = int(round(split_offset * T / B))
        bounds[1:world] = np.clip(bounds[1:world] + shift, 0, T)
    bounds = np.maximum.accumulate(bounds)
    bounds[world] = np.iinfo(np.int64).max // 4          # every unit < T lies in some block

    # segment s of pair b starts at unit u0[b, s] and spends `stride` units per slot; rank r
    # holds the slots whose first unit lies in [bounds[r], bounds[r + 1])
    u0 = np.stack([base[:-1], base[:-1] + slots[:, 0], base[:-1] + slots[:, 0] + slots[:, 1]], axis=1)
    stride = np.array([1, 1, CP_COST], np.int64)
    edge = -(-(bounds[None, None, :] - u0[:, :, None]) // stride[None, :, None])    # [B, 3, world + 1]
    edge = np.minimum(slots[:, :, None], np.maximum(0, edge))
    rng = np.stack([edge[:, :, :-1], edge[:, :, 1:]], axis=3)                         # [B, 3, world, 2]
    first = np.minimum(base[:-1], max(T - 1, 0))
    owner = np.clip(np.searchsorted(bounds, first, side="right") - 1, 0, world - 1).astype(np.int64)
    present = rng[:, :, :, 1] > rng[:, :, :, 0]                                       # [B, 3, world]
    others = np.ones((B, world), bool)
    others[np.arange(B), owner] = False
    split = np.any(present & others[:, None, :], axis=(1, 2))
    wrow = np.full(B, -1, np.int64)
    crow = np.full(B, -1, np.int64)
    sw = slots[split, 0] + slots[split, 1]
    wrow[split] = np.concatenate([[0], np.cumsum(sw)[:-1]]) if sw.size else sw
    crow[split] = np.concatenate([[0], np.cumsum(slots[split, 2])[:-1]]) if sw.size else sw
    return ShardPlan(world, B, slots, rng, owner, split, wrow, crow, int(sw.sum()), int(slots[split, 2].sum()))


# ------------------------------------------------------------------------------ exchange
class Exchange:
    """Fixed-size f64 record gathers over the default (or given) process group.

    ``device``: where the exchanged tensors live.  Default: this rank's GPU under RCCL
    ("nccl"), the CPU under gloo.  A test may pass a CUDA device with gloo to run the
    device-tensor code (upload and gather on the split-pair stream, read-back) on one GPU."""

    def __init__(self, group=None, device: Optional[torch.device] = None):
        self.group = group
        self.on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.on else 1
        self.rank = dist.get_rank(group) if self.on else 0
        backend = dist.get_backend(group) if self.on else "gloo"
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.dev = torch.device(device)

    stream: Optional[torch.cuda.Stream] = None    # RCCL: the stream the exchanged records live on
    # run the collectives at world size 1 too (tests: a one-rank RCCL group takes the
    # device-tensor path on the box's one GPU, tests/test_gpu_rccl.py)
    collect_at_one: bool = False

    @property
    def local(self) -> bool:
        """No collective is issued: no process group, or one rank (unless collect_at_one)."""
        return not self.on or (self.world == 1 and not self.collect_at_one)

    def gather_blocks(self, local: np.ndarray, counts: Sequence[int], failed: Optional[BaseException]) -> np.ndarray:
        """Rank r contributes counts[r] rows of k f64; returns the rows of every rank in rank
        order (one all_gather_into_tensor of (max count + 1 flag row) x k per rank).  A
        failure anywhere raises on every rank.  With RCCL the collective is ordered on
        ``stream`` (the split-pair stream), not behind the interior groups of the launch
        stream."""
        if self.dev.type == "cuda" and self.stream is not None:
            with torch.cuda.stream(self.stream):
                return self._gather_blocks(local, counts, failed)
        return self._gather_blocks(local, counts, failed)

    def _gather_blocks(self, local: np.ndarray, counts: Sequence[int], failed: Optional[BaseException]) -> np.ndarray:
        k = local.shape[1]
        if self.local:
            if failed is not None:
                raise failed
            return np.ascontiguousarray(local, np.float64)
        S = int(max(counts)) if len(counts) else 0
        mine = np.zeros((S + 1, k), np.float64)
        if failed is None:
            mine[:local.shape[0]] = local
        mine[S, 0] = 1.0 if failed is not None else 0.0
        t = torch.from_numpy(mine).to(self.dev, non_blocking=self.dev.type == "cuda")
        out = torch.empty((self.world * (S + 1), k), dtype=torch.float64, device=self.dev)
        dist.all_gather_into_tensor(out, t, group=self.group)
        allr = out.cpu().numpy().reshape(self.world, S + 1, k)
        bad = [r for r in range(self.world) if allr[r, S, 0] != 0.0]
        if failed is not None:
            raise failed
        if bad:
            raise ShardError(f"window-sharded analysis failed on rank(s) {bad}")
        return np.concatenate([allr[r, :counts[r]] for r in range(self.world)], axis=0) if S else np.zeros((0, k))

    def allreduce_max(self, vals: np.ndarray, failed: Optional[BaseException]) -> np.ndarray:
        """Element-wise maximum over the ranks (C2: power_to_db's top_db reference of a file
        whose frames are split); the error flag rides along as one more element."""
        if self.local:
            if failed is not None:
                raise failed
            return np.asarray(vals, np.float64)
        buf = np.concatenate([np.asarray(vals, np.float64), [1.0 if failed is not None else 0.0]])
        if self.dev.type == "cuda" and self.stream is not None:
            # the upload, the collective and the read-back all on the split-pair stream: the
            # host waits for this exchange only, not for the interior groups queued on the
            # launch stream
            with torch.cuda.stream(self.stream):
                t = torch.from_numpy(buf).to(self.dev, non_blocking=True)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                out = t.cpu().numpy()
        else:
            t = torch.from_numpy(buf).to(self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            out = t.cpu().numpy()
        if failed is not None:
            raise failed
        if out[-1] != 0.0:
            raise ShardError("window-sharded analysis failed on another rank")
        return out[:-1]

    def check(self, failed: Optional[BaseException]) -> None:
        """Fail together: one flag gather."""
        self.gather_blocks(np.zeros((0, 1)), [0] * self.world, failed)

    def gather_objects(self, local: list) -> list:
        if self.local:
            return list(local)
        buf: List[Optional[list]] = [None] * self.world
        dist.all_gather_object(buf, local, group=self.group)
        out: list = []
        for part in buf:
            out.extend(part)
        return out

    def gather_bytes(self, blob: bytes, failed: Optional[BaseException] = None) -> List[memoryview]:
        """Every rank's byte string, in rank order: one all_gather_into_tensor of the lengths
        and one of the strings padded to the longest (uint8; device tensors under RCCL, on the
        split-pair stream).  The parts are views of one host buffer: nothing is copied per rank.
        Fail together: a rank with ``failed`` sends length -1 instead, and every rank raises
        after the first collective (that rank its own exception, the others ShardError)."""
        if self.local:
            if failed is not None:
                raise failed
            return [memoryview(blob)]
        ctx = torch.cuda.stream(self.stream) if self.dev.type == "cuda" and self.stream is not None \
            else contextlib.nullcontext()
        with ctx:
            n = torch.tensor([-1 if failed is not None else len(blob)], dtype=torch.int64).to(self.dev)
            ns = torch.empty(self.world, dtype=torch.int64, device=self.dev)
            dist.all_gather_into_tensor(ns, n, group=self.group)
            sizes = ns.cpu().tolist()
            if failed is not None:
                raise failed
            bad = [q for q in range(self.world) if sizes[q] < 0]
            if bad:
                raise ShardError(f"window-sharded result gather failed on rank(s) {bad}")
            S = max(1, int(max(sizes)))
            mine = np.zeros(S, np.uint8)
            mine[:len(blob)] = np.frombuffer(blob, np.uint8)
            t = torch.from_numpy(mine).to(self.dev)
            out = torch.empty(self.world * S, dtype=torch.uint8, device=self.dev)
            dist.all_gather_into_tensor(out, t, group=self.group)
            h = memoryview(out.cpu().numpy())
        return [h[q * S:q * S + int(sizes[q])] for q in range(self.world)]


# ------------------------------------------------------------------------------ result records
# The gather of every pair's outcome to every rank (gather=True) sends plain arrays, no pickle:
# per owned pair a fixed-size result row (RES_FIELDS: the AnalysisResult numbers a caller reads
# first) and, per assembly group, the inputs assemble_pair read (engine.AsmContext: the group's
# host result arrays and plan).  A receiving rank reads the result rows as one table
# (GatheredOutcomes.table) and rebuilds a whole PairOutcome (report text, warnings, logs, detail)
# with the same assemble_pair call on first access.
RES_FIELDS = ("ok", "tempo_ratio", "tempo_lo", "tempo_hi", "pitch_ratio", "pitch_lo", "pitch_hi", "ibi_ratio",
              "ibi_lo", "ibi_hi", "n_source_pitch_windows", "n_nc_pitch_windows", "n_source_tempo_windows",
              "n_nc_tempo_windows", "nc_duration", "src_duration", "nc_median_bpm", "src_median_bpm",
              "intro_offset_sec")
_NAN = float("nan")


def _opt(v) -> float:
    return _NAN if v is None else float(v)


_ROW_GET = operator.attrgetter("tempo_ratio", "tempo_ci", "pitch_ratio", "pitch_ci", "ibi_ratio", "ibi_ci",
                                "n_source_pitch_windows", "n_nc_pitch_windows", "n_source_tempo_windows",
                                "n_nc_tempo_windows", "nc_duration", "src_duration", "nc_median_bpm",
                                "src_median_bpm", "intro_offset_sec")
_ERR_ROW = (0.0,) + (_NAN,) * (len(RES_FIELDS) - 1)


def result_row(o: PairOutcome) -> tuple:
    """The RES_FIELDS row of one outcome (None where the result has None: the f64 table makes
    it NaN; ok = 0 for an error outcome)."""
    r = o.result
    if r is None:
        return _ERR_ROW
    tr, tc, pr, pc, ir, ic, a, b, c, d, e, f, g, h, i = _ROW_GET(r)
    ic = ic or (None, None)
    return (1.0, tr, tc[0], tc[1], pr, pc[0], pc[1], ir, ic[0], ic[1], a, b, c, d, e, f, g, h, i)


_DTYPES: Dict[str, np.dtype] = {}


def pack_tables(tables: Dict[str, np.ndarray], views: Optional[Dict[str, tuple]] = None) -> bytes:
    """Named numeric arrays as one byte string: an 8-byte header length, a JSON header (name,
    dtype, shape, offset of each array) and the raw bytes.  Arrays of one dtype are laid out
    back to back (one concatenation per dtype, each dtype block 8-byte aligned).  ``views``:
    {name: (table name, byte offset, dtype str, shape)} — arrays that are stretches of another
    table's bytes, sent as header entries only (an arena's views)."""
    groups: Dict[str, list] = {}
    for name, a in tables.items():
        a = np.asarray(a)
        if a.dtype.kind not in "biuf":
            raise TypeError(f"record table {name!r}: dtype {a.dtype} is not numeric")
        groups.setdefault(a.dtype.str, []).append((name, a))
    chunks, off, at = [], 0, {}
    for dt, items in groups.items():
        flat = [a.reshape(-1) for _, a in items]
        block = np.concatenate(flat) if len(flat) > 1 else np.ascontiguousarray(flat[0])
        isz = block.itemsize
        o = off
        for name, a in items:
            at[name] = (dt, a.shape, o)
            o += a.size * isz
        if block.nbytes:
            chunks.append(block.view(np.uint8))
        pad = -block.nbytes % 8
        if pad:
            chunks.append(bytes(pad))
        off += block.nbytes + pad
    meta = [(name,) + at[name] for name in tables]            # the tables' own order
    for name, (base, o, dt, shape) in (views or {}).items():
        meta.append((name, dt, shape, at[base][2] + o))
    head = json.dumps(meta, separators=(",", ":")).encode()
    head += b" " * (-len(head) % 8)
    return b"".join([len(head).to_bytes(8, "little"), head] + chunks)


def unpack_tables(buf) -> Dict[str, np.ndarray]:
    """pack_tables' arrays as read-only views of ``buf`` (nothing is copied)."""
    mv = memoryview(buf)
    n = int.from_bytes(mv[:8], "little")
    base = 8 + n
    out = {}
    for name, dt, shape, off in json.loads(bytes(mv[8:base])):
        d = _DTYPES.get(dt)
        if d is None:
            d = _DTYPES[dt] = np.dtype(dt)
        a = np.frombuffer(mv, d, math.prod(shape), base + off)
        out[name] = a if len(shape) == 1 else a.reshape(tuple(shape))
    return out


def _list_array(v) -> np.ndarray:
    a = np.asarray(v)
    if a.dtype.kind not in "biuf":
        raise TypeError(f"assembly list of dtype {a.dtype} cannot travel as a record")
    return a if a.size else np.zeros(0, np.float64)


def _ctx_tables(ctx: AsmContext, pre: str, out: Dict[str, np.ndarray], views: Dict[str, tuple]) -> None:
    """An assembly context as arrays (keys prefixed ``pre``).  Host views: every array, not the
    derived python lists ("x_l" is rebuilt from "x" by _HostViews) nor the engine's boolean
    screens; a list with no array behind it (the split-pair path's "clag_l", ...) as its array.
    The views still carved from the group's host arena travel as the arena's bytes once plus
    a header entry each (``views``)."""
    h = ctx.h
    lay = {}
    if ctx.arena is not None:
        hb, lay = ctx.arena
        out[pre + "arena"] = hb
    for k, v in h.items():
        if k.startswith("ibi_") or isinstance(v, bool):
            continue
        if k.endswith("_l"):
            if k[:-2] not in h:
                out[pre + "h." + k[:-2]] = _list_array(v)
            continue
        a = lay.get(k)
        if a is not None and a[0] is v:
            views[pre + "h." + k] = (pre + "arena", a[1], v.dtype.str, v.shape)
        else:
            out[pre + "h." + k] = np.asarray(v)
    if ctx.ibi is not None:
        for k, v in ctx.ibi.items():
            out[pre + "i." + k] = np.asarray(v)
    starts = ctx.starts_a if ctx.starts_a is not None else ctx.starts
    starts = [np.asarray(s, np.int64) for s in starts]
    out[pre + "starts"] = np.concatenate(starts) if starts else np.zeros(0, np.int64)
    out[pre + "starts_n"] = np.array([len(s) for s in starts], np.int64)
    out[pre + "w0"] = np.asarray(ctx.w0, np.int64)
    out[pre + "w1"] = np.asarray(ctx.w1, np.int64)
    for k in ("f_len", "strip_len", "lead", "trail"):
        out[pre + k] = np.asarray(getattr(ctx, k))
    out[pre + "intro"] = np.array(ctx.intro, np.float64).reshape(-1)       # None -> NaN
    out[pre + "intro_none"] = np.array([v is None for v in ctx.intro], np.bool_)
    if ctx.align is not None:
        out[pre + "align"] = np.array([(_NAN, _NAN) if a is None else a for a in ctx.align], np.float64).reshape(-1, 2)
        out[pre + "align_none"] = np.array([a is None for a in ctx.align], np.bool_)
    out[pre + "chunks"] = np.array(ctx.pair_chunks, np.int64).reshape(-1, 2)
    out[pre + "scal"] = np.array([ctx.win_n, ctx.n_cp, ctx.nj, ctx.n_pitch_jobs, ctx.ibi is not None], np.int64)


def _ctx_from_tables(t: Dict[str, np.ndarray], pre: str) -> AsmContext:
    """_ctx_tables' inverse: the same values, types and python lists assemble_pair reads."""
    n = len(pre)
    h = _HostViews({k[n + 2:]: v for k, v in t.items() if k.startswith(pre + "h.")})   # (arena views included)
    win_n, n_cp, nj, n_pj, has_ibi = t[pre + "scal"].tolist()
    ibi = {k[n + 2:]: v for k, v in t.items() if k.startswith(pre + "i.")} if has_ibi else None
    flat, cnt = t[pre + "starts"].tolist(), t[pre + "starts_n"].tolist()
    starts, o = [], 0
    for c in cnt:
        starts.append(flat[o:o + c])
        o += c
    intro = [None if none else v for v, none in zip(t[pre + "intro"].tolist(), t[pre + "intro_none"].tolist())]
    align = None
    if pre + "align" in t:
        align = [None if none else tuple(a) for a, none in zip(t[pre + "align"].tolist(), t[pre + "align_none"].tolist())]
    chunks = [tuple(c) for c in t[pre + "chunks"].tolist()]
    return AsmContext(h, ibi, starts, t[pre + "w0"].tolist(), t[pre + "w1"].tolist(), t[pre + "f_len"],
                      t[pre + "strip_len"], t[pre + "lead"], t[pre + "trail"], intro, win_n, chunks, n_cp, nj, n_pj,
                      align)


def _melodia_tables(rec, pre: str, out: Dict[str, np.ndarray]) -> None:
    """The MELODIA hook's answer on the owner (engine.assemble_pair): its (src, nc) Hz lists or
    None, its log lines, and the bootstrap of the accepted lists."""
    pick, lines, boot = rec
    out[pre + "lines"] = np.frombuffer("\0".join(lines).encode(), np.uint8)
    out[pre + "nlines"] = np.array([len(lines)], np.int64)
    if pick is not None:
        for side, vals in zip(("src", "nc"), pick):
            out[pre + side] = np.array([_opt(v) for v in vals], np.float64)
            out[pre + side + "_none"] = np.array([v is None for v in vals], np.bool_)
    if boot is not None:
        out[pre + "boot"] = np.array([boot[0], boot[1][0], boot[1][1]], np.float64)


class _MelodiaReplay:
    """The receiving rank's MELODIA hook: the owner's lines and answer, and its bootstrap."""

    def __init__(self, t: Dict[str, np.ndarray], pre: str):
        self.lines = bytes(t[pre + "lines"]).decode().split("\0") if int(t[pre + "nlines"][0]) else []
        self.pick = None
        if pre + "src" in t:
            self.pick = tuple([None if none else v for v, none in zip(t[pre + s].tolist(),
                                                                      t[pre + s + "_none"].tolist())]
                              for s in ("src", "nc"))
        self.pitch_boot = None
        if pre + "boot" in t:
            pt, lo, hi = t[pre + "boot"].tolist()
            self.pitch_boot = (pt, (lo, hi))

    def __call__(self, _b, _point_st, log, _span):
        for x in self.lines:
            log(x)
        return self.pick


class _StepRecords:
    """One rank's owned outcomes of one step as records, built a segment at a time (``add``:
    the engine's pipeline adds each pair group as it is assembled, while later groups are still
    on the device; the split pairs are added after their consensus).  ``bytes()``: a fixed
    prefix the result table reads without parsing anything else — the row, segment and
    context counts, "pairs" = (pair, context, index in the context) int64 rows, "res" =
    RES_FIELDS f64 rows, the segment of each context and the segment lengths — then the
    segments: pack_tables of each distinct assembly context once ("c<k>.…") and the MELODIA
    hook's recorded answer where it ran ("m<pair>.…"), parsed only when an outcome is rebuilt."""

    def __init__(self):
        self.rows: List[Tuple[int, int, int]] = []
        self.res: List[tuple] = []
        self.ctx_seg: List[int] = []
        self.segs: List[bytes] = []

    def add(self, outs) -> None:
        ctx_id: Dict[int, int] = {}
        tables: Dict[str, np.ndarray] = {}
        views: Dict[str, tuple] = {}
        for b, o in outs:
            a = o._asm
            if a is None:
                if o != PairOutcome():
                    raise ValueError(f"pair {b}'s outcome was not built by assemble_pair: it cannot travel as records")
                self.rows.append((b, -1, 0))   # an empty outcome (nothing to rebuild)
                self.res.append(_ERR_ROW)
                continue
            ctx, j = a
            k = ctx_id.get(id(ctx))
            if k is None:
                k = ctx_id[id(ctx)] = len(self.ctx_seg)
                self.ctx_seg.append(len(self.segs))
                _ctx_tables(ctx, f"c{k}.", tables, views)
            self.rows.append((b, k, j))
            self.res.append(result_row(o))
            if o._melodia is not None:
                _melodia_tables(o._melodia, f"m{b}.", tables)
        if tables:
            self.segs.append(pack_tables(tables, views))

    def bytes(self) -> bytes:
        n = len(self.rows)
        head = np.array([n, len(self.segs), len(self.ctx_seg)], np.int64).tobytes()
        return b"".join([head, np.array(self.rows, np.int64).tobytes(),
                         np.array(self.res, np.float64).reshape(n, len(RES_FIELDS)).tobytes(),
                         np.array(self.ctx_seg, np.int64).tobytes(),
                         np.array([len(x) for x in self.segs], np.int64).tobytes()] + self.segs)


def pack_outcomes(outs: List[Tuple[int, PairOutcome]]) -> bytes:
    """A rank's owned [(global pair index, outcome)] of one step as records (_StepRecords, one
    segment)."""
    rec = _StepRecords()
    rec.add(outs)
    return rec.bytes()


class _Part:
    """One rank's records of one step: the result rows read in place, a segment's assembly
    tables parsed on the first rebuild of one of its pairs."""
    __slots__ = ("raw", "pairs", "res", "ctx_seg", "seg", "t", "ctx", "where")

    def __init__(self, raw):
        mv = memoryview(raw)
        if len(mv) < 24:
            raise ShardError(f"a gathered record part of {len(mv)} bytes has no header")
        n, ns, nc = np.frombuffer(mv, np.int64, 3).tolist()
        o = 24 + 8 * n * (3 + len(RES_FIELDS)) + 8 * (nc + ns)
        if min(n, ns, nc) < 0 or len(mv) < o:
            raise ShardError(f"a gathered record part of {len(mv)} bytes is shorter than its header says")
        self.pairs = np.frombuffer(mv, np.int64, 3 * n, 24).reshape(n, 3)
        self.res = np.frombuffer(mv, np.float64, len(RES_FIELDS) * n, 24 + 24 * n).reshape(n, len(RES_FIELDS))
        self.ctx_seg = np.frombuffer(mv, np.int64, nc, o - 8 * (nc + ns))
        ends = o + np.cumsum(np.frombuffer(mv, np.int64, ns, o - 8 * ns))
        if ns and ends[-1] > len(mv):
            raise ShardError(f"a gathered record part of {len(mv)} bytes is shorter than its segments")
        self.seg = [(int(e - l), int(e)) for l, e in zip(np.diff(ends, prepend=o), ends)]
        self.raw = mv
        self.t: Dict[int, Dict[str, np.ndarray]] = {}
        self.ctx: Dict[int, AsmContext] = {}
        self.where = None

    def tables(self, seg: int) -> Dict[str, np.ndarray]:
        t = self.t.get(seg)
        if t is None:
            a, e = self.seg[seg]
            t = self.t[seg] = unpack_tables(self.raw[a:e])
        return t

    def outcome(self, b: int, p: Params) -> Optional[PairOutcome]:
        if self.where is None:
            self.where = {x: i for i, x in enumerate(self.pairs[:, 0].tolist())}
        i = self.where.get(b)
        if i is None:
            return None
        _, k, j = self.pairs[i].tolist()
        if k < 0:
            return PairOutcome()
        t = self.tables(int(self.ctx_seg[k]))
        ctx = self.ctx.get(k)
        if ctx is None:
            ctx = self.ctx[k] = _ctx_from_tables(t, f"c{k}.")
        span, q = None, p
        if f"m{b}.nlines" in t:        # replay the owner's MELODIA answer and lines
            q, span = dataclasses.replace(p, melodia=_MelodiaReplay(t, f"m{b}.")), (b, None)
        elif p.melodia is not None:
            q = dataclasses.replace(p, melodia=None)
        return ctx.assemble(j, q, span=span)


class GatheredOutcomes(collections.abc.Sequence):
    """Every pair's outcome on every rank, in pair order (``analyze_sharded`` with
    ``gather=True``).  This rank's own outcomes are the objects it assembled; the other ranks'
    arrived as record tables (``pack_outcomes``, one byte all-gather per call) and are rebuilt by
    assemble_pair on first access to one of their pairs.  ``table()`` returns every pair's
    RES_FIELDS row without rebuilding anything.  Indexing, slicing, iteration, ``len`` and
    comparison with a list behave as on the list of outcomes."""

    def __init__(self, n: int, owner: np.ndarray, own: Sequence[Tuple[int, PairOutcome]],
                 parts: Dict[int, memoryview], p: Optional[Params] = None):
        self._n = int(n)
        self._owner = np.asarray(owner)
        self._items: Dict[int, PairOutcome] = dict(own)
        self._parts = {q: _Part(v) for q, v in parts.items()}
        self._p = p or Params()
        self._table = None

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        i = int(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError("pair index out of range")
        o = self._items.get(i)
        if o is None:
            part = self._parts.get(int(self._owner[i]))
            o = part.outcome(i, self._p) if part is not None else None
            if o is None:
                raise ShardError(f"pair {i} is missing from rank {int(self._owner[i])}'s gathered outcomes")
            self._items[i] = o
        return o

    def __iter__(self):
        for i in range(self._n):
            yield self[i]

    def __eq__(self, other):
        return isinstance(other, collections.abc.Sequence) and list(self) == list(other)

    def table(self) -> np.ndarray:
        """[pair][RES_FIELDS] f64 (NaN for None): the other ranks' rows straight from their
        records, this rank's from its own outcomes."""
        if self._table is None:
            tab = np.full((self._n, len(RES_FIELDS)), np.nan)
            for part in self._parts.values():
                tab[part.pairs[:, 0]] = part.res
            own = [(b, o) for b, o in self._items.items() if int(self._owner[b]) not in self._parts]
            if own:
                tab[[b for b, _ in own]] = [result_row(o) for _, o in own]
            self._table = tab
        return self._table

    def decoded(self) -> int:
        """How many pairs are still only records (diagnostics)."""
        return self._n - len(self._items)

    def __repr__(self) -> str:
        return f"GatheredOutcomes({self._n} pairs, {self.decoded()} not yet rebuilt from records)"


# Fault-injection points of the fail-together tests (tests/test_sharded_cpu.py): host-only
# steps ("records", "consensus") mapped to the call (1-based) that raises.  Empty in use.
FAULTS: dict = {}


def _fault(point: str) -> None:
    if point in FAULTS:
        FAULTS[point] -= 1
        if FAULTS[point] == 0:
            raise RuntimeError(f"injected failure in {point}")


def _try(fn, *args):
    """(result, None), or (None, the exception) for an ``Exception`` (carried into the next
    collective).  KeyboardInterrupt, SystemExit and GeneratorExit propagate at once: an
    interrupt is not a stage failure to deliver to the other ranks, and it reaches them too."""
    try:
        return fn(*args), None
    except Exception as exc:           # noqa: BLE001 - re-raised after the collective
        return None, exc


# ------------------------------------------------------------------------------ device stages
class DeviceStages:
    """The stage operations of one rank on its GPU (libncgpu), over signals resident in HBM
    (files nc_0, src_0, nc_1, src_1, ... of the pairs this rank touches, one buffer).  The
    stages run on their own HIP stream with their own workspaces ("sp_*"), so they overlap
    the engine's pipelined interior groups without sharing scratch with them."""

    def __init__(self, eng: Engine, signals: DeviceSignals, stream: Optional[torch.cuda.Stream] = None):
        self.eng = eng
        self.sig = signals
        self.off = signals.off
        self.length = signals.length
        self._win = None
        self._blocks = None     # the last trim's block sums (the window energies come from them)
        if stream is None:
            stream = getattr(eng, "_split_stream", None) or torch.cuda.Stream(eng.dev)
            eng._split_stream = stream
        self.stream = stream
        self.stream.wait_stream(torch.cuda.current_stream(eng.dev))   # the upload of the signals

    def restrict(self, files: Sequence[int]) -> "DeviceStages":
        f = np.asarray(files, np.int64)
        return DeviceStages(self.eng, DeviceSignals(self.sig.buf, self.off[f], self.length[f]), self.stream)

    def pipeline(self, files: Sequence[int], p: Params, steps: int = 1, on_group=None):
        """The engine's pipelined group generator over the pairs of `files` (interior pairs),
        ``steps`` complete analyses back to back (Engine.analyze_batches); ``on_group(step,
        first pair, outcomes)`` as each group is assembled (Engine._analyze_gen)."""
        f = np.asarray(files, np.int64)
        return self.eng._analyze_gen([DeviceSignals(self.sig.buf, self.off[f], self.length[f])] * steps, p, None,
                                     None, on_group)

    def trim(self, p: Params) -> Tuple[np.ndarray, np.ndarray]:
        with torch.cuda.stream(self.stream):
            eng = self.eng
            nF = self.sig.n_files
            up = _Upload()
            up.add("off", self.off, np.int64)
            up.add("len", self.length, np.int64)
            d0 = up.commit(eng.dev)
            lens = np.ascontiguousarray(self.length, np.int64)
            # a fresh workspace, kept: its block sums give the window energies (windows()), as
            # in the engine's pipelined groups
            ws = torch.empty(eng.ctx.lib.nc_trim_workspace_bytes(lens.ctypes.data, nF), dtype=torch.uint8,
                             device=eng.dev)
            se = torch.empty(2 * nF, dtype=torch.int64, device=eng.dev)
            eng.call("nc_trim_bounds", self.sig.buf.data_ptr(), d0["off"].data_ptr(), d0["len"].data_ptr(), nF,
                     int(np.sum(1 + lens // 512)), float(p.silence_strip_db), se[:nF].data_ptr(), se[nF:].data_ptr(),
                     ws.data_ptr(), ws.numel(), eng.stream())
            self._blocks = _TrimBlocks(ws, d0["off"], 0, nF, None)
            h = se.cpu().numpy()
        return h[:nF].copy(), h[nF:].copy()

    def align(self, start: np.ndarray, end: np.ndarray) -> List[Tuple[float, float]]:
        o, s = self.sig.off, start
        with torch.cuda.stream(self.stream):
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
        with torch.cuda.stream(self.stream):
            off = torch.from_numpy(np.ascontiguousarray(win_abs, np.int64)).to(eng.dev)
            onset = torch.empty(n * T, dtype=torch.float32, device=eng.dev)
            tg = torch.empty(n * acw, dtype=torch.float64, device=eng.dev)
            en = torch.empty(n, dtype=torch.float64, device=eng.dev)
            ws = eng.workspace("sp_win", eng.ctx.lib.nc_window_stage_workspace_bytes(eng.ctx.h, n, win_n, HOP_LENGTH))
            en_ptr = en.data_ptr()
            tb = self._blocks
            if tb is not None:          # energies from the trim's block sums (engine._launch_group)
                wf = np.searchsorted(np.asarray(self.off, np.int64), np.asarray(win_abs, np.int64), side="right") - 1
                wf_d = torch.from_numpy(wf.astype(np.int32)).to(eng.dev)
                eng.call("nc_window_energy_blocks", self.sig.buf.data_ptr(), tb.ws.data_ptr(), tb.f1 - tb.f0,
                         tb.off.data_ptr(), off.data_ptr(), wf_d.data_ptr(), n, win_n, en_ptr, eng.stream())
                en_ptr = None
            eng.call("nc_window_stage", self.sig.buf.data_ptr(), off.data_ptr(), None, n, win_n, HOP_LENGTH,
                     onset.data_ptr(), tg.data_ptr(), en_ptr, ws.data_ptr(), ws.numel(), eng.stream())
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
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("on_off", np.asarray(sel, np.int64) * T, np.int64)
            up.add("on_len", np.full(n, T), np.int32)
            up.add("start", start_bpm, np.float64)
            up.add("sel", np.asarray(sel, np.int64), np.int64)
            d = up.commit(eng.dev)
            tg = w["tg"].view(-1, acw)[d["sel"]].contiguous()
            res = torch.zeros(4 * n, dtype=torch.float64, device=eng.dev)
            lag = torch.zeros(n, dtype=torch.int32, device=eng.dev)
            nb = torch.zeros(n, dtype=torch.int32, device=eng.dev)
            ws = eng.workspace("sp_beats", eng.ctx.lib.nc_tempo_beats_workspace_bytes(n * T))  # any window length
            eng.call("nc_tempo_beats", w["onset"].data_ptr(), d["on_off"].data_ptr(), d["on_len"].data_ptr(), n, T,
                     tg.data_ptr(), acw, d["start"].data_ptr(), None, None, HOP_LENGTH, 1, res[:n].data_ptr(),
                     lag.data_ptr(), nb.data_ptr(), res[3 * n:].data_ptr(), None, n * T, ws.data_ptr(), ws.numel(),
                     eng.stream())
            res[n:2 * n] = nb.to(torch.float64)
            res[2 * n:3 * n] = lag.to(torch.float64)
            return res.cpu().numpy().reshape(4, n).T.copy()        # one read-back for the four fields

    def chunks(self, chunk_off: Sequence[int], chunk_len: Sequence[int]) -> np.ndarray:
        """Mean chroma of every chunk (files interleaved src, nc per chunk pair) and the
        pair lags -> [n_pairs, 30]: lag, tuning (src, nc), chroma (src 12, nc 12), lag margin,
        tuning margins (src, nc)."""
        eng, n = self.eng, len(chunk_off)
        if n == 0:
            return np.zeros((0, CP_FIELDS - 1), np.float64)
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("off", chunk_off, np.int64)
            up.add("len", chunk_len, np.int64)
            up.add("si", np.arange(0, n, 2), np.int32)
            up.add("ni", np.arange(1, n, 2), np.int32)
            d = up.commit(eng.dev)
            chroma = torch.empty(n * 12, dtype=torch.float32, device=eng.dev)
            tun = torch.empty(n, dtype=torch.float32, device=eng.dev)
            lag = torch.empty(n // 2, dtype=torch.int32, device=eng.dev)
            tmg = torch.empty(n, dtype=torch.int32, device=eng.dev)
            tot = int(np.sum(chunk_len))
            ws = eng.workspace("sp_chroma", eng.ctx.lib.nc_chroma_workspace_bytes(eng.ctx.h, n, tot))
            eng.call("nc_chroma_mean", self.sig.buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(), n, tot,
                     int(max(chunk_len)), chroma.data_ptr(), tun.data_ptr(), None, tmg.data_ptr(), ws.data_ptr(), ws.numel(),
                     eng.stream())
            mg = torch.empty(n // 2, dtype=torch.float64, device=eng.dev)
            eng.call("nc_chroma_lag_margin", chroma.data_ptr(), d["si"].data_ptr(), d["ni"].data_ptr(), n // 2,
                     lag.data_ptr(), mg.data_ptr(), eng.stream())
            rec = torch.cat([lag.to(torch.float64)[:, None], tun.to(torch.float64).view(-1, 2),
                             chroma.to(torch.float64).view(-1, 24), mg[:, None], tmg.to(torch.float64).view(-1, 2)],
                            dim=1)
            return rec.cpu().numpy()

    def bootstrap(self, jobs, seed: int):
        if not jobs:
            return []
        with torch.cuda.stream(self.stream):
            return self.eng.bootstrap(jobs, seed=seed, ws_tag="sp_")

    def ibi(self, f_off: np.ndarray, f_len: np.ndarray, start_bpm: np.ndarray):
        """estimate_ibis_global of each file span -> (ibis (array, or None under 4), IBI
        counts, beat counts, tempo lags)."""
        eng, n = self.eng, len(f_off)
        if n == 0:
            z = np.zeros(0, np.int64)
            return [], z, z, z
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("off", f_off, np.int64)
            up.add("len", f_len, np.int64)
            up.add("start", start_bpm, np.float64)
            d = up.commit(eng.dev)
            core = eng.ibi_core(self.sig.buf, d["off"], d["len"], np.asarray(f_len, np.int64), d["start"],
                                torch.arange(n, dtype=torch.int32, device=eng.dev), ws_tag="sp_")
            vals, nibi = core["ibis"].cpu().numpy(), core["nibi"].cpu().numpy()
            fb = core["fbase_h"]
            ibis = [vals[fb[i]:fb[i] + nibi[i]].copy() if nibi[i] >= 4 else None for i in range(n)]
            return ibis, nibi, core["nbeats"].cpu().numpy(), core["lag"].cpu().numpy()


    # ---- the hop-64 IBI pass of split pairs, split over the ranks (C2-C4; csrc/ibi.hip part D)
    def ibi_mel(self, f_off, f_len, t0, t1) -> np.ndarray:
        """Mel dB rows for this rank's onset frames [t0, t1) of each file -> per-file max."""
        eng, n = self.eng, len(f_off)
        T = 1 + np.asarray(f_len, np.int64) // IBI_HOP
        t0, t1 = np.asarray(t0, np.int64), np.asarray(t1, np.int64)
        rr = _ibi_mel_rows(T, t0, t1)
        rows = int((rr[:, 1] - rr[:, 0]).sum())
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("off", f_off, np.int64)
            up.add("len", f_len, np.int64)
            up.add("t0", t0, np.int64)
            up.add("t1", t1, np.int64)
            d = up.commit(eng.dev)
            ws = eng.workspace("sp_ibi_rng", eng.ctx.lib.nc_ibi_range_workspace_bytes(eng.ctx.h, n, rows))
            mx = torch.empty(n, dtype=torch.float32, device=eng.dev)
            eng.call("nc_ibi_mel_range", self.sig.buf.data_ptr(), d["off"].data_ptr(), d["len"].data_ptr(), n,
                     d["t0"].data_ptr(), d["t1"].data_ptr(), IBI_HOP, rows, mx.data_ptr(), ws.data_ptr(), ws.numel(),
                     eng.stream())
            self._ibi = dict(d=d, ws=ws, rows=rows, n=n, total=int(np.maximum(0, t1 - t0).sum()))
            return mx.cpu().numpy()

    def ibi_onset(self, gmax: np.ndarray) -> np.ndarray:
        """This rank's onset frames [t0, t1) of every file (concatenated) against the global maxima."""
        eng, st = self.eng, self._ibi
        if st["total"] == 0:
            return np.zeros(0, np.float32)
        with torch.cuda.stream(self.stream):
            g = torch.from_numpy(np.asarray(gmax, np.float32)).to(eng.dev)
            out = torch.empty(st["total"], dtype=torch.float32, device=eng.dev)
            eng.call("nc_ibi_onset_range", st["n"], st["d"]["t0"].data_ptr(), IBI_HOP, st["total"], g.data_ptr(),
                     out.data_ptr(), st["ws"].data_ptr(), st["rows"], eng.stream())
            return out.cpu().numpy()

    def ibi_tiles(self, onsets: List[np.ndarray], b0, b1) -> np.ndarray:
        """Tempogram partial rows of this rank's 2048-frame tiles [b0, b1) of each file, from the
        full onsets -> [tiles, N] in (file, tile) order."""
        eng = self.eng
        T = np.array([len(o) for o in onsets], np.int64)
        n, total, mxf = len(T), int(T.sum()), int(T.max())
        N = int(int(8.0 * SR) // IBI_HOP)
        ntb = -(-mxf // IBI_TILE)
        sel = [f * ntb + b for f in range(n) for b in range(int(b0[f]), int(b1[f]))]
        if not sel:
            return np.zeros((0, N))
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("onset", np.concatenate(onsets), np.float32)
            up.add("fb", np.concatenate([[0], np.cumsum(T)]), np.int64)
            up.add("b0", b0, np.int64)
            up.add("b1", b1, np.int64)
            up.add("sel", sel, np.int64)
            d = up.commit(eng.dev)
            slab = torch.zeros(n * ntb * N, dtype=torch.float64, device=eng.dev)
            ws = eng.workspace("sp_ibi_tg", eng.ctx.lib.nc_ibi_tempogram_workspace_bytes(eng.ctx.h, n, total, mxf,
                                                                                        IBI_HOP))
            eng.call("nc_ibi_tempogram_tiles", d["onset"].data_ptr(), d["fb"].data_ptr(), n, total, mxf, IBI_HOP,
                     d["b0"].data_ptr(), d["b1"].data_ptr(), slab.data_ptr(), ws.data_ptr(), ws.numel(), eng.stream())
            return slab.view(n * ntb, N)[d["sel"]].cpu().numpy()

    def ibi_reduce(self, tiles: List[List[np.ndarray]], T: np.ndarray) -> np.ndarray:
        """Fixed-order sum of every tile's row / T_f (nc_ibi_tempogram_reduce) -> [files, N]."""
        eng = self.eng
        n, N = len(tiles), len(tiles[0][0])
        ntb = max(len(t) for t in tiles)
        full = np.zeros((n, ntb, N), np.float64)
        for f, rows in enumerate(tiles):
            full[f, :len(rows)] = np.stack(rows)
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("slab", full, np.float64)
            up.add("fb", np.concatenate([[0], np.cumsum(T)]), np.int64)
            d = up.commit(eng.dev)
            tg = torch.empty(n * N, dtype=torch.float64, device=eng.dev)
            eng.call("nc_ibi_tempogram_reduce", d["slab"].data_ptr(), d["fb"].data_ptr(), n, int(np.max(T)), IBI_HOP,
                     tg.data_ptr(), eng.stream())
            return tg.cpu().numpy().reshape(n, N)

    def ibi_beats(self, onsets: List[np.ndarray], tgs: np.ndarray, start_bpm) -> tuple:
        """beat_track on the full onsets with their tempogram means, then the IBIs
        (tempo.py:158-172) -> (ibis (array, or None under 4), IBI counts, beat counts, tempo lags)."""
        eng = self.eng
        T = np.array([len(o) for o in onsets], np.int64)
        n, total = len(T), int(T.sum())
        N = tgs.shape[1]
        with torch.cuda.stream(self.stream):
            up = _Upload()
            up.add("onset", np.concatenate(onsets), np.float32)
            up.add("fb", np.concatenate([[0], np.cumsum(T)]), np.int64)
            up.add("len", T, np.int32)
            up.add("tg", tgs, np.float64)
            up.add("start", start_bpm, np.float64)
            up.add("pidx", np.arange(n), np.int32)
            d = up.commit(eng.dev)
            bpm = torch.zeros(n, dtype=torch.float64, device=eng.dev)
            lag = torch.zeros(n, dtype=torch.int32, device=eng.dev)
            nb = torch.zeros(n, dtype=torch.int32, device=eng.dev)
            mg = torch.zeros(n, dtype=torch.float64, device=eng.dev)
            beats = torch.empty(max(1, total), dtype=torch.int32, device=eng.dev)
            ws = eng.workspace("sp_ibi_beats", eng.ctx.lib.nc_tempo_beats_workspace_bytes(total))
            eng.call("nc_tempo_beats", d["onset"].data_ptr(), d["fb"].data_ptr(), d["len"].data_ptr(), n, int(T.max()),
                     d["tg"].data_ptr(), N, d["start"].data_ptr(), d["pidx"].data_ptr(), None, IBI_HOP, 1,
                     bpm.data_ptr(), lag.data_ptr(), nb.data_ptr(), mg.data_ptr(), beats.data_ptr(), total,
                     ws.data_ptr(), ws.numel(), eng.stream())
            ibis = torch.empty(max(1, total), dtype=torch.float64, device=eng.dev)
            nibi = torch.zeros(n, dtype=torch.int32, device=eng.dev)
            eng.call("nc_ibi_from_beats", beats.data_ptr(), d["fb"].data_ptr(), nb.data_ptr(), n, IBI_HOP, 4,
                     ibis.data_ptr(), nibi.data_ptr(), eng.stream())
            vals, ni = ibis.cpu().numpy(), nibi.cpu().numpy()
            fb = np.concatenate([[0], np.cumsum(T)])
            out = [vals[fb[i]:fb[i] + ni[i]].copy() if ni[i] >= 4 else None for i in range(n)]
            return out, ni, nb.cpu().numpy(), lag.cpu().numpy()


# ------------------------------------------------------------------------------ orchestration
def _gate(energy: np.ndarray, w0, w1, threshold_db: float) -> np.ndarray:
    """io.energy_gate (io.py:115-126) for every file: keep energy >= file max + threshold."""
    act = np.zeros(len(energy), bool)
    for a, b in zip(w0, w1):
        if b > a:
            e = energy[a:b]
            act[a:b] = e >= e.max() + threshold_db
    return act


def _files(pairs: Sequence[int]) -> List[int]:
    return [f for j in pairs for f in (2 * j, 2 * j + 1)]


class _Pump:
    """Advances the engine's interior group pipeline one group at a time (no-op without one).

    It never raises an ``Exception``: the pump runs between the collectives of the split-pair
    stages, where an exception on one rank would leave the others in a collective.  An
    exception from the pipeline ends it and is kept in ``error``; ``drain`` raises it after the
    last split-pair collective, before the final flag check that every rank meets.
    KeyboardInterrupt, SystemExit and GeneratorExit are not held: they propagate at once."""

    def __init__(self, gen):
        self.gen, self.value, self.error = gen, None, None

    def __call__(self, n: int = 1) -> None:
        for _ in range(n):
            if self.gen is None:
                return
            try:
                next(self.gen)
            except StopIteration as stop:
                self.value, self.gen = stop.value, None
            except Exception as exc:           # noqa: BLE001 - raised by drain(); interrupts propagate
                self.error, self.gen = exc, None

    def drain(self):
        while self.gen is not None:
            self()
        if self.error is not None:
            raise self.error
        return self.value


def analyze_sharded(stages, p: Optional[Params] = None, group=None, *, lengths: Optional[Sequence[int]] = None,
                    local_pairs: Optional[Sequence[int]] = None, split_offset: float = 0.0, gather: bool = True,
                    steps: int = 1, exchange_device: Optional[torch.device] = None):
    """pipeline.run's analysis of a batch with its windows and chunk pairs split over the
    ranks of ``group`` (module docstring).

    ``stages`` holds the signals of the pairs ``local_pairs`` (global pair indices, in
    order; None: every pair of the batch), and ``lengths`` the untrimmed lengths of all
    2B files (None: those of ``stages``, which then holds the whole batch).  With
    ``gather`` every rank returns all outcomes in pair order; without, this rank's owned
    pairs as [(pair index, outcome)].  ``steps`` > 1 analyses the batch that many times
    back to back, the interior groups pipelined across steps as Engine.analyze_batches
    does (the benchmark's timed region), and returns one such list per step.
    ``exchange_device`` overrides where the exchanged records live (``Exchange``).  A
    ``Params.melodia`` hook is called with global pair indices.  Python's cyclic
    collector is paused for the call, as in Engine.analyze (a generation-2 pass, ~10 ms, would
    otherwise stall the host loop that keeps the device queues full)."""
    gc_was_enabled = gc.isenabled()
    gc.disable()
    try:
        return _analyze_sharded(stages, p, group, lengths, local_pairs, split_offset, gather, steps, exchange_device)
    finally:
        if gc_was_enabled:
            gc.enable()


def _local_melodia(p: Params, index: Sequence[int]) -> Params:
    """Params whose melodia hook maps the engine's local pair index to the global one."""
    if p.melodia is None:
        return p
    hook, index = p.melodia, list(index)
    return dataclasses.replace(p, melodia=lambda b, st, log, span: hook(index[b], st, log, span))


def _analyze_sharded(stages, p, group, lengths, local_pairs, split_offset, gather, steps, exchange_device=None):
    p = p or Params()
    ex = Exchange(group, exchange_device)
    r, world = ex.rank, ex.world
    L = np.asarray(stages.length if lengths is None else lengths, np.int64)
    sp = shard_plan(L, p, world, split_offset)
    local_pairs = list(range(sp.B)) if local_pairs is None else list(local_pairs)
    pos = {b: j for j, b in enumerate(local_pairs)}
    ibi_split = p.compute_ibi and world > 1 and bool(sp.split.any())   # C2-C4 for the split pairs
    touched = sp.touched(r)
    needed = sp.needed(r, ibi_split)
    missing = [b for b in needed if b not in pos]
    # held, not raised: the other ranks are about to enter the step's collectives
    err: Optional[BaseException] = \
        ValueError(f"rank {r} needs pairs {missing} that its stages do not hold") if missing else None
    ex.stream = getattr(stages, "stream", None)
    exchange = sp.n_wrows > 0 or sp.n_crows > 0          # identical on every rank
    interior = [b for b in touched if not sp.split[b]] if err is None else []
    fast = getattr(stages, "pipeline", None) is not None and bool(interior)
    stage_pairs = ([b for b in needed if sp.split[b]] if fast else needed) if err is None else []
    # the result gather's records (gather over ranks): the interior groups are packed as the
    # pipeline assembles them, while the later groups still run on the device
    recs = [_StepRecords() for _ in range(steps)] if gather and not ex.local else None

    def on_group(k, g0, outs):
        recs[k].add(list(zip(interior[g0:g0 + len(outs)], outs)))

    pump = _Pump(stages.pipeline(_files([pos[b] for b in interior]), _local_melodia(p, interior), steps,
                                 **({"on_group": on_group} if recs is not None else {}))
                 if fast else None)
    pump(3)                                     # Engine.GROUPS_IN_FLIGHT groups queued before any wait
    split_st = stages.restrict(_files([pos[b] for b in stage_pairs]))
    per_step = []
    for _ in range(steps):
        res, exc = _try(_split_stages, split_st, p, ex, sp, r, stage_pairs, pump, err)
        if exc is not None:                     # a collective raised: it did so on every rank
            err = exc
            break
        outs, err = res
        if err is None:
            per_step.append(outs)
            if recs is not None:
                _, err = _try(recs[len(per_step) - 1].add, outs)
        elif not exchange:                      # no collective before the final check
            break
        # else: the next step's first gather carries the error (or the final check does)
    if err is None and fast:
        res, err = _try(pump.drain)
        if err is None:
            for k in range(steps):
                per_step[k] = per_step[k] + list(zip(interior, res[k]))
    if not ex.local:
        ex.check(err)                           # fail together before the result gather
    elif err is not None:
        raise err
    for outs in per_step:
        outs.sort(key=lambda t: t[0])
    if not gather:
        result = per_step
    elif ex.local:
        result = [[o for _, o in outs] for outs in per_step]
    else:
        # every rank's owned outcomes to every rank as record tables (_StepRecords: result rows
        # and the assembly inputs, plain arrays): one byte all-gather for the call's steps (a
        # rank's part is its steps' blobs behind a table of their lengths); the other ranks'
        # outcomes rebuilt by assemble_pair on access, their result rows readable at once
        blobs, err = _try(lambda: _pack_steps([recs[k].bytes() for k in range(len(per_step))]))
        parts = ex.gather_bytes(blobs or b"", err)          # a packing error raises on every rank
        mine = {q: _unpack_steps(parts[q], len(per_step)) for q in range(world) if q != r}
        result = [GatheredOutcomes(sp.B, sp.owner, outs, {q: mine[q][k] for q in mine}, p)
                  for k, outs in enumerate(per_step)]
    return result[0] if steps == 1 else result


def _pack_steps(blobs: List[bytes]) -> bytes:
    """Several steps' gather blobs as one: their int64 lengths, then the blobs."""
    return np.array([len(b) for b in blobs], np.int64).tobytes() + b"".join(blobs)


def _unpack_steps(part: memoryview, n: int) -> List[memoryview]:
    lens = np.frombuffer(part[:8 * n], np.int64) if n else np.zeros(0, np.int64)
    ends = 8 * n + np.cumsum(lens)
    return [part[int(e - l):int(e)] for l, e in zip(lens, ends)]


def _split_stages(stages, p: Params, ex: Exchange, sp: ShardPlan, r: int, pairs: List[int], pump,
                  err: Optional[BaseException] = None):
    """Stages 1-3 of the module docstring for ``pairs`` (global indices) held by ``stages``
    (files nc, src per pair, in that order) -> ([(pair, outcome)] of the owned ones, held
    error).  ``err`` is an error held from before the step; while one is held no stage runs
    and the error rides into the next collective.  Only the collectives raise, and they raise
    on every rank; a local error after the step's last collective is returned, not raised."""
    nP = len(pairs)
    exchange = sp.n_wrows > 0 or sp.n_crows > 0          # identical on every rank
    cw_cnt = [len(sp.contrib_w(q)) for q in range(sp.world)] if exchange else []
    cc_cnt = [len(sp.contrib_c(q)) for q in range(sp.world)] if exchange else []
    cw_all = np.concatenate([sp.contrib_w(q) for q in range(sp.world)]) if exchange else None
    cc_all = np.concatenate([sp.contrib_c(q) for q in range(sp.world)]) if exchange else None
    cw, cc = sp.contrib_w(r), sp.contrib_c(r)
    st = {}                                              # phase state

    def gather(table_rows, local_rows, local_vals, cnt, all_rows, n_rows, width, failed):
        """Exchange-table rows of the split pairs: this rank's `local_rows` (values
        `local_vals`) in, the whole table out (None without an exchange, where a held error
        simply stays held)."""
        if not exchange:
            return None
        mine = np.zeros((len(table_rows), width), np.float64)   # slots past a trimmed count stay empty
        if failed is None:
            row_of = {int(rw): i for i, rw in enumerate(local_rows) if rw >= 0}
            for i, rw in enumerate(table_rows):
                if int(rw) in row_of:
                    mine[i] = local_vals[row_of[int(rw)]]
        rows = ex.gather_blocks(mine, cnt, failed)
        table = np.zeros((n_rows, width), np.float64)
        table[all_rows.astype(np.int64)] = rows
        return table

    # ---- phase 0: trim, plan, this rank's items; windows + source tempo (start_bpm 120)
    def phase0():
        start, end = stages.trim(p) if (p.silence_strip_db is not None and nP) else \
            (np.zeros(2 * nP, np.int64), np.asarray(stages.length, np.int64).copy())
        align = stages.align(start, end) if (p.auto_align and p.src_trim_sec == 0.0 and nP) else None
        pl = plan_batch(stages.off, stages.length, start, end, p, align)
        pump()
        # this rank's windows (plan indices) and chunk pairs: its slot ranges within the
        # trimmed counts, with the exchange row of each (-1 for pairs whose items are all local)
        wl, wl_src, wl_row, cpl, cpl_row = [], [], [], [], []
        for j, b in enumerate(pairs):
            for side, f in ((0, 2 * j + 1), (1, 2 * j)):
                lo, hi = sp.rng[b, side, r]
                for k in range(lo, min(hi, int(pl.w1[f] - pl.w0[f]))):
                    wl.append(int(pl.w0[f]) + k)
                    wl_src.append(side == 0)
                    wl_row.append(sp.window_row(b, side, k) if sp.split[b] else -1)
            lo, hi = sp.rng[b, 2, r]
            c0, c1 = pl.pair_chunks[j] if p.compute_pitch else (0, 0)
            for k in range(lo, min(hi, c1 - c0)):
                cpl.append(c0 + k)
                cpl_row.append(int(sp.crow[b] + k) if sp.split[b] else -1)
        wl = np.asarray(wl, np.int64)
        wl_src = np.asarray(wl_src, bool)
        rec = np.zeros((len(wl), W_FIELDS), np.float64)
        rec[:, R_EXISTS] = 1.0
        rec[:, R_ENERGY] = stages.windows(pl.win_abs[wl] if len(wl) else np.zeros(0, np.int64), pl.win_n)
        src_sel = np.flatnonzero(wl_src)
        if len(src_sel):
            rec[src_sel, R_BPM:] = stages.tempo(src_sel, np.full(len(src_sel), 120.0))
        pump()
        st.update(pl=pl, align=align, wl=wl, wl_src=wl_src, wl_row=wl_row, cpl=cpl, cpl_row=cpl_row, rec=rec)

    if err is None:
        _, err = _try(phase0)
    gtab = gather(cw, st.get("wl_row", []), st.get("rec"), cw_cnt, cw_all, sp.n_wrows, W_FIELDS, err)       # C1a

    def fill(full, have, table):
        """Plan-order rows of the split pairs' windows held by other ranks, from `table`."""
        pl = st["pl"]
        for j, b in enumerate(pairs):
            if not sp.split[b]:
                continue
            for side, f in ((0, 2 * j + 1), (1, 2 * j)):
                for w in range(int(pl.w0[f]), int(pl.w1[f])):
                    if not have[w]:
                        row = table[sp.window_row(b, side, w - int(pl.w0[f]))]
                        if row[R_EXISTS] != 1.0:
                            raise ShardError(f"window record of pair {b} missing from the exchange")
                        full[w] = row

    # ---- phase 1: gate, nc prior (pipeline.py:174-183), nightcore tempo, chunk pairs
    def phase1():
        pl, wl, wl_src, rec = st["pl"], st["wl"], st["wl_src"], st["rec"]
        full = np.zeros((pl.n_win, W_FIELDS), np.float64)
        have = np.zeros(pl.n_win, bool)
        full[wl] = rec
        have[wl] = True
        if gtab is not None:
            fill(full, have, gtab)
        energy = full[:, R_ENERGY].copy()
        active = _gate(energy, pl.w0, pl.w1, p.energy_gate_db)
        prior = np.full(nP, 120.0)
        pair_of = np.zeros(max(1, pl.n_win), np.int64)
        for j in range(nP):
            fs, fn = 2 * j + 1, 2 * j
            pair_of[pl.w0[fn]:pl.w1[fn]] = j
            pair_of[pl.w0[fs]:pl.w1[fs]] = j
            valid = [full[w, R_BPM] for w in range(int(pl.w0[fs]), int(pl.w1[fs]))
                     if active[w] and full[w, R_NBEATS] >= MIN_BEATS]
            nc_dur, src_dur = pl.f_len[fn] / SR, pl.f_len[fs] / SR
            if valid and nc_dur > 0 and src_dur > 0:
                prior[j] = C._median(valid) * (src_dur / nc_dur)
        nc_sel = np.flatnonzero(~wl_src & active[wl]) if len(wl) else np.zeros(0, np.int64)
        if len(nc_sel):
            rec[nc_sel, R_BPM:] = stages.tempo(nc_sel, prior[pair_of[wl[nc_sel]]])
        pump()
        cpl = st["cpl"]
        crec = np.zeros((len(cpl), CP_FIELDS), np.float64)
        if len(cpl):
            crec[:, 0] = 1.0
            crec[:, 1:] = stages.chunks([pl.chunk_off[2 * c + k] for c in cpl for k in (0, 1)],
                                        [pl.chunk_len[2 * c + k] for c in cpl for k in (0, 1)])
        pump()
        st.update(full=full, have=have, energy=energy, active=active, prior=prior, crec=crec)

    if err is None:
        _, err = _try(phase1)
    gtab = gather(cw, st.get("wl_row", []), st.get("rec"), cw_cnt, cw_all, sp.n_wrows, W_FIELDS, err)       # C1b
    ctab = gather(cc, st.get("cpl_row", []), st.get("crec"), cc_cnt, cc_all, sp.n_crows, CP_FIELDS, None)
    pump()

    # ---- phase 2: every record in plan order, then consensus on the owner of each pair
    def records():
        _fault("records")
        pl, full, have = st["pl"], st["full"], st["have"]
        full[st["wl"]] = st["rec"]
        if gtab is not None:
            fill(full, have, gtab)
        cps = np.zeros((pl.n_cp, CP_FIELDS - 1), np.float64)
        got = np.zeros(pl.n_cp, bool)
        if len(st["cpl"]):
            cps[st["cpl"]] = st["crec"][:, 1:]
            got[st["cpl"]] = True
        for j, b in enumerate(pairs):
            if sp.split[b] and p.compute_pitch:
                c0, c1 = pl.pair_chunks[j]
                for k in range(c1 - c0):
                    if not got[c0 + k]:
                        row = ctab[sp.crow[b] + k]
                        if row[0] != 1.0:
                            raise ShardError(f"chunk-pair record of pair {b} missing from the exchange")
                        cps[c0 + k] = row[1:]
        st["cps"] = cps

    if err is None:
        _, err = _try(records)
    ibi_pre = None
    if p.compute_ibi and exchange:
        # the hop-64 pass of every split pair, its frames split over all ranks (C2-C4); every
        # rank holds every split pair (ShardPlan.needed); the owners get the results.  Every
        # rank enters it, a held error included, so the collectives stay matched.
        ibi_pre, err = _sharded_ibi(stages, ex, sp, st.get("pl"), pairs, st.get("prior"), r, pump, err)
    if err is not None:
        return [], err

    def consensus():
        _fault("consensus")
        owned = [j for j, b in enumerate(pairs) if sp.owner[b] == r]
        res = _consensus(stages, p, st["pl"], st["align"], st["active"], st["energy"], st["full"], st["prior"],
                         st["cps"], owned, ibi_pre, index=pairs)
        return [(pairs[j], o) for j, o in zip(owned, res)]

    return _try(consensus)


def _ibi_share(T: int, world: int, r: int) -> Tuple[int, int, int, int]:
    """Rank r's share of a T-frame file in the split hop-64 pass: tempogram tiles [b0, b1)
    (contiguous blocks of 2048-frame tiles) and the onset frames [t0, t1) those tiles cover."""
    b0, b1 = shard_range(-(-T // IBI_TILE), world, r)
    return b0, b1, min(T, b0 * IBI_TILE), min(T, b1 * IBI_TILE)


def _ibi_mel_rows(T: np.ndarray, t0: np.ndarray, t1: np.ndarray) -> np.ndarray:
    """Mel dB rows [r0, r1) a rank computes for its onset frames [t0, t1) of each T-frame
    file: the rows its onsets read, [t0 - pad, t1 - pad + 1), and, for the share that ends
    the file, every row up to T — rows T - pad + 1 .. T - 1 feed no onset but do feed
    power_to_db's maximum (the C2 reference), exactly as over the whole file on one GPU.
    csrc/ibi.hip ibi_range_plan_kernel computes the same bounds."""
    T, t0, t1 = (np.asarray(x, np.int64) for x in (T, t0, t1))
    r0 = np.maximum(0, t0 - IBI_PAD)
    r1 = np.where((t1 >= T) & (t1 > t0), T, np.minimum(T, t1 - IBI_PAD + 1))
    return np.stack([r0, np.maximum(r0, r1)], axis=1)


def _sharded_ibi(stages, ex: Exchange, sp: ShardPlan, pl, pairs: List[int], prior, r: int, pump,
                 err: Optional[BaseException] = None):
    """estimate_ibis_global (tempo.py:120-173) of every split pair's two files with the frames
    split over the ranks:
      rank r: mel dB of its frames' rows -> C2 all-reduce MAX of each file's dB maximum (the
      power_to_db top_db reference) -> onsets of its frames -> C4 all-gather of the onset
      segments (every rank: the full onsets) -> tempogram partial rows of its tiles -> C3
      all-gather of the tile rows, summed in tile order (the one-GPU bits) -> the owner runs
      the beat tracker on the full onset and the IBI extraction.
    Returns ({plan pair index: (ibis (nc, src), IBI counts, beat counts, tempo lags)} for the
    split pairs this rank owns, held error).  A held ``err`` rides into C2; every collective
    raises on every rank; an error after C3 is returned."""
    W = ex.world
    js = [j for j, b in enumerate(pairs) if sp.split[b]]
    nF = 2 * len(js)
    g = {}

    def prep():
        files = [f for j in js for f in (2 * j, 2 * j + 1)]
        g["f_off"], g["f_len"] = pl.f_off[files], pl.f_len[files]
        g["T"] = T = 1 + np.asarray(g["f_len"], np.int64) // IBI_HOP
        g["share"] = share = [[_ibi_share(int(t), W, q) for t in T] for q in range(W)]
        g["b0"], g["b1"], g["t0"], g["t1"] = (np.array([m[i] for m in share[r]], np.int64) for i in range(4))
        return stages.ibi_mel(g["f_off"], g["f_len"], g["t0"], g["t1"])

    mx, err = _try(prep) if err is None else (None, err)
    gmax = ex.allreduce_max(mx if err is None else np.full(nF, -np.inf), err)                       # C2
    pump()
    T, share = g["T"], g["share"]
    seg, err = _try(stages.ibi_onset, gmax)
    cnt = [sum(m[3] - m[2] for m in share[q]) for q in range(W)]
    rows = ex.gather_blocks(np.asarray(seg if err is None else np.zeros(0), np.float64)[:, None], cnt, err)  # C4

    def onsets_of(rows):
        onsets = [np.zeros(int(t), np.float32) for t in T]
        pos = 0
        for q in range(W):
            for f, m in enumerate(share[q]):
                onsets[f][m[2]:m[3]] = rows[pos:pos + m[3] - m[2], 0]
                pos += m[3] - m[2]
        g["onsets"] = onsets
        pump()
        return stages.ibi_tiles(onsets, g["b0"], g["b1"])

    N = int(int(8.0 * SR) // IBI_HOP)
    slab, err = _try(onsets_of, rows)
    cnt = [sum(m[1] - m[0] for m in share[q]) for q in range(W)]
    rows = ex.gather_blocks(slab if err is None else np.zeros((0, N)), cnt, err)                    # C3

    def tail():
        onsets = g["onsets"]
        tiles = [[None] * int(-(-t // IBI_TILE)) for t in T]
        pos = 0
        for q in range(W):
            for f, m in enumerate(share[q]):
                for b in range(m[0], m[1]):
                    tiles[f][b] = rows[pos]
                    pos += 1
        tg = stages.ibi_reduce(tiles, T)
        pump()
        out = {}
        for i, j in enumerate(js):
            if sp.owner[pairs[j]] == r:
                out[j] = stages.ibi_beats([onsets[2 * i], onsets[2 * i + 1]], tg[2 * i:2 * i + 2], [prior[j], 120.0])
        return out

    return _try(tail)


def _consensus(stages, p: Params, pl, align, active, energy, full, prior, cps, owned: List[int],
               ibi_pre: Optional[dict] = None, index: Optional[Sequence[int]] = None) -> list:
    """Bootstraps, IBI pass and host assembly of the held pairs ``owned`` (plan indices);
    ``ibi_pre`` holds the split pairs' IBI results of the sharded pass; ``index`` maps plan
    indices to the global pair indices a ``Params.melodia`` hook is called with."""
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
    bpm, nbeats = full[:, R_BPM], full[:, R_NBEATS]

    def valid_tempos(f):
        return [bpm[w] for w in range(w0[f], w1[f]) if active[w] and nbeats[w] >= MIN_BEATS and bpm[w] > 0
                and math.isfinite(bpm[w])]

    tempo_jobs, pitch_jobs, shift_jobs = [], [], []
    for b in owned:
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
        ibi_pre = ibi_pre or {}
        rest = [b for b in owned if b not in ibi_pre]
        files = [f for b in rest for f in (2 * b, 2 * b + 1)]
        sb = np.array([prior[f // 2] if f % 2 == 0 else 120.0 for f in files])
        r_ibis, r_nibi, r_nb, r_lg = stages.ibi(pl.f_off[files], pl.f_len[files], sb)
        ibis, nibi, nb, lg = [], [], [], []
        k = 0
        for b in owned:                 # the owned pairs' (nc, src) results, in owned order
            if b in ibi_pre:
                pi, pn, pb, pg = ibi_pre[b]
                ibis += list(pi)
                nibi += list(pn)
                nb += list(pb)
                lg += list(pg)
            else:
                ibis += list(r_ibis[2 * k:2 * k + 2])
                nibi += list(r_nibi[2 * k:2 * k + 2])
                nb += list(r_nb[2 * k:2 * k + 2])
                lg += list(r_lg[2 * k:2 * k + 2])
                k += 1
        files = [f for b in owned for f in (2 * b, 2 * b + 1)]
        nF = 2 * B
        ibi = dict(nibi=np.zeros(nF, np.int64), nbeats=np.zeros(nF, np.int64), lag=np.zeros(nF, np.int64),
                   out=np.full(3 * B, np.nan))
        for k, f in enumerate(files):
            ibi["nibi"][f] = nibi[k]
            ibi["nbeats"][f], ibi["lag"][f] = nb[k], lg[k]
        jobs = [(b, (ibis[2 * i + 1], ibis[2 * i])) for i, b in enumerate(owned)
                if ibis[2 * i] is not None and ibis[2 * i + 1] is not None]
        for (b, _), (pt, (lo_, hi_)) in zip(jobs, stages.bootstrap([j for _, j in jobs], 42)):
            ibi["out"][b], ibi["out"][B + b], ibi["out"][2 * B + b] = pt, lo_, hi_

    pvals = np.concatenate([shifts, nc_hz, src_hz]) if n_cp else np.zeros(3)
    tun = cps[:, 1:3].reshape(-1).astype(np.float32) if n_cp else np.zeros(0, np.float32)
    chroma = cps[:, 3:27].reshape(-1).astype(np.float32) if n_cp else np.zeros(0, np.float32)
    h = {"active_l": active.tolist(), "energy": energy, "clag_l": lags, "pvals": pvals, "pvals_l": pvals.tolist(),
         "sout_l": sout.tolist(), "bout_l": bout.tolist(), "tuning": tun, "chroma": chroma,
         "cmargin": cps[:, 27].copy() if n_cp else np.zeros(0),
         "tmargin": cps[:, 28:30].reshape(-1).astype(np.int32) if n_cp else np.zeros(0, np.int32),
         "bpm_l": bpm.tolist(), "nbeats_l": [int(v) for v in nbeats], "prior_l": prior.tolist(),
         "margin": full[:, R_MARGIN]}
    starts_l = [s.tolist() for s in pl.starts]
    w0l, w1l = [int(v) for v in w0], [int(v) for v in w1]
    def span(b):
        """(global pair index, trimmed (src, nc) spans relative to the files) for the hook."""
        if p.melodia is None:
            return None
        fs, fn = 2 * b + 1, 2 * b
        rel = lambda f: (int(pl.f_off[f] - stages.off[f]), int(pl.f_len[f]))
        return (index[b] if index is not None else b, (rel(fs), rel(fn)))

    ctx = AsmContext(h, ibi, starts_l, w0l, w1l, pl.f_len, pl.strip_len, pl.lead, pl.trail, list(pl.intro),
                     pl.win_n, pl.pair_chunks, n_cp, nj, n_pj, align)
    return [ctx.assemble(b, p, span=span(b)) for b in owned]


def run_window_sharded(pairs: Sequence[Tuple[np.ndarray, np.ndarray]], p: Optional[Params] = None,
                       group=None, device: Optional[int] = None, split_offset: float = 0.0,
                       gather: bool = True, exchange_device: Optional[torch.device] = None):
    """Upload the (nc, src) pairs this rank touches to its GPU and run ``analyze_sharded``
    (``pairs`` may hold every pair of the batch; only the touched ones are uploaded)."""
    from .engine import get_engine
    eng = get_engine(device)
    p = p or Params()
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0
    lengths = [len(a) for nc, src in pairs for a in (nc, src)]
    touched = shard_plan(lengths, p, world, split_offset).needed(rank, p.compute_ibi and world > 1)
    from .io import Pcm16
    flat = [a if isinstance(a, Pcm16) else np.asarray(a, np.float32) for b in touched for a in pairs[b]]
    sig = eng.upload_signals(flat) if flat else DeviceSignals(torch.zeros(64, device=eng.dev),
                                                             np.zeros(0, np.int64), np.zeros(0, np.int64))
    return analyze_sharded(DeviceStages(eng, sig), p, group, lengths=lengths, local_pairs=touched,
                           split_offset=split_offset, gather=gather, exchange_device=exchange_device)
