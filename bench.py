#!/usr/bin/env python3
"""Benchmark: 10 s windows/sec of the per-window hot path on MI355X.

Workload (BASELINE.json configs[2], "config 3"): per GPU a batch of 64 synthetic
3-min 22.05 kHz mono (nightcore, source) pairs (chords + clicks
every 10 752 samples + -50 dBFS noise; nc = resample_poly(src, 4, 5)), seed
1000 + global pair index.  One step = one pass of pipeline.run's analysis over
the batch with the inputs already resident in HBM: silence trim, 10 s / 5 s
windows (62 per pair), energy gate, onset + tempogram + tempo + beat tracking
per window, nc tempo prior, 20 s-chunk CQT chroma (14 per pair) + lag,
tempo/pitch bootstraps, result assembly.  The hop-64 IBI pass is not part of
the windows/sec metric and is reported beside it.

N > 1 (BASELINE config 4 at N = 8): one process per GPU (torch.distributed.run); the
batch is 64 pairs per GPU and its 10 s windows and 20 s chunk pairs are split over the
ranks in pair-major blocks (nightcore_analyzer.sharded, north_star's window split; weak
scaling).  A rank makes and uploads only the pairs its block touches; pairs cut by a
block boundary exchange their per-window and chunk-pair records (RCCL all-gathers).
With 64 equal pairs per rank the blocks fall on pair boundaries, so the headline has no
cut pair; the line also times whole pairs per rank ("pairs") and the same split with every
boundary moved half a pair ("windows_split": N - 1 cut pairs, both exchanges per step).
Barrier + synchronize around the K timed steps, max elapsed over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import numpy as np
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
WIN_BYTES = 220500 * 4         # algorithmic bytes per 10 s window
CHUNK_BYTES = 441000 * 4       # algorithmic bytes per 20 s CQT chunk
VALU_PEAK_TFS = 157.3          # MI355X f32 vector (= f32 MFMA) peak, MI355X_MICROARCH.md
# Algorithmic FLOPs (a real N-point FFT counted as 2.5 N log2 N):
#   STFT->mel frame: rFFT 2048 (56 320) + power (3 075) + Slaney mel, ~2 050 taps x 2 (4 100)
#   -> 63 495; a 10 s window has 431 frames.
# The CQT on the matrix cores (csrc/cqt.hip cqt_mfma_kernel + cqt_mfma_low_kernel): per octave
# a [862 x 1024] . [1024 x 72] GEMM with hi/lo split f16 operands (3 products), 7 octaves:
# 7 x 862 x 1024 x 72 x 2 x 3 per chunk, against the dense f16 MFMA peak over the CQT span.
CHUNK_FLOP_MFMA = 7 * 862 * 1024 * 72 * 2 * 3
MFMA_F16_PEAK_TFS = 2500.0     # MI355X dense f16/bf16 MFMA peak, MI355X_MICROARCH.md
WIN_FLOP = 431 * 63495
# window_tg (csrc/nc_tgcorr.h) per 10 s window: the six lag correlations, 345 lags x 6 x
# (T + acw = 775) f64 FMAs, plus the normalisers, 431 frames x 344 taps; its own I/O is the
# S_db rows + frame max / energy in, onset + tempogram mean + energy out.
F64_PEAK_TFS = 78.6            # MI355X f64 vector peak, MI355X_MICROARCH.md
WTG_FLOP = 2 * (345 * 6 * 775 + 431 * 344)
WTG_BYTES = 431 * (128 * 4 + 4 + 8) + 431 * 4 + 344 * 8 + 8


def _gen(args):
    seconds, seed = args
    from nightcore_analyzer import synth
    return synth.make_pair(seconds, seed)


def make_pairs(n, seconds, base_seed, workers):
    with ProcessPoolExecutor(max_workers=workers) as ex:
        return list(ex.map(_gen, [(seconds, base_seed + i) for i in range(n)]))


def make_pairs_ids(ids, seconds, base_seed, workers):
    """The synthetic pairs with global indices `ids` (seed base_seed + index)."""
    with ProcessPoolExecutor(max_workers=workers) as ex:
        return list(ex.map(_gen, [(seconds, base_seed + i) for i in ids]))


def synth_lengths(seconds):
    from nightcore_analyzer import synth
    return synth.pair_lengths(seconds)


def build_provenance():
    """What build a measurement comes from: the sha256 of the kernel sources (csrc/*, include/,
    prefix 16), of the loaded libncgpu.so, and the git commit (git, or .build_commit written by
    tools/stamp_commit.sh before a GPU call: the snapshot sent to the box has no .git)."""
    import hashlib
    import subprocess
    h = hashlib.sha256()
    src = sorted((REPO / "nightcore-to-flac-analyzer_amd" / "csrc").glob("*")) + sorted((REPO / "include").glob("*.h"))
    for f in src:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    lib = Path(os.environ.get("NCGPU_LIB") or REPO / "nightcore-to-flac-analyzer_amd" / "nightcore_analyzer" / "_lib"
               / "libncgpu.so")
    lib_sha = hashlib.sha256(lib.read_bytes()).hexdigest()[:16] if lib.exists() else None
    try:
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], cwd=REPO, capture_output=True,
                                text=True, timeout=10).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        commit = ""
    if not commit and (REPO / ".build_commit").exists():
        commit = (REPO / ".build_commit").read_text().strip()
    return {"src_sha": h.hexdigest()[:16], "lib_sha": lib_sha, "commit": commit or "unknown"}


def _pmc_traffic(kernel_tag, prov=None):
    """HBM bytes per launch of a kernel from the newest committed rocprofv3 PMC pass
    (profiles/r*_traffic.json, FETCH_SIZE x 2 + WRITE_SIZE per MI355X_MICROARCH.md), if one
    exists for this workload; counters cannot be read from inside a timed run.  `stale`: the
    file's kernel-source hash differs from this build's (or it records none)."""
    best = None
    for f in sorted((REPO / "profiles").glob("r*_traffic.json")):
        try:
            d = json.loads(f.read_text())
        except ValueError:
            continue
        k = d.get("kernels", {}).get(kernel_tag)
        if k and d.get("workload") == "config3-64pairs":
            best = {"bytes_per_launch": k["hbm_bytes_per_launch"], "source": f"profiles/{f.name}",
                    "commit": d.get("commit"), "src_sha": d.get("src_sha"),
                    "stale": prov is None or d.get("src_sha") != prov["src_sha"]}
    return best


def _cpu_worker(args):
    """One CPU worker: regenerate its pair (untimed), wait for the others, then time
    oracle/refglue.run_arrays on it with BLAS/OMP limited to one thread."""
    seconds, seed, barrier = args
    from threadpoolctl import threadpool_limits
    from nightcore_analyzer import synth
    from oracle import refglue
    nc, src = synth.make_pair(seconds, seed)
    nw = len(refglue.slice_windows(nc)) + len(refglue.slice_windows(src))
    ncp = len(refglue.chunk_plan(len(src), len(nc)))
    barrier.wait()
    with threadpool_limits(limits=1):
        t0 = time.time()
        res = refglue.run_arrays(nc, src, compute_ibi=False)
        t1 = time.time()
    return nw, t0, t1, res["tempo_ratio"], res["pitch_ratio"], ncp


def host_cores():
    """Host cores this process may run on (one CPU worker per core).  On the
    GPU box the affinity mask can show the whole machine; the per-GPU CPU share is what
    OMP_NUM_THREADS is set to there, so the count is capped at it when it is set."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_baseline(seconds, base_seed, workers):
    """The oracle (oracle/refglue.py, the CPU port of the reference glue on the numpy
    restatement of librosa) on the first `workers` pairs of the batch, one pair per
    process, one thread each (process pool, BLAS threads = 1);
    windows/s = all windows / (last finish - first start)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        barrier = m.Barrier(workers)
        with ctx.Pool(workers) as pool:
            rows = pool.map(_cpu_worker, [(seconds, base_seed + i, barrier) for i in range(workers)])
    nw = sum(r[0] for r in rows)
    wall = max(r[2] for r in rows) - min(r[1] for r in rows)
    return {"value": nw / wall, "unit": "windows/s", "cores": workers, "kind": "port",
            "sample": f"pairs 0..{workers - 1} of the batch ({nw} windows + {sum(r[5] for r in rows)} CQT chunk pairs + "
                      f"bootstraps), oracle/refglue.run_arrays(compute_ibi=False), {workers} processes x 1 thread, "
                      f"{wall:.1f} s wall, {sum(r[2] - r[1] for r in rows):.1f} s CPU",
            "tempo_ratio": rows[0][3], "pitch_ratio": rows[0][4]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=64, help="pairs per GPU (config 3: 64)")
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ibi", action="store_true")
    ap.add_argument("--no-config5", action="store_true", help="skip the 60-min pair (BASELINE configs[4]) timing")
    ap.add_argument("--no-spectral", action="store_true", help="skip the spectral.analyze (SURVEY.md §8f) timing")
    ap.add_argument("--no-resample", action="store_true", help="skip the load-time resampler (SURVEY.md §8f) timing")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="CPU baseline processes, one pair each (0: the host cores this process may run on)")
    ap.add_argument("--no-upload", action="store_true", help="skip the upload-included throughput")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="time K separate analyze calls instead of one pipelined analyze_batches call")
    ap.add_argument("--shard", choices=("pairs", "windows"), default="windows",
                    help="N > 1: the batch's windows and chunk pairs split over the ranks (default; "
                         "nightcore_analyzer.sharded, BASELINE config 4), or whole pairs per rank; the other mode "
                         "and the split-boundary variant are timed beside the headline")
    ap.add_argument("--workers", type=int, default=min(16, os.cpu_count() or 1))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the synthetic pairs are made (forked workers) before this process touches the GPU.
    # N > 1, window mode (BASELINE config 4, the default there): the batch is all ranks'
    # pairs (64 per GPU, seeds 1000 + global pair index) and its items (windows, chunk pairs)
    # are split over the ranks by sharded.shard_plan; a rank makes and uploads only the pairs
    # its blocks touch (its own 64, plus the neighbour pairs the split-boundary variant cuts).
    # Pair mode: each rank its own 64 pairs (weak scaling, no exchange).
    win_mode = world > 1 and args.shard != "pairs"
    P = args.pairs
    own_ids = list(range(rank * P, (rank + 1) * P))
    # (both modes: the side variants timed beside the headline include the split-boundary one)
    ids = sorted(set(own_ids) | ({rank * P - 1, (rank + 1) * P} & set(range(world * P)) if world > 1 else set()))
    pairs = dict(zip(ids, make_pairs_ids(ids, args.seconds, 1000, max(1, args.workers // max(1, world)))))
    # NC_BENCH_REHEARSE=1: rehearse the N > 1 path on fewer GPUs than ranks (ranks share devices
    # round-robin; gloo instead of RCCL, which refuses two ranks on one device).  Never used for
    # a reported number: the line then says so in "data".
    rehearse = world > 1 and os.environ.get("NC_BENCH_REHEARSE") == "1"
    dev = local % max(1, torch.cuda.device_count()) if rehearse else local
    if world > 1:
        torch.cuda.set_device(dev)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    from nightcore_analyzer import engine as E

    eng = E.get_engine(dev)
    flat = []
    for b in ids:
        flat += list(pairs[b])
    signals = eng.upload_signals(flat)           # resident in HBM before timing
    sel = np.array([f for j, b in enumerate(ids) if b in set(own_ids) for f in (2 * j, 2 * j + 1)], np.int64)
    own = E.DeviceSignals(signals.buf, signals.off[sel], signals.length[sel])
    torch.cuda.synchronize()
    params = E.Params(compute_ibi=False)

    def step():
        return eng.analyze(signals=own, params=params)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device="cpu" if rehearse else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([float(v)], dtype=torch.float64, device="cpu" if rehearse else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    lengths = [n for _ in range(world * P) for n in synth_lengths(args.seconds)]

    def run_windows(k, split_offset=0.0, gather=True):
        """k steps of the window-sharded analysis (interior groups pipelined across steps).
        gather=True is analyze_sharded's default: every step's outcomes of all pairs end on
        every rank (one byte all-gather of record tables per call after the last record
        exchange: result rows readable at once, the other ranks' outcomes rebuilt from their
        records on first access: sharded.GatheredOutcomes).  Returns
        one sequence of outcomes per step (gather) or of this rank's (pair, outcome)."""
        from nightcore_analyzer.sharded import DeviceStages, analyze_sharded
        res = analyze_sharded(DeviceStages(eng, signals), params, lengths=lengths, local_pairs=ids,
                              split_offset=split_offset, gather=gather, steps=k)
        res = [res] if k == 1 else res
        return res

    outs = step()
    bad = [i for i, o in enumerate(outs) if o.error is not None]
    if bad:
        raise RuntimeError(f"pairs {bad} failed: {outs[bad[0]].error}")
    win_per_step = sum(o.detail["energy_src"].size + o.detail["energy_nc"].size for o in outs)
    chunks_per_step = 2 * sum(len(o.detail["chunk_lags"]) for o in outs)
    tr = outs[0].result.tempo_ratio
    pr = outs[0].result.pitch_ratio
    for _ in range(max(0, args.warmup - 1)):
        step()
    if not win_mode and not args.no_pipeline and args.warmup > 0:
        # the pipelined call itself is warmed at the timed size: its first-use paths (trims queued
        # ahead on the trim stream, their workspaces and pinned read-back buffers) and the host
        # memory its K batches of results take.  A first K-batch call in the process ran
        # 10.2-10.3 ms per step where the next ones ran 9.5-9.7 (profiles/r4_bench_timing_variants.txt)
        eng.analyze_batches([own] * max(2, args.steps), params)
    if win_mode:   # warmed at the timed size, as the pipelined call above
        for off in (0.0, 0.5):
            run_windows(max(1, args.warmup, args.steps), off)

    # timed region: K steps with every launch of the roofline kernels (stft_mel, cqt_low,
    # cqt_high, window_tg) bracketed by a HIP event pair on the stream it runs on (nc_profile
    # mode 4), so the per-kernel durations below come from exactly the launches the headline
    # number times.  The roofline divides by the event durations (dispatch to completion on the
    # kernel's stream, what rocprofv3 --kernel-trace reports, waiting for CUs the other stream
    # holds included).  No other kernel is timed in the region: events around every launch cost
    # the step ~5 %, the kernels' own execution spans ~3 % (profiles/r4_timer_modes_probe.txt);
    # every kernel's time alone is in roofline.isolated
    eng.kernel_profile(4)
    barrier()
    torch.cuda.synchronize()
    # a marker launch (torch.cumsum: no engine kernel is a scan) on each side of the timed region,
    # so a rocprofv3 --kernel-trace of this command can be cut to exactly the timed launches
    # (tools/rocprof_timed.py: their average durations against this line's)
    marker = torch.arange(8, dtype=torch.float64, device=eng.dev)
    torch.cumsum(marker, 0)
    torch.cuda.synchronize()
    # pair mode: the K steps are K complete analyses of the batch, issued as one pipelined
    # Engine.analyze_batches call (batch k + 1's trims and first groups are queued while batch
    # k's last groups run: no device idle at a batch's start-up); --no-pipeline times K
    # separate analyze calls (reported beside it as single_call_ms_per_step).  Window mode:
    # one analyze_sharded call of K steps (its interior groups pipelined the same way)
    pipelined = not args.no_pipeline
    gather_rebuild = None
    t0 = time.perf_counter()
    if win_mode:
        res = run_windows(args.steps)
        # the caller's read of every step's results on every rank, inside the timed region: each
        # pair's result row (ratios, CIs, counts) straight from the gathered records
        # (sharded.GatheredOutcomes.table; the whole outcome is rebuilt only on access, below)
        tabs = [r.table() for r in res]
    elif pipelined:
        res = eng.analyze_batches([own] * args.steps, params)
    else:
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    torch.cumsum(marker, 0)
    torch.cuda.synchronize()
    if win_mode:
        if any(len(r) != world * P for r in res):
            raise RuntimeError("a window-sharded step returned an incomplete result")
        if any(not (t[:, 0] == 1.0).all() for t in tabs):
            raise RuntimeError("a window-sharded step failed")
        if rank == 0 and (tabs[0][0, 1] != tr or tabs[0][0, 4] != pr):
            raise RuntimeError("the window-sharded result of pair 0 differs from the single-GPU engine's")
        from nightcore_analyzer.sharded import result_row
        # every outcome of the first step rebuilt from the records (report text, logs, detail:
        # assemble_pair on the receiving rank), after the timed region, per received pair
        tu = time.perf_counter()
        mine = list(res[0])                     # gather=True: every pair's outcome on every rank
        n_recv = sum(1 for b in range(len(mine)) if int(res[0]._owner[b]) != rank)
        gather_rebuild = {"ms_per_received_pair": max_over_ranks((time.perf_counter() - tu) * 1e3 / max(1, n_recv)),
                          "received_pairs_per_rank_step": n_recv,
                          "how": "outside the timed region: one step's outcomes of the other ranks' pairs rebuilt "
                                 "from the gathered records by assemble_pair (engine.AsmContext), as a caller pays "
                                 "on first access to a pair's report or logs; the timed steps read every pair's "
                                 "result row (GatheredOutcomes.table)"}
        if any(o.error is not None for o in mine):
            raise RuntimeError("a window-sharded step failed")
        win_total = sum(o.detail["energy_src"].size + o.detail["energy_nc"].size for o in mine)
        if any(not np.array_equal(tabs[0][b], np.array(result_row(o), np.float64), equal_nan=True)
               for b, o in enumerate(mine)):
            raise RuntimeError("a gathered result row differs from its rebuilt outcome")
        del res, mine, tabs                     # not kept (see below)
    elif pipelined:
        if len(res) != args.steps or any(len(r) != len(outs) for r in res):
            raise RuntimeError("analyze_batches returned an incomplete result")
        if any(r[0].result.tempo_ratio != tr or r[0].result.pitch_ratio != pr for r in res):
            raise RuntimeError("a pipelined batch differs from the single-call result")
        # the checked outcomes (K x 64 pairs) are not kept: holding them slowed the side legs
        # measured after (spectral.analyze 5.0 -> 9.9 ms per call; profiles/r4_bench_timing_variants.txt)
        del res
    evt = eng.kernel_times()
    spans = eng.kernel_spans()
    eng.kernel_profile(False)

    # device idle, untraced: extra steps of the same call with every kernel recording its own
    # execution span (profile mode 2, ~3 % slower than the timed steps), then 1 - the union of the
    # spans over their extent (nc_profile_read_busy).  The extent starts at the call's first
    # kernel, so the call's start-up (first trim read-back, first group plan) is in it
    n_idle = max(2, min(args.steps, 10))
    eng.kernel_profile(2)
    barrier()
    torch.cuda.synchronize()
    if win_mode:
        run_windows(n_idle)
    elif pipelined:
        eng.analyze_batches([own] * n_idle, params)
    else:
        for _ in range(n_idle):
            step()
    busy_ms, extent_ms, idle_launches = eng.device_busy()
    eng.kernel_profile(False)
    idle_frac = max_over_ranks(1.0 - busy_ms / extent_ms) if extent_ms > 0 else None
    device_idle = {"frac": idle_frac, "busy_ms": busy_ms, "extent_ms": extent_ms, "steps": n_idle,
                   "launches": idle_launches,
                   "how": "untimed steps of the headline call, the execution spans of the engine's timed kernels "
                          "recorded (stft_mel, window_tg, tuning_peaks, decimate, tuning_select, cqt_low, cqt_high, "
                          "tempo_beat, trim_blocks; the small unspanned kernels count as idle, so this is an upper "
                          "bound): 1 - union of spans / first start..last end (nc_profile_read_busy); max over ranks"}
    el = max_over_ranks(el)
    step_ms = el / args.steps * 1e3
    value = (win_total if win_mode else world * win_per_step) * args.steps / el

    # N > 1: the other modes beside the headline, K steps each, same clock
    modes = None
    if world > 1:
        modes = {}
        # windows_nogather: the headline's steps without the final outcome all-gather (each rank
        # keeps the outcomes of the pairs it owns)
        variants = [("windows_nogather", 0.0, False), ("pairs", None, False), ("windows_split", 0.5, True)] \
            if win_mode else [("windows", 0.0, True), ("windows_split", 0.5, True)]
        # NC_BENCH_MODES_EXTRA=1 (rehearsal diagnostics): the headline's steps again after the
        # modes, untraced with and without the gather, then under the headline's roofline events
        # (profile mode 4)
        extra = win_mode and os.environ.get("NC_BENCH_MODES_EXTRA", "0") == "1"
        if extra:
            variants += [("windows_gather_again", 0.0, True), ("windows_nogather_again", 0.0, False),
                         ("windows_gather_again_prof4", 0.0, True)]
        for name, off, gat in variants:
            if name.endswith("_prof4"):
                eng.kernel_profile(4)
            barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            if off is None:
                eng.analyze_batches([own] * args.steps, params)
            else:
                r_ = run_windows(args.steps, off, gat)
                if gat:
                    tabs_ = [r.table() for r in r_]     # the caller's read, as in the headline
            torch.cuda.synchronize()
            barrier()
            e1 = max_over_ranks(time.perf_counter() - t1)
            # windows counted after the clock (a gathered outcome's detail is rebuilt on access)
            if off is None:
                n_win = world * win_per_step
            else:
                n_win = (sum(o.detail["energy_src"].size + o.detail["energy_nc"].size for o in r_[0]) if gat else
                         sum_over_ranks(sum(o.detail["energy_src"].size + o.detail["energy_nc"].size
                                            for _, o in r_[0])))
            modes[name] = {"value": n_win * args.steps / e1, "ms_per_step": e1 / args.steps * 1e3}
            if name.endswith("_prof4"):
                eng.kernel_times()
                eng.kernel_profile(False)
        from nightcore_analyzer.sharded import shard_plan
        sp = shard_plan(lengths, params, world, 0.5)
        modes["windows_split"].update(split_pairs=int(sp.split.sum()),
                                      exchanged_rows_per_step=2 * sp.n_wrows + sp.n_crows,
                                      how="every inner block boundary moved half a pair (split_offset 0.5): the "
                                          "cut pairs' window and chunk-pair records all-gathered (C1a, C1b)")
    # {kernel: (average launch ms, launches per step)} from the spans of the timed region
    kper = {k: (ms / n, n / args.steps) for k, (ms, n) in evt.items()}
    kspan = {k: ms / n for k, (ms, n) in spans.items()}
    # per-step kernel time: the event durations where recorded, the execution spans otherwise
    kstep = {k: ms / args.steps for k, (ms, n) in spans.items()}
    kstep.update({k: v[0] * v[1] for k, v in kper.items()})

    # the same steps as separate analyze calls (each with its own start-up), for comparison
    single_ms = None
    if pipelined:
        torch.cuda.synchronize()
        ts = time.perf_counter()
        nsc = max(1, min(args.steps, 5))
        for _ in range(nsc):
            step()
        torch.cuda.synchronize()
        single_ms = (time.perf_counter() - ts) / nsc * 1e3

    # entry-point HIP-event timers (separate, untimed steps)
    eng.start_timers()
    ksteps = max(1, min(args.steps, 3))
    for _ in range(ksteps):
        step()
    timers = eng.stop_timers()
    per = {k: (ms / n, n // ksteps) for k, (ms, n) in timers.items()}

    # algorithmic bytes / flops per launch = SURVEY.md §8d per-unit figure x units per launch
    units = {"stft_mel": (win_per_step, WIN_BYTES, WIN_FLOP),
             "cqt_chroma": (chunks_per_step, CHUNK_BYTES, CHUNK_FLOP_MFMA)}
    # compute roof per kernel: f32 VALU for the FFT kernels, f64 VALU for the tempogram
    compute_roof = {"window_tg": ("valu_f64", F64_PEAK_TFS), "cqt_chroma": ("mfma_f16", MFMA_F16_PEAK_TFS)}

    prov = build_provenance()

    def roof(tag, times, table=None, span=None):
        table = table or units
        if tag not in times or tag not in table:
            return None
        avg_ms, launches = times[tag]
        alg = table[tag][0] / launches * table[tag][1]
        flop = table[tag][0] / launches * table[tag][2]
        a = alg / (avg_ms * 1e-3) / 1e9
        c = flop / (avg_ms * 1e-3) / 1e12
        cb, cp = compute_roof.get(tag, ("valu_f32", VALU_PEAK_TFS))
        tr = _pmc_traffic(tag, prov)
        out = {"bound": "hbm", "kernel": tag, "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": a / HBM_PEAK_GBS, "traffic": tr["bytes_per_launch"] if tr else None,
               "traffic_source": tr["source"] if tr else None,
               "traffic_commit": tr["commit"] if tr else None,
               "traffic_stale": tr["stale"] if tr else None,
               "alg_bytes_per_launch": alg, "avg_launch_ms": avg_ms,
               "launches_per_step": launches, "timing": "HIP events around each launch on its stream",
               "exec_span_ms": span.get(tag) if span else None,
               # the roof that actually binds: VALU / f64 VALU / matrix cores
               "compute": {"bound": cb, "achieved": c, "peak": cp, "unit": "TFLOP/s",
                           "frac": c / cp, "alg_flop_per_launch": flop}}
        if tag == "cqt_chroma":
            # the MFMA figures count the three split products; the useful contraction is one of
            # them (7 x 862 x 1024 x 72 x 2 flop per chunk)
            out["cqt_dtype"] = "f16x3 split operands (hi/lo, ~22-bit), f32 accumulate"
            out["compute"]["useful_frac"] = c / 3.0 / cp
            out["compute"]["useful_achieved"] = c / 3.0
            out["parts_ms"] = {k: times[k][0] for k in ("cqt_low", "cqt_high") if k in times}
        return out

    # the dominant kernel = the single kernel with the largest total time per step, as rocprofv3
    # --stats ranks them (stft_mel against cqt_low and cqt_high, the two kernels of a CQT chunk,
    # each on its own; until round 4 their sum competed, which in a round-5 run made the chunk's
    # pair "dominant" at 4.24 ms per step beside stft_mel's 3.87 while stft_mel_kernel stayed the
    # top row of the rocprof table); the §8d unit of that kernel is priced, and the other unit
    # (stft_mel / cqt_chroma, north_star's named target) is always reported beside it
    def total(k):
        return kper.get(k, (0, 0))[0] * kper.get(k, (0, 0))[1]
    dom = "stft_mel" if total("stft_mel") >= max(total("cqt_low"), total("cqt_high")) else "cqt_chroma"
    roofline = roof(dom, kper, span=kspan)
    for other in units:
        if other != dom and other in kper:
            roofline[other] = roof(other, kper, span=kspan)
    # the per-window tempogram kernel against its f64 roof (its bytes are the S_db scratch)
    wtg_units = {"window_tg": (win_per_step, WTG_BYTES, WTG_FLOP)}
    if "window_tg" in kper:
        roofline["window_tg"] = roof("window_tg", kper, wtg_units, span=kspan)
    # the same kernels launched alone (streams serialized for one more untimed step): their own
    # speed, where the timed launches share the chip with the other streams' chains
    eng.set_serial(True)
    eng.kernel_profile(1)
    step()
    iso = eng.kernel_times()
    eng.kernel_spans()
    eng.kernel_profile(False)
    eng.set_serial(False)
    iso_t = {k: (ms / n, n) for k, (ms, n) in iso.items()}
    roofline["isolated"] = {"kernels_ms_per_step": {k: round(v[0], 4) for k, v in iso.items()},
                            **{k: roof(k, iso_t) for k in units if k in iso_t},
                            **({"window_tg": roof("window_tg", iso_t, wtg_units)} if "window_tg" in iso_t else {})}

    # upload included: the same K steps with every step's 64 pairs copied host -> HBM from
    # pinned memory on a copy stream, double-buffered (step j + 1 uploads while step j runs)
    upl = None
    if not args.no_upload and world == 1:
        host = signals.buf.cpu().pin_memory()
        bufs = [signals.buf, torch.empty_like(signals.buf)]
        cs = torch.cuda.Stream(eng.dev)
        evs = [torch.cuda.Event(), torch.cuda.Event()]

        def upload(j):
            with torch.cuda.stream(cs):
                bufs[j % 2].copy_(host, non_blocking=True)
                evs[j % 2].record(cs)
        n_up = max(2, min(args.steps, 10))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        upload(0)
        for j in range(n_up):
            if j + 1 < n_up:
                upload(j + 1)
            torch.cuda.current_stream(eng.dev).wait_event(evs[j % 2])
            eng.analyze(signals=E.DeviceSignals(bufs[j % 2], own.off, own.length), params=params)
        torch.cuda.synchronize()
        t_up = time.perf_counter() - t1
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(cs):
            e0.record(cs)
            bufs[1].copy_(host, non_blocking=True)
            e1.record(cs)
        torch.cuda.synchronize()
        h2d_ms = e0.elapsed_time(e1)
        upl = {"value": world * win_per_step * n_up / t_up, "unit": "windows/s", "steps": n_up,
               "ms_per_step": t_up / n_up * 1e3, "bytes_per_step": int(host.numel() * 4),
               "h2d_ms_per_step_alone": h2d_ms, "h2d_gb_per_s": host.numel() * 4 / (h2d_ms * 1e-3) / 1e9,
               "how": "pinned host staging, H2D on its own stream, double-buffered against the analysis"}
        del host

        # the same with 16-bit PCM sources (a mono 16-bit WAV as io.load_audio(keep_pcm16=True)
        # keeps it): the batch quantized to int16, its 2-byte samples copied host -> HBM and
        # widened on the copy stream (nc_pcm16_to_f32, k / 32768), half the PCIe bytes
        q16 = torch.clamp(torch.round(signals.buf * 32768.0), -32768, 32767).to(torch.int16)
        host16 = q16.cpu().pin_memory()
        raw = [q16, torch.empty_like(q16)]
        bufs = [torch.empty_like(signals.buf), torch.empty_like(signals.buf)]   # the resident batch kept

        def upload16(j):
            with torch.cuda.stream(cs):
                raw[j % 2].copy_(host16, non_blocking=True)
                eng.call("nc_pcm16_to_f32", raw[j % 2].data_ptr(), raw[j % 2].numel(), bufs[j % 2].data_ptr(),
                         cs.cuda_stream)
                evs[j % 2].record(cs)
        upload16(0)
        torch.cuda.synchronize()
        eng.analyze(signals=E.DeviceSignals(bufs[0], own.off, own.length), params=params)   # warm
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        upload16(0)
        for j in range(n_up):
            if j + 1 < n_up:
                upload16(j + 1)
            torch.cuda.current_stream(eng.dev).wait_event(evs[j % 2])
            eng.analyze(signals=E.DeviceSignals(bufs[j % 2], own.off, own.length), params=params)
        torch.cuda.synchronize()
        t16 = time.perf_counter() - t1
        upl["pcm16"] = {"value": world * win_per_step * n_up / t16, "ms_per_step": t16 / n_up * 1e3,
                        "bytes_per_step": int(host16.numel() * 2),
                        "vs_f32_upload": (world * win_per_step * n_up / t16) / upl["value"],
                        "how": "the batch quantized to 16-bit PCM (a 16-bit WAV source), int16 staged in pinned "
                               "memory, H2D + nc_pcm16_to_f32 widening on the copy stream, double-buffered"}
        del host16, raw, q16, bufs

    ibi = None
    if not args.no_ibi and rank == 0:
        sub = E.DeviceSignals(own.buf, own.off[:4], own.length[:4])
        eng.analyze(signals=sub, params=E.Params(compute_ibi=True))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        o2 = eng.analyze(signals=sub, params=E.Params(compute_ibi=True))
        torch.cuda.synchronize()
        t_ibi = time.perf_counter() - t1
        t1 = time.perf_counter()
        eng.analyze(signals=sub, params=E.Params(compute_ibi=False))
        torch.cuda.synchronize()
        t_no = time.perf_counter() - t1
        frames = int(sum(1 + int(n) // 64 for n in sub.length))
        ibi = {"pairs": 2, "seconds_per_pair": (t_ibi - t_no) / 2, "hop64_frames_per_s": frames / max(1e-9, t_ibi - t_no),
               "ibi_ratio_pair0": o2[0].result.ibi_ratio}

    # BASELINE configs[1]: one 3-min pair, the whole run() with its defaults (hop-64 IBI pass
    # included), host arrays in: upload + analysis + result assembly, latency per call
    cfg2 = None
    if not args.no_config5 and rank == 0 and world == 1:
        nc2, src2 = pairs[own_ids[0]]
        for _ in range(2):
            eng.analyze(signals=eng.upload_signals([nc2, src2]), params=E.Params())
        torch.cuda.synchronize()
        reps = 5
        t1 = time.perf_counter()
        for _ in range(reps):
            o2c, = eng.analyze(signals=eng.upload_signals([nc2, src2]), params=E.Params())
        torch.cuda.synchronize()
        t2 = (time.perf_counter() - t1) / reps
        nw2 = int(o2c.detail["energy_src"].size + o2c.detail["energy_nc"].size)
        cfg2 = {"workload": "config 2: one 3-min pair (host arrays), run() defaults incl. the hop-64 IBI pass; "
                            "upload + analysis + result assembly per call, 5 calls",
                "seconds_per_pair": t2, "windows": nw2, "windows_per_s": nw2 / t2,
                "tempo_ratio": o2c.result.tempo_ratio, "pitch_ratio": o2c.result.pitch_ratio,
                "ibi_ratio": o2c.result.ibi_ratio}

    # BASELINE configs[4]: one 60-min pair, the whole run() incl. the hop-64 IBI pass, plus the
    # waveform xcorr verification search (xcorr.estimate_speed_xcorr) over the same signals
    cfg5 = None
    if not args.no_config5 and rank == 0 and world == 1:
        from nightcore_analyzer import xcorr as X
        from nightcore_analyzer import synth
        nc5, src5 = synth.make_pair(3600.0, 5000)          # in-process: no fork after GPU init
        sig5 = eng.upload_signals([nc5, src5])
        eng.analyze(signals=sig5, params=E.Params(compute_ibi=True))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        o5, = eng.analyze(signals=sig5, params=E.Params(compute_ibi=True))
        torch.cuda.synchronize()
        t_run = time.perf_counter() - t1
        t1 = time.perf_counter()
        xr = X.estimate_speed_xcorr_arrays(src5, nc5)
        t_x = time.perf_counter() - t1
        cfg5 = {"workload": "config 5: one 60-min pair (src 3600 s, nc = resample_poly(src, 4, 5)), run() with "
                            "the hop-64 IBI pass; xcorr search src vs nc (host upload included)",
                "seconds_run": t_run, "seconds_xcorr": t_x,
                "hop64_frames": int((1 + len(nc5) // 64) + (1 + len(src5) // 64)),
                "windows": int(o5.detail["energy_src"].size + o5.detail["energy_nc"].size),
                "tempo_ratio": o5.result.tempo_ratio, "ibi_ratio": o5.result.ibi_ratio, "xcorr_ratio": xr[0]}

    # spectral.analyze statistics of every resident file of the batch in one
    # call (spectral.py:52-94); per-kernel HIP events on the launch stream, the oracle beside it
    spec = None
    if not args.no_spectral and rank == 0:
        srs = [22050] * own.n_files
        ev, h, keep = eng.spectral_frames(own.buf, own.off, own.length, srs)
        ev.synchronize()
        reps = 3
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            ev, h, keep = eng.spectral_frames(own.buf, own.off, own.length, srs)
            ev.synchronize()
            res = eng.spectral_finish(h)
        t_spec = (time.perf_counter() - t1) / reps
        eng.kernel_profile(2)
        for _ in range(reps):
            eng.spectral_frames(own.buf, own.off, own.length, srs)[0].synchronize()
        sk = {k: (ms / n, n / reps) for k, (ms, n) in eng.kernel_spans().items()}
        eng.kernel_profile(False)
        frames = int(h["T"].sum())
        fr_ms = sk["spectral_frames"][0]
        bins_ms = sk["spectral_bins"][0]
        spec = {"workload": f"spectral.analyze of the {own.n_files} resident 3-min files (22.05 kHz), one call",
                "files": own.n_files, "frames": frames, "ms_per_call": t_spec * 1e3,
                "frames_per_s": frames / t_spec, "files_per_s": own.n_files / t_spec,
                "kernels_ms_per_call": {k: round(v[0] * v[1], 4) for k, v in sk.items()},
                # spectral_frames: each input sample read once (512 x 4 B per frame hop);
                # spectral_bins: the dB rows streamed once (1025 x 4 B per frame)
                "roofline_frames": {"bound": "hbm", "achieved": frames * 2048 / (fr_ms * 1e-3) / 1e9,
                                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": frames * 2048 / (fr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "roofline_bins": {"bound": "hbm", "achieved": frames * 4100 / (bins_ms * 1e-3) / 1e9,
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": frames * 4100 / (bins_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "check": {"centroid_file0": res[0]["centroid"],
                          "effective_bandwidth_hz_file0": res[0]["effective_bandwidth_hz"]}}
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, str(REPO))
            from oracle import refglue
            y0 = pairs[own_ids[0]][1]
            t1 = time.perf_counter()
            refglue.spectral_analyze(y0, 22050)
            t_cpu = time.perf_counter() - t1
            spec["cpu_baseline"] = {"value": (1 + len(y0) // 512) / t_cpu, "unit": "frames/s", "cores": 1,
                                    "kind": "port", "sample": "oracle/refglue.spectral_analyze of file 1 "
                                                              "(one 3-min src), numpy, 1 process"}

    # the load-time resampler (io.py:54) on 44.1 kHz copies of the batch's
    # src files, resident in HBM (nc_resample_poly, bit-identical to scipy.signal.resample_poly)
    rsmp = None
    if not args.no_resample and rank == 0:
        import scipy.signal
        from nightcore_analyzer.ops import poly_plan
        n_files = min(16, len(own_ids))
        x44 = [scipy.signal.resample_poly(pairs[own_ids[i]][1], 2, 1).astype(np.float32) for i in range(n_files)]
        sig44 = eng.upload_signals(x44)
        up_, down_, hh, pre = poly_plan(1, 2, int(sig44.length.max()))
        n_out = np.array([-(-int(n) * up_ // down_) for n in sig44.length], np.int64)
        o_off = np.concatenate([[0], np.cumsum(n_out)[:-1]]).astype(np.int64)
        dev = eng.dev
        tens = {k: torch.from_numpy(np.asarray(v)).to(dev) for k, v in
                (("in_off", sig44.off), ("in_len", sig44.length), ("out_off", o_off), ("out_len", n_out), ("h", hh))}
        yout = torch.empty(int(n_out.sum()), dtype=torch.float32, device=dev)

        def _rs():
            eng.call("nc_resample_poly", sig44.buf.data_ptr(), tens["in_off"].data_ptr(), tens["in_len"].data_ptr(),
                     n_files, yout.data_ptr(), tens["out_off"].data_ptr(), tens["out_len"].data_ptr(),
                     int(n_out.max()), tens["h"].data_ptr(), len(hh), up_, down_, pre, eng.stream())
        _rs()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            _rs()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        n_in = int(sig44.length.sum())
        alg = n_in * 4 + int(n_out.sum()) * 4          # every input sample read once, every output written once
        rsmp = {"workload": f"{n_files} x 3-min 44.1 kHz files -> 22.05 kHz (resample_poly 1/2, 42-tap f64 FIR)",
                "ms_per_call": ms, "input_samples_per_s": n_in / (ms * 1e-3),
                "roofline": {"bound": "hbm", "achieved": alg / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}}
        if world == 1 and not args.no_cpu_baseline:
            t1 = time.perf_counter()
            scipy.signal.resample_poly(x44[0].astype(np.float64), 1, 2)
            rsmp["cpu_baseline"] = {"value": len(x44[0]) / (time.perf_counter() - t1), "unit": "input samples/s",
                                    "cores": 1, "kind": "port",
                                    "sample": "scipy.signal.resample_poly of one 3-min 44.1 kHz file, 1 process"}

    if rank == 0:
        line = {
            "metric": "10 s windows/sec (CQT+onset, 22.05 kHz mono) at 1/2/4/8 GPUs; % HBM roofline",
            "value": value,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "arithmetic": {"stft_mel / tuning FFTs": "f32 (VALU)", "tempogram, decisions, bootstrap": "f64",
                           "cqt": "f16x3 split operands (hi/lo, ~22-bit) on the matrix cores, f32 accumulate"},
            "data": "synthetic (SURVEY.md §8d chords+clicks+noise, nc = resample_poly(src, 4, 5)), resident in HBM"
                    + (f"; REHEARSAL: {world} ranks on {torch.cuda.device_count()} GPU(s), gloo" if rehearse else ""),
            "config": {"workload": ("config 3: per GPU a batch of 64 x 3-min 22.05 kHz mono pairs" if world == 1 else
                                    f"config 4 shape: a batch of {world} x 64 x 3-min 22.05 kHz mono pairs, its windows "
                                    "and chunk pairs split over the ranks (sharded.shard_plan), every step's outcomes "
                                    "all-gathered to every rank as record tables and every pair's result row read on "
                                    "every rank (analyze_sharded's default gather=True; without it: "
                                    "modes.windows_nogather)" if win_mode else
                                    f"{world} x 64 x 3-min pairs, whole pairs per rank")
                                   + "; step = pipeline.run analysis of the batch without the hop-64 IBI pass"
                                   + ("; the K steps issued as one pipelined call (batch k+1's trim and first "
                                      "groups queued while batch k's last groups run)" if pipelined else ""),
                       "single_call_ms_per_step": single_ms,
                       "pairs_per_gpu": args.pairs, "windows_per_gpu_step": win_per_step,
                       "cqt_chunks_per_gpu_step": chunks_per_step, "parallelism": f"dp{world} (" + ("windows sharded, split-pair record all-gathers)" if win_mode else
                                                    "pairs sharded)")},
            # avg_launch_ms: HIP events around each launch of the timed steps on its stream
            # (rocprofv3's kernel duration, sharing the chip with the concurrent chain;
            # tools/rocprof_timed.py checks them against a trace of this command); exec_span_ms:
            # the kernel's own first-start .. last-end span; isolated: the same kernels with the
            # other streams idle
            "roofline": roofline,
            "device_idle_frac": idle_frac,
            "device_idle": device_idle,
            "kernels_ms_per_step": {**{k: round(v[0], 4) for k, v in iso.items()},
                                    **{k: round(v, 4) for k, v in kstep.items()}},
            "kernels_ms_per_step_timing": {
                "timed_region": sorted(kstep),
                "isolated_step": sorted(set(iso) - set(kstep)),
                "how": "the roofline kernels: HIP events around their launches in the timed steps (sharing the "
                       "chip with the other streams); every other kernel: HIP events in one more step with the "
                       "streams serialized (roofline.isolated)"},
            "entry_points_ms_per_step": {k: round(v[0] * v[1], 4) for k, v in per.items()},
            "check": {"tempo_ratio_pair0": tr, "pitch_ratio_pair0": pr},
            "build": prov,
        }
        if modes is not None:
            line["modes"] = modes
        if win_mode:
            # the timed steps end with every rank holding every pair's result rows (read in the
            # region) and the records its whole outcome is rebuilt from on access (cost here)
            line["gather_rebuild"] = gather_rebuild
        if upl is not None:
            line["upload_included"] = upl
        if ibi is not None:
            line["ibi_pass"] = ibi
        if cfg2 is not None:
            line["config2"] = cfg2
        if cfg5 is not None:
            line["config5"] = cfg5
        if spec is not None:
            line["spectral"] = spec
        if rsmp is not None:
            line["resample"] = rsmp
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.seconds, 1000, args.cpu_workers or host_cores())
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
