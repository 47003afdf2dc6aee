#!/usr/bin/env python3
"""One rank's share of the N > 1 window-sharded step, measured on the box's one GPU: a one-rank
"nccl" (RCCL) group with sharded.Exchange.collect_at_one, so the step's outcome gather (record
tables + byte all-gather + the caller's read of every result row) runs as on every rank of an
8-GPU job, against the same step without the gather and against Engine.analyze_batches (the
N = 1 headline).  Rotated, minimum per variant.  Then the receive side of an 8-GPU rank: the
other seven ranks' parts (here: this rank's own records, seven times) read as result tables,
and the cost of rebuilding a whole outcome from the records (assemble_pair) per pair.
usage: tools/rank_step_probe.py [K] [ROUNDS]"""
import os
import socket
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import bench
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    import torch
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from nightcore_analyzer import engine as E
    from nightcore_analyzer import sharded as S
    S.Exchange.collect_at_one = True
    eng = E.get_engine(0)
    flat = [a for nc, src in pairs for a in (nc, src)]
    sig = eng.upload_signals(flat)
    lengths = [len(a) for a in flat]
    params = E.Params(compute_ibi=False)

    def windows(gather):
        res = S.analyze_sharded(S.DeviceStages(eng, sig), params, lengths=lengths, gather=gather, steps=K)
        if gather:
            for r in res:
                r.table()                   # the caller's read of every pair's result row
        return res

    def windows_nopack():
        # the gather with empty records (timing only): what the packing itself costs the step
        add = S._StepRecords.add
        S._StepRecords.add = lambda self, outs: None
        try:
            return windows(True)
        finally:
            S._StepRecords.add = add

    variants = {"analyze_batches": lambda: eng.analyze_batches([sig] * K, params),
                "windows_gather": lambda: windows(True),
                "windows_gather_nopack": windows_nopack,
                "windows_nogather": lambda: windows(False)}
    for f in variants.values():
        f()
    best = {k: [] for k in variants}
    for _ in range(R):
        for k, f in variants.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = f()
            torch.cuda.synchronize()
            best[k].append((time.perf_counter() - t0) / K * 1e3)
            del res
    for k, v in best.items():
        print(f"{k:>18}: {min(v):7.3f} ms/step min, {sorted(v)[len(v) // 2]:7.3f} median "
              f"(runs {[round(x, 3) for x in v]})", flush=True)
    # where the gather's host time goes: one more windows_gather call with its parts timed
    acc = {}

    def timed(owner, name):
        f = getattr(owner, name)

        def w(*a, **kw):
            t = time.perf_counter()
            try:
                return f(*a, **kw)
            finally:
                n, s_ = acc.get(name, (0, 0.0))
                acc[name] = (n + 1, s_ + time.perf_counter() - t)
        setattr(owner, name, w)
        return f

    # records.add runs inside the pipeline as each group is assembled (overlapping the device);
    # records.bytes and gather_bytes run after the last step
    saved = [(S._StepRecords, "add", timed(S._StepRecords, "add")),
             (S._StepRecords, "bytes", timed(S._StepRecords, "bytes")),
             (S.Exchange, "gather_bytes", timed(S.Exchange, "gather_bytes"))]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    windows(True)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) / K * 1e3
    for owner, name, f in saved:
        setattr(owner, name, f)
    print(f"windows_gather (parts timed) {tot:.3f} ms/step; per step: " +
          ", ".join(f"{k} {v[1] / K * 1e3:.3f} ms ({v[0] / K:.1f} calls)" for k, v in acc.items()), flush=True)
    # where records.add's time goes (cProfile around each call only)
    import cProfile
    import pstats
    prof = cProfile.Profile()
    add = S._StepRecords.add

    def profiled(self, outs):
        prof.enable()
        try:
            return add(self, outs)
        finally:
            prof.disable()
    S._StepRecords.add = profiled
    windows(True)
    S._StepRecords.add = add
    pstats.Stats(prof, stream=sys.stdout).sort_stats("tottime").print_stats(14)
    # the receive side of one rank of an 8-GPU job: 7 parts of 64 pairs per step read as tables
    own = windows(False)
    import numpy as np
    B = 8 * 64
    owner = np.repeat(np.arange(8), 64)
    # rank q's part of step k: this rank's records with the pairs numbered as rank q's (64 q + i),
    # one segment per assembly group as the pipeline builds them

    def step_blob(outs, q):
        rec, groups = S._StepRecords(), {}
        for b, o in outs:
            groups.setdefault(id(o._asm[0]) if o._asm is not None else -1, []).append((b + 64 * q, o))
        for v in groups.values():
            rec.add(v)
        return rec.bytes()
    blobs = [{q: step_blob(outs, q) for q in range(1, 8)} for outs in own]
    t0 = time.perf_counter()
    for k in range(K):
        g = S.GatheredOutcomes(B, owner, [], {q: memoryview(v) for q, v in blobs[k].items()}, params)
        tab = g.table()
    rx = (time.perf_counter() - t0) / K * 1e3
    t0 = time.perf_counter()
    n = 0
    for b in range(64, 128):
        g[b]
        n += 1
    rb = (time.perf_counter() - t0) / n * 1e3
    print(f"receive (7 parts x 64 pairs as result tables): {rx:.3f} ms/step; {np.isnan(tab[64:, 1]).sum()} missing "
          f"rows; whole-outcome rebuild from records: {rb:.3f} ms per pair; "
          f"blob {len(blobs[0][1]) / 1024:.1f} KiB per rank-step", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
