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

    variants = {"analyze_batches": lambda: eng.analyze_batches([sig] * K, params),
                "windows_gather": lambda: windows(True),
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
        print(f"{k:>18}: {min(v):7.3f} ms/step (runs {[round(x, 3) for x in v]})", flush=True)
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

    saved = [(S, "pack_outcomes", timed(S, "pack_outcomes")),
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
    # the receive side of one rank of an 8-GPU job: 7 parts of 64 pairs per step read as tables
    own = windows(False)
    blobs = [S.pack_outcomes(outs) for outs in own]
    import numpy as np
    B = 8 * 64
    owner = np.repeat(np.arange(8), 64)
    t0 = time.perf_counter()
    for k in range(K):
        parts = {q: memoryview(blobs[k]) for q in range(1, 8)}
        g = S.GatheredOutcomes(B, owner, [], parts, params)
        # rank q's part holds pairs 0..63 of its own numbering: shift to the global indices
        for q, part in g._parts.items():
            t = part.tables()
            t["pairs"] = t["pairs"].copy()
            t["pairs"][:, 0] += 64 * q
            part.where = {int(b): i for i, b in enumerate(t["pairs"][:, 0].tolist())}
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
          f"blob {len(blobs[0]) / 1024:.1f} KiB per rank-step", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
