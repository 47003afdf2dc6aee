"""BASELINE config 4 as a tested workload: 512 three-minute pairs
(seeds 1000 + i) window-sharded over 8 ranks, the 8 ranks here sharing the box's one GPU
and exchanging over gloo (on the driver's 8-GPU node they are 8 GPUs and RCCL).

Each rank generates and uploads only the pairs it needs (ShardPlan.needed), then runs
``sharded.analyze_sharded`` twice, as the reference's pipeline.run would analyse each
pair (pipeline.py:23-216; the nc tempo prior pipeline.py:169-193 is what a split pair
exchanges):

* split_offset 0, Params(compute_ibi=False): the bench's config-4 step; equal pairs fall
  on block boundaries, so every pair is interior (pipelined engine, no exchange);
* split_offset 0.5, run()'s defaults (hop-64 IBI on): every inner boundary cuts a pair,
  so 7 pairs exchange their window and chunk-pair records (C1a, C1b) and split their
  hop-64 IBI pass over the ranks (C2-C4); the API default gather=True then all-gathers the
  outcomes, so every rank holds all 512 (the same list on every rank, checked by digest).

Every rank compares each outcome it owns with ``Engine.analyze`` of the same pairs on
that rank alone, field for field (results, report text, logs, per-window detail).  Against
the CPU oracle (refglue.run_arrays): the owners of pairs 0 and 511 at split_offset 0, and
the owners of the 7 cut pairs at split_offset 0.5, whose windows, chunk pairs and hop-64
IBI pass were split over two ranks and exchanged (IBI ratio and CI included; VERDICT r5
item 5).
"""
import dataclasses
import hashlib
import math
import os
import socket
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import synth

pytestmark = pytest.mark.gpu

WORLD = 8
N_PAIRS = 512
SECONDS = 180.0
CASES = [(0.0, dict(compute_ibi=False)), (0.5, dict())]
ORACLE_PAIRS = (0, N_PAIRS - 1)


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, float) and not math.isfinite(x):
        return repr(x)
    if isinstance(x, np.ndarray):
        return _norm(x.tolist())
    return x


def _key(o):
    d = {k: _norm(v) for k, v in o.detail.items()}
    if o.error is not None:
        return ("error", type(o.error).__name__, str(o.error), o.logs, d)
    return ("ok", _norm(dataclasses.asdict(o.result)), str(o.result), o.logs, d)


def _lengths():
    ln, ls = synth.pair_lengths(SECONDS)
    return [ln, ls] * N_PAIRS


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from nightcore_analyzer.sharded import DeviceStages, analyze_sharded, shard_plan
    from test_gpu_batch import check_against_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = _lengths()
        plans = [(off, E.Params(**kw), shard_plan(L, E.Params(**kw), world, off)) for off, kw in CASES]
        need = sorted(set().union(*(sp.needed(rank, p.compute_ibi) for _, p, sp in plans)))
        with ThreadPoolExecutor(2) as tp:                 # only the pairs this rank needs
            arrays = dict(zip(need, tp.map(lambda b: synth.make_pair(SECONDS, 1000 + b), need)))
        print(f"[config4 rank {rank}] {len(need)} pairs generated", flush=True)
        eng = E.get_engine(0)
        report, keep = [], {}
        for off, p, sp in plans:
            local = sp.needed(rank, p.compute_ibi)
            sig = eng.upload_signals([a for b in local for a in arrays[b]])
            # split_offset 0.5 through the API default gather=True: every rank receives all 512
            # outcomes (its owned ones are checked below, the whole list's digest across ranks)
            gat = off != 0.0
            got = analyze_sharded(DeviceStages(eng, sig), p, lengths=L, local_pairs=local, split_offset=off,
                                  gather=gat)
            owned = sp.owned(rank)
            n_all, digest = None, None
            if gat:
                n_all = len(got)
                digest = hashlib.sha256(repr([_key(o) for o in got]).encode()).hexdigest()
                got = [(b, got[b]) for b in owned]
            ref = eng.analyze([arrays[b] for b in owned], p) if owned else []
            mism = [b for (b, o), r in zip(got, ref) if _key(o) != _key(r)]
            errs = [b for b, o in got if o.error is not None]
            report.append(dict(off=off, owned=[b for b, _ in got], expect=owned, mism=mism, errors=errs,
                               split=int(sp.split.sum()), split_owned=[b for b in owned if sp.split[b]],
                               n_all=n_all, digest=digest))
            if off == 0.0:
                keep = {b: (o, False) for b, o in got if b in ORACLE_PAIRS}
            else:                                          # the cut pairs this rank owns
                keep.update({b: (o, True) for b, o in got if sp.split[b]})
            print(f"[config4 rank {rank}] split_offset {off}: {len(got)} owned, {len(mism)} mismatches", flush=True)
            del sig
        oracle = []
        for b, (o, ibi) in keep.items():                   # pairs 0 and 511; the cut pairs with IBI
            from oracle import refglue
            nc, src = arrays[b]
            try:
                check_against_oracle(o, (nc, src), refglue.run_arrays(nc, src, compute_ibi=ibi), tag=f"pair {b}",
                                     ibi=ibi)
                oracle.append((b, ibi, None))
            except AssertionError as exc:
                oracle.append((b, ibi, repr(exc)))
            print(f"[config4 rank {rank}] pair {b} against the oracle (ibi {ibi}): "
                  f"{'ok' if oracle[-1][2] is None else 'MISMATCH'}", flush=True)
        q.put((rank, dict(cases=report, oracle=oracle)))
    except Exception as exc:          # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_config4_512_pairs_eight_ranks_equal_engine():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=840) for _ in range(WORLD))
    finally:
        for p in procs:
            p.join(timeout=60)
    for p in procs:
        assert p.exitcode == 0
    owned_all = {off: [] for off, _ in CASES}
    split_all = {off: [] for off, _ in CASES}
    oracle_seen = []
    for r in range(WORLD):
        assert isinstance(res[r], dict), (r, res[r])
        for c in res[r]["cases"]:
            assert c["owned"] == c["expect"], (r, c["off"])
            assert not c["errors"], (r, c)
            assert not c["mism"], (r, c["off"], c["mism"])
            owned_all[c["off"]] += c["owned"]
            split_all[c["off"]] += c["split_owned"]
        for b, ibi, err in res[r]["oracle"]:
            assert err is None, (r, b, err)
            oracle_seen.append((b, ibi))
    for off, _ in CASES:
        assert sorted(owned_all[off]) == list(range(N_PAIRS)), off       # every pair owned exactly once
    # gather=True (split_offset 0.5): every rank holds all 512 outcomes, the same list on every rank
    # (each pair's outcome checked against Engine.analyze by its owner above)
    gathered = [c for r in range(WORLD) for c in res[r]["cases"] if c["off"] == 0.5]
    assert [c["n_all"] for c in gathered] == [N_PAIRS] * WORLD
    assert len({c["digest"] for c in gathered}) == 1
    assert split_all[0.0] == [] and len(split_all[0.5]) == WORLD - 1       # 0: no exchange; 0.5: 7 cut pairs
    # pairs 0 and 511 (interior, split_offset 0) and the 7 cut pairs of split_offset 0.5 (IBI on)
    assert sorted(b for b, ibi in oracle_seen if not ibi) == list(ORACLE_PAIRS)
    assert sorted(b for b, ibi in oracle_seen if ibi) == sorted(split_all[0.5])
