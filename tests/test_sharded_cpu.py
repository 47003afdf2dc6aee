"""Window-sharded multi-rank analysis (nightcore_analyzer.sharded) over gloo on the CPU:
the per-window record exchange, the energy gate over gathered energies, the nc prior
from gathered source records, the chunk-pair split and the consensus on each pair's
owner, with the stage work done by the oracle (tests/sharded_oracle.py).

Results on every rank must equal the reference's own pipeline.run goldens field for
field (report text and logs included), for a single pair spread over 2 ranks and for
2 pairs over 3 ranks (one rank owns no pair)."""
import dataclasses
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nightcore_analyzer import synth
from golden.cases import make_case

N_LOAD_LINES = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, float) and not math.isfinite(x):
        return repr(x)
    return x


def _worker(rank, world, port, names, q, fail_rank, fail_in, split_offset=0.0):
    import torch.distributed as dist
    from nightcore_analyzer.engine import Params
    from nightcore_analyzer.sharded import analyze_sharded
    from sharded_oracle import OracleStages
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pairs = [make_case(synth, n)[:2] for n in names]
        st = OracleStages(pairs, fail_in=fail_in if rank == fail_rank else None)
        outs = analyze_sharded(st, Params(), split_offset=split_offset)
        q.put((rank, "ok", [(None if o.error is None else (type(o.error).__name__, str(o.error)),
                             None if o.result is None else _norm(dataclasses.asdict(o.result)),
                             None if o.result is None else str(o.result), o.logs) for o in outs]))
    except Exception as exc:               # noqa: BLE001
        q.put((rank, "raised", (type(exc).__name__, str(exc))))
    finally:
        dist.destroy_process_group()


def _run(world, names, fail_rank=-1, fail_in=None, split_offset=0.0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, names, q, fail_rank, fail_in,
                                                                split_offset)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (kind, v)) for r, kind, v in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _check_golden(outs, names, golden):
    assert len(outs) == len(names)
    for (err, res, text, logs), n in zip(outs, names):
        g = golden[n]
        assert logs == g["log"][N_LOAD_LINES:], n
        if "error" in g:                      # run() raises: the outcome carries the same exception
            assert err == (g["error"]["type"], g["error"]["message"]), (n, err)
            continue
        assert err is None, (n, err)
        for k, v in g["result"].items():
            assert res[k] == v, (n, k)
        assert text == g["str"], n


@pytest.mark.parametrize("world,names", [(2, ["chords80"]), (3, ["sweep30", "chords80"])])
def test_window_sharded_matches_reference_goldens(golden_pipeline, world, names):
    res = _run(world, names)
    for r in range(world):
        kind, outs = res[r]
        assert kind == "ok", (r, outs)
        _check_golden(outs, names, golden_pipeline)


def test_window_sharded_failure_raises_on_every_rank():
    # sweep30 on 2 ranks: rank 0 holds the 8 windows, rank 1 the chunk pair (shard_plan)
    res = _run(2, ["sweep30"], fail_rank=1, fail_in="chunks")
    assert res[1] == ("raised", ("RuntimeError", "injected failure in chunks"))
    assert res[0][0] == "raised" and res[0][1][0] == "ShardError"


def test_shard_plan_blocks():
    """The item plan: every slot on exactly one rank, contiguous pair-major blocks of nearly
    equal cost, owners non-decreasing, and no split pair when the blocks align with pairs."""
    from nightcore_analyzer.engine import Params
    from nightcore_analyzer.sharded import CP_COST, shard_plan
    p = Params()
    L = [3175200, 3969000] * 16                    # 16 equal 3-min pairs (config 3/4 shape)
    for world in (1, 2, 4, 8):
        sp = shard_plan(L, p, world)
        assert not sp.split.any() and sp.n_wrows == 0
        assert [len(sp.owned(r)) for r in range(world)] == [16 // world] * world
    sp = shard_plan(L, p, 4, split_offset=0.5)     # every inner boundary through a pair's middle
    assert sp.split.sum() == 3 and sp.n_wrows == 3 * 62 and sp.n_crows == 3 * 7
    lens = [int(x) for x in np.random.default_rng(5).integers(200_000, 4_000_000, 22)]
    for world, off in ((3, 0.0), (5, 0.3), (7, 0.9)):
        sp = shard_plan(lens, p, world, off)
        cover = np.zeros_like(sp.slots)
        for r in range(world):
            cover += sp.rng[:, :, r, 1] - sp.rng[:, :, r, 0]
        assert np.array_equal(cover, sp.slots)
        assert np.all(np.diff(sp.owner) >= 0)
        rows = np.concatenate([sp.contrib_w(r) for r in range(world)])
        assert np.array_equal(np.sort(rows), np.arange(sp.n_wrows))
        cost = [(sp.rng[:, 0, r, 1] - sp.rng[:, 0, r, 0] + sp.rng[:, 1, r, 1] - sp.rng[:, 1, r, 0]).sum()
                + CP_COST * (sp.rng[:, 2, r, 1] - sp.rng[:, 2, r, 0]).sum() for r in range(world)]
        if off == 0.0:
            assert max(cost) - min(cost) <= 2 * CP_COST, cost
        for b in range(sp.B):
            assert sp.owner[b] in [r for r in range(world) if sp.on_rank(b, r)] or sp.slots[b].sum() == 0


def test_window_sharded_split_pairs_match_reference_goldens(golden_pipeline):
    """Four pairs on three ranks with every block boundary moved into a pair: split pairs
    exchange their window and chunk-pair records (C1a, C1b); an error-path pair raises the
    reference's ValueError with its logs."""
    names = ["chords80", "sweep30", "sweep30_nc_tail_quiet", "chords80"]
    res = _run(3, names, split_offset=0.37)
    for r in range(3):
        kind, outs = res[r]
        assert kind == "ok", (r, outs)
        _check_golden(outs, names, golden_pipeline)
