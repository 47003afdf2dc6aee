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


# ---- fail together: a failure at any point of a window-sharded
# step raises on every rank (the failing rank's own exception, ShardError on the others) and
# leaves no rank inside a collective.  All cases run one after another in ONE process group:
# a rank left behind in a collective would mismatch (or hang) the next case's collectives.
FAULT_LENGTHS = [882000, 1102500] * 5          # 5 pairs of 40 s / 50 s; world 3, split_offset 0.37:
FAULT_OFFSET = 0.37                            # pairs 2 and 3 split, IBI exchange on (C2-C4)
# (point, failing rank, steps, failing call): rank 2 runs interior pair 4 through the pipeline;
# ranks 0 and 1 own the split pairs (ibi_beats); rank 1 holds split chunk pairs
FAULT_CASES = [("missing", 1, 1, 1), ("missing", 1, 2, 1),
               ("windows", 2, 1, 1), ("tempo", 1, 2, 2), ("chunks", 1, 1, 1), ("chunks", 1, 2, 1),
               ("records", 2, 1, 1), ("records", 0, 2, 1),
               ("ibi_mel", 2, 1, 1), ("ibi_onset", 0, 2, 1), ("ibi_tiles", 1, 1, 1), ("ibi_tiles", 1, 2, 2),
               ("ibi_reduce", 2, 1, 1), ("ibi_reduce", 2, 2, 1), ("ibi_beats", 0, 1, 1), ("ibi_beats", 0, 2, 1),
               ("bootstrap", 1, 2, 1), ("consensus", 2, 1, 1), ("consensus", 2, 2, 1), ("consensus", 0, 2, 2),
               ("pipeline", 2, 1, 1), ("pipeline", 2, 2, 1), ("none", -1, 2, 1)]


def _fault_worker(rank, world, port, q):
    import torch.distributed as dist
    from nightcore_analyzer import sharded
    from nightcore_analyzer.engine import Params
    from sharded_oracle import FakeStages
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = Params(compute_ibi=True)
    out = []
    try:
        for point, fr, steps, call in FAULT_CASES:
            mine = rank == fr
            sharded.FAULTS.clear()
            if mine and point in ("records", "consensus"):
                sharded.FAULTS[point] = call
            st = FakeStages(FAULT_LENGTHS, fail_in=point if mine else None, fail_call=call)
            local = None
            if mine and point == "missing":
                sp = sharded.shard_plan(FAULT_LENGTHS, p, world, FAULT_OFFSET)
                need = sp.needed(rank, True)
                local = [b for b in range(sp.B) if b != need[0]]
                st = st.restrict([f for b in local for f in (2 * b, 2 * b + 1)])
            try:
                res = sharded.analyze_sharded(st, p, lengths=FAULT_LENGTHS, local_pairs=local,
                                              split_offset=FAULT_OFFSET, steps=steps)
                out.append(("ok", len(res)))
            except Exception as exc:        # noqa: BLE001
                out.append(("raised", type(exc).__name__, str(exc)))
        q.put((rank, out))
    except BaseException as exc:            # noqa: BLE001
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


def test_window_sharded_fails_together_at_every_point():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_fault_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert isinstance(res[r], list), (r, res[r])
        assert len(res[r]) == len(FAULT_CASES)
        for (point, fr, steps, call), got in zip(FAULT_CASES, res[r]):
            case = (point, fr, steps, call, r)
            if point == "none":
                assert got == ("ok", steps), case
            elif r != fr:
                assert got[:2] == ("raised", "ShardError"), (case, got)
            elif point == "missing":
                assert got[:2] == ("raised", "ValueError") and "needs pairs" in got[2], (case, got)
            else:
                assert got == ("raised", "RuntimeError", f"injected failure in {point}"), (case, got)


def _loud_tail_signal(seconds=12.0, seed=7):
    """A quiet body (noise + tone at -60 dB) with a loud 3 kHz burst in the file's last 14 ms:
    the loudest mel bin lies in rows no onset reads (T - 16 .. T - 1 at hop 64)."""
    rng = np.random.default_rng(seed)
    n = int(seconds * 22050)
    t = np.arange(n) / 22050
    y = 1e-3 * (rng.standard_normal(n) + np.sin(2 * np.pi * 440 * t))
    y[-300:] += np.sin(2 * np.pi * 3000 * t[-300:])
    return y.astype(np.float32)


def test_split_ibi_share_bounds_cover_the_maximum():
    """in the split hop-64 pass the share that ends a file also computes
    mel rows T - 16 .. T - 1, which feed only power_to_db's maximum.  Over world 1..4 the
    all-reduced maximum of the shares equals the maximum over every row, as on one GPU, and
    the split onsets equal the oracle's whole-file onsets."""
    from nightcore_analyzer.sharded import IBI_PAD, _ibi_mel_rows, _ibi_share
    from oracle import ncref
    from sharded_oracle import OracleStages
    y = _loud_tail_signal()
    S = ncref.mel_db(y, 22050, 2048, 64)
    T = S.shape[1]
    assert T == 1 + len(y) // 64
    # the case is sensitive: the rows the onsets read miss the maximum by a wide margin
    assert S.max() > S[:, :T - IBI_PAD + 1].max() + 3.0
    full = ncref.onset_strength(y, 22050, 64)
    st = OracleStages([(y, y)])
    for world in (1, 2, 3, 4):
        shares = [_ibi_share(T, world, q) for q in range(world)]
        rows = _ibi_mel_rows([T] * world, [s[2] for s in shares], [s[3] for s in shares])
        assert max(r[1] for r in rows) == T and rows[0][0] == 0
        mx = max(float(st.ibi_mel([0], [len(y)], [s[2]], [s[3]])[0]) for s in shares)
        assert mx == float(S.max())
        seg = []
        for s in shares:
            st.ibi_mel([0], [len(y)], [s[2]], [s[3]])
            seg.append(st.ibi_onset(np.array([mx])))
        np.testing.assert_array_equal(np.concatenate(seg), full)


def _melodia_worker(rank, world, port, q):
    import torch.distributed as dist
    from nightcore_analyzer import sharded
    from nightcore_analyzer.engine import Params
    from sharded_oracle import FakeStages
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def hook(b, chroma_st, log, span):
            calls.append((b, span))
            log("    melodia hook")
            return None
        st = FakeStages(FAULT_LENGTHS)
        st.pipeline = None                    # every pair through the stage path
        sp = sharded.shard_plan(FAULT_LENGTHS, Params(), world, FAULT_OFFSET)
        local = sp.needed(rank, True)
        st = st.restrict([f for b in local for f in (2 * b, 2 * b + 1)])
        st.pipeline = None
        outs = sharded.analyze_sharded(st, Params(compute_ibi=True, melodia=hook), lengths=FAULT_LENGTHS,
                                       local_pairs=local, split_offset=FAULT_OFFSET, gather=False)
        q.put((rank, (calls, [b for b, _ in outs], sp.owned(rank))))
    except BaseException as exc:            # noqa: BLE001
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


def test_window_sharded_melodia_hook_gets_global_pairs():
    """in window mode the MELODIA hook is called for every owned pair with
    the pair's GLOBAL index and its trimmed (src, nc) spans relative to the files, as
    pipeline.run_batch calls it (essentia itself is absent: the hook here records its calls)."""
    from nightcore_analyzer.engine import Params
    from nightcore_analyzer.sharded import _local_melodia
    seen = []
    p = _local_melodia(Params(melodia=lambda b, st, log, span: seen.append(b)), [5, 9, 11])
    p.melodia(1, 0.0, None, None)
    assert seen == [9]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_melodia_worker, args=(r, 3, port, q)) for r in range(3)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=240) for _ in range(3))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for r in range(3):
        assert isinstance(res[r], tuple), res[r]
        calls, got, owned = res[r]
        assert got == owned
        assert [b for b, _ in calls] == owned
        for b, span in calls:
            assert span == ((0, FAULT_LENGTHS[2 * b + 1]), (0, FAULT_LENGTHS[2 * b])), (b, span)
