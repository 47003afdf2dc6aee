"""The window-sharded result gather on the CPU: every rank's owned outcomes travel as record
tables, not pickles (sharded.pack_outcomes: a fixed-size result row per pair and, per assembly
group, the inputs assemble_pair read), one byte all-gather per call (Exchange.gather_bytes),
the other ranks' outcomes rebuilt by the same assemble_pair call on first access and their
result rows readable as one table (sharded.GatheredOutcomes).

The outcomes are real ones: the oracle stages (tests/sharded_oracle.py) analyse the golden
sweep30 pair, once with the hop-64 IBI pass, once through the energy-gate failure path, and
once with a stand-in MELODIA hook whose answer and log lines the receiver replays."""
import dataclasses
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nightcore_analyzer import sharded as S
from nightcore_analyzer import synth
from nightcore_analyzer.engine import Params
from golden.cases import make_case


def _melodia_hook(b, point_st, log, span):
    """A stand-in for essentia's MELODIA step (engine.assemble_pair calls it on the owner)."""
    log("    MELODIA: stand-in accepted")
    log(f"    MELODIA shift {point_st:+.3f} st")
    return [440.0, None, 441.5, 439.0], [550.0, 551.0, None, 552.5]


CASES = {
    "ibi": Params(),
    "gate_error": Params(energy_gate_db=1.0, compute_ibi=False),
    "melodia": Params(compute_ibi=False, melodia=_melodia_hook),
}


@pytest.fixture(scope="module")
def outcomes():
    """The owners' outcomes.  The MELODIA case's bootstrap of the accepted lists runs on the
    device in the product (consensus._bootstrap_ratio); here the oracle's numpy restatement
    stands in for it on the owner, and the receiver must replay the owner's answer, not redo it."""
    from oracle import refglue
    from nightcore_analyzer import consensus as C
    from sharded_oracle import OracleStages
    pair = make_case(synth, "sweep30")[:2]
    mp_ = pytest.MonkeyPatch()
    mp_.setattr(C, "_bootstrap_ratio", lambda a, b: refglue.bootstrap_ratio(a, b))
    try:
        return {k: S.analyze_sharded(OracleStages([pair]), p)[0] for k, p in CASES.items()}
    finally:
        mp_.undo()


def _norm(x):
    if isinstance(x, float) and math.isnan(x):
        return "nan"
    if isinstance(x, np.ndarray):
        return (x.dtype.str, x.shape, _norm(x.tolist()))
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [type(x).__name__] + [_norm(v) for v in x]
    return x


def _key(o):
    return (None if o.result is None else (_norm(dataclasses.asdict(o.result)), str(o.result)),
            None if o.error is None else (type(o.error).__name__, str(o.error)), o.logs, _norm(o.detail))


def test_tables_round_trip():
    t = {"a": np.arange(12, dtype=np.float32).reshape(3, 4), "b": np.array([1, -2, 7], np.int32),
         "c": np.zeros((0,), np.float64), "d": np.array([True, False]), "e": np.array(3.5),
         "f": np.arange(5, dtype=np.uint8), "g": np.array([2 ** 40, -3], np.int64)}
    got = S.unpack_tables(S.pack_tables(t))
    assert list(got) == list(t)
    for k, v in t.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape and np.array_equal(got[k], v), k
    with pytest.raises(TypeError):
        S.pack_tables({"o": np.array([None, 1.0], dtype=object)})


@pytest.mark.parametrize("case", list(CASES))
def test_outcome_rebuilt_from_records_equals_the_owners(outcomes, case):
    """Another rank's view of a pair: result, report text, warnings, logs (MELODIA's replayed
    lines included), error and every detail array (values, dtypes, shapes) equal the owner's."""
    o = outcomes[case]
    assert o._asm is not None
    blob = S.pack_outcomes([(1, o)])
    g = S.GatheredOutcomes(2, np.array([0, 1]), [], {1: memoryview(blob)}, CASES[case])
    assert g.decoded() == 2
    r = g[1]
    assert r is not o and _key(r) == _key(o)
    assert g.decoded() == 1 and g[1] is r and g[-1] is r
    if case == "melodia":
        assert r.result.pitch_method == "chroma+melodia" and "    MELODIA: stand-in accepted" in r.logs
    if case == "gate_error":
        assert isinstance(r.error, RuntimeError) and r.result is None
    with pytest.raises(S.ShardError):
        g[0]                              # rank 0's part did not arrive


def test_result_table_without_rebuilding(outcomes):
    """table(): every pair's RES_FIELDS row from the records, nothing rebuilt."""
    own = [(0, outcomes["ibi"])]
    blob = S.pack_outcomes([(1, outcomes["gate_error"]), (2, outcomes["ibi"])])
    g = S.GatheredOutcomes(3, np.array([0, 1, 1]), own, {1: memoryview(blob)})
    tab = g.table()
    assert g.decoded() == 2
    assert tab.shape == (3, len(S.RES_FIELDS))
    r = outcomes["ibi"].result
    assert tab[2, S.RES_FIELDS.index("tempo_ratio")] == r.tempo_ratio
    assert tab[2, S.RES_FIELDS.index("ibi_hi")] == r.ibi_ci[1]
    assert np.array_equal(tab[0], tab[2], equal_nan=True) and tab[1, 0] == 0.0 and np.isnan(tab[1, 1:]).all()
    assert _norm(tab[2].tolist()) == _norm(np.array(S.result_row(outcomes["ibi"]), np.float64).tolist())


def test_records_in_segments(outcomes):
    """A step's records built a pair group at a time (the engine pipeline's on_group hook adds
    each group as it is assembled): every segment's pairs rebuild from their own segment, the
    result table reads every row without parsing a segment, and a truncated part is refused."""
    from nightcore_analyzer.engine import PairOutcome
    o = outcomes["ibi"]
    rec = S._StepRecords()
    rec.add([(3, o)])
    rec.add([(1, PairOutcome()), (0, o)])
    rec.add([])
    blob = rec.bytes()
    g = S.GatheredOutcomes(4, np.array([1, 1, 0, 1]), [], {1: memoryview(blob)})
    tab = g.table()
    assert g.decoded() == 4 and len(g._parts[1].seg) == 2
    assert tab[1, 0] == 0.0 and np.isnan(tab[2]).all()
    assert _norm(tab[0].tolist()) == _norm(tab[3].tolist()) == _norm(np.array(S.result_row(o), np.float64).tolist())
    assert _key(g[3]) == _key(o) and _key(g[0]) == _key(o) and g[1] == PairOutcome()
    assert len(g._parts[1].t) == 2             # both segments parsed, once each
    for cut in (10, len(blob) - 1):
        with pytest.raises(S.ShardError):
            S.GatheredOutcomes(4, np.array([1, 1, 0, 1]), [], {1: memoryview(blob[:cut])})


def test_arena_views_travel_as_one_array(outcomes):
    """The engine's host views are carved from one pinned arena (engine._Arena.to_host): the
    records send the arena's bytes once and a header entry per view, and the rebuilt outcome
    equals the owner's.  A view replaced after the arena was made travels as its own array."""
    import dataclasses as dc
    from nightcore_analyzer.engine import _HostViews
    o = outcomes["ibi"]
    ctx, j = o._asm
    arrays = {k: np.asarray(v) for k, v in ctx.h.items()
              if isinstance(v, np.ndarray) and not k.endswith("_l") and not k.startswith("ibi_")}
    offs, total = {}, 0
    for k, v in arrays.items():
        total = (total + 15) & ~15
        offs[k] = total
        total += v.nbytes
    hb = np.zeros(max(16, total), np.uint8)
    h = _HostViews({k: v for k, v in ctx.h.items() if k not in arrays and k[:-2] not in arrays})
    lay = {}
    for k, v in arrays.items():
        view = hb[offs[k]:offs[k] + v.nbytes].view(v.dtype).reshape(v.shape)
        view[...] = v
        h[k] = view
        lay[k] = (view, offs[k])
    moved = next(iter(arrays))
    h[moved] = arrays[moved].copy()            # no longer the arena's view
    actx = dc.replace(ctx, h=h, arena=(hb, lay))
    ref = actx.assemble(j, CASES["ibi"])
    assert _key(ref) == _key(o)
    rec = S._StepRecords()
    rec.add([(1, ref)])
    g = S.GatheredOutcomes(2, np.array([0, 1]), [], {1: memoryview(rec.bytes())}, CASES["ibi"])
    assert _key(g[1]) == _key(o)
    t = g._parts[1].tables(0)
    assert "c0.arena" in t and t["c0.arena"].nbytes == hb.nbytes
    for k in arrays:                            # every view but the replaced one points into the arena
        inside = np.shares_memory(t["c0.h." + k], t["c0.arena"])
        assert inside == (k != moved), k


def test_outcome_without_assembly_inputs_is_refused():
    """An outcome not built by assemble_pair cannot be rebuilt elsewhere: refused (an empty
    one, e.g. a stage fake's, travels as empty)."""
    from nightcore_analyzer.engine import PairOutcome
    o = PairOutcome()
    o._log_ops.append("a line")
    with pytest.raises(ValueError):
        S.pack_outcomes([(0, o)])
    g = S.GatheredOutcomes(1, np.array([1]), [], {1: memoryview(S.pack_outcomes([(0, PairOutcome())]))})
    assert g[0] == PairOutcome() and g.table()[0, 0] == 0.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, blobs, owner, q, at_one=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = S.Exchange()
        ex.collect_at_one = at_one
        assert ex.local == (world == 1 and not at_one)
        if at_one:
            rows = np.arange(6.0).reshape(2, 3)
            assert np.array_equal(ex.gather_blocks(rows, [2], None), rows)
            assert np.array_equal(ex.allreduce_max(np.array([1.5, -2.0]), None), [1.5, -2.0])
            try:
                ex.check(KeyError("held"))
                raise AssertionError("the held error did not raise")
            except KeyError:
                pass
        parts = ex.gather_bytes(blobs[rank])
        assert len(parts) == world
        assert all(bytes(parts[r]) == blobs[r] for r in range(world))
        g = S.GatheredOutcomes(len(owner), np.array(owner), [], {r: parts[r] for r in range(world)},
                               CASES["ibi"])
        q.put((rank, [_key(o) for o in g], g.table().tolist()))
    except Exception as exc:     # noqa: BLE001
        q.put((rank, repr(exc), None))
    finally:
        dist.destroy_process_group()


def _spawn(world, blobs, owner, at_one=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, blobs, owner, q, at_one)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (k, t) for r, k, t in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_byte_gather_three_ranks_every_rank_holds_every_outcome(outcomes):
    """Three gloo ranks, rank 2 owning nothing: every rank rebuilds all four outcomes (one
    Params for the batch, as in analyze_sharded) and reads the same result table."""
    o = outcomes["ibi"]
    per_rank = [[(0, o), (1, o)], [(2, o), (3, o)], []]
    owner = [0, 0, 1, 1]
    blobs = [S.pack_outcomes(x) for x in per_rank]
    res = _spawn(3, blobs, owner)
    ref = [_key(o)] * 4
    for r in range(3):
        keys, tab = res[r]
        assert keys == ref, (r, keys)
        assert _norm(tab) == _norm([np.array(S.result_row(o), np.float64).tolist()] * 4)


def test_one_rank_group_runs_the_collectives_with_collect_at_one(outcomes):
    """Exchange.collect_at_one (the one-rank RCCL test on the GPU box, tests/test_gpu_rccl.py):
    at world size 1 the record gather, the all-reduce, the flag and the byte gather are still
    issued and return the rank's own data."""
    assert S.Exchange().local          # no process group: nothing is issued
    o = outcomes["ibi"]
    res = _spawn(1, [S.pack_outcomes([(0, o)])], [0], at_one=True)
    keys, _ = res[0]
    assert keys == [_key(o)], keys


@pytest.mark.parametrize("sizes", [[5], [0, 7, 3], [300, 1, 0, 44]])
def test_steps_pack_round_trip(sizes):
    """analyze_sharded(steps=K) gathers the K steps' blobs as one: lengths table, then blobs."""
    blobs = [bytes((i * 7 + j) % 256 for j in range(n)) for i, n in enumerate(sizes)]
    got = S._unpack_steps(memoryview(S._pack_steps(blobs)), len(blobs))
    assert [bytes(x) for x in got] == blobs


def _fail_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = S.Exchange()
        err = ValueError("cannot pack") if rank == 1 else None
        try:
            ex.gather_bytes(b"abc", err)
            got = ("ok",)
        except Exception as exc:     # noqa: BLE001
            got = ("raised", type(exc).__name__)
        parts = ex.gather_bytes(bytes([rank]) * (rank + 1))   # the group is still in step
        q.put((rank, got, [bytes(x) for x in parts]))
    finally:
        dist.destroy_process_group()


def test_byte_gather_fails_together():
    """A rank whose outcomes cannot be packed raises its own error; the others raise ShardError
    after the same collective, and the next gather still matches across the ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = {r: (g, parts) for r, g, parts in (q.get(timeout=120) for _ in range(3))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(3):
        g, parts = res[r]
        assert g == ("raised", "ValueError" if r == 1 else "ShardError"), (r, g)
        assert parts == [bytes([q_]) * (q_ + 1) for q_ in range(3)]
