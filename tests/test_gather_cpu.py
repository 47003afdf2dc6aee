"""The window-sharded result gather on the CPU (gloo): every rank's owned outcomes pickled
with their log lines unrendered (engine._Lines), one byte all-gather per step
(sharded.Exchange.gather_bytes), the other ranks' outcomes unpickled on first access
(sharded.GatheredOutcomes)."""
import os
import pickle
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from nightcore_analyzer import consensus as C
from nightcore_analyzer import engine as E
from nightcore_analyzer import sharded as S


def _outcome(b: int) -> E.PairOutcome:
    o = E.PairOutcome()
    o._log_ops.append(f"pair {b}")
    o._log_ops.append(E._Lines(E._log_tempo_windows, np.arange(3, dtype=np.int64) * 110250 + b, 220500))
    o._log_ops.append(E._Lines(E._log_chroma, 0.25 * b, -0.5, 1.0 + b, 1 + b % 2))
    o.detail.update(energy_src=np.linspace(0, 1, 5 + b), n_src_windows=b)
    if b % 3 == 2:
        o.error = ValueError(f"pair {b} failed")
    else:
        o.result = C.AnalysisResult(tempo_ratio=1.0 + b, pitch_ratio=1.0, tempo_ci=(1.0, 2.0), pitch_ci=(0.5, 1.5),
                                    classification="x", n_source_pitch_windows=1, n_nc_pitch_windows=1,
                                    n_source_tempo_windows=2, n_nc_tempo_windows=2, src_tempos_raw=[120.0, None])
    return o


def _key(o):
    return (None if o.result is None else repr(o.result), repr(o.error), o.logs,
            {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in o.detail.items()})


def test_deferred_lines_pickle_and_render_the_same():
    o = _outcome(4)
    o2 = pickle.loads(pickle.dumps(o))
    assert o2.logs == o.logs
    assert o.logs[1] == "    tempo window 1/3  [0.0–10.0 s]"


def test_gathered_outcomes_single_process_view():
    own = [(1, _outcome(1)), (3, _outcome(3))]
    other = S._dumps_outcomes([(0, _outcome(0)), (2, _outcome(2))])
    g = S.GatheredOutcomes(4, np.array([1, 0, 1, 0]), own, {1: memoryview(other)})
    assert len(g) == 4 and g.decoded() == 1
    assert g[1] is own[0][1] and g.decoded() == 1         # own pairs: no unpickling
    assert [_key(o) for o in g] == [_key(_outcome(b)) for b in range(4)]
    assert g.decoded() == 0 and g[-1] is g[3] and [_key(o) for o in g[1:3]] == [_key(_outcome(b)) for b in (1, 2)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, at_one=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = 7
        owner = np.array([b * world // B for b in range(B)])
        own = [(b, _outcome(b)) for b in range(B) if owner[b] == rank]
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
        parts = ex.gather_bytes(S._dumps_outcomes(own))
        assert len(parts) == world
        g = S.GatheredOutcomes(B, owner, own, {r: parts[r] for r in range(world) if r != rank})
        q.put((rank, [_key(o) for o in g]))
    except Exception as exc:     # noqa: BLE001
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


def test_byte_gather_three_ranks_every_rank_holds_every_outcome():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = [_key(_outcome(b)) for b in range(7)]
    for r in range(world):
        assert res[r] == ref, res[r]


def test_one_rank_group_runs_the_collectives_with_collect_at_one():
    """Exchange.collect_at_one (the one-rank RCCL test on the GPU box, tests/test_gpu_rccl.py):
    at world size 1 the record gather, the all-reduce, the flag and the byte gather are still
    issued and return the rank's own data."""
    assert S.Exchange().local          # no process group: nothing is issued
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), q, True))
    p.start()
    r, got = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert got == [_key(_outcome(b)) for b in range(7)], got


def test_fast_pickler_round_trips_arrays():
    """sharded._OutcomePickler sends numeric arrays as (dtype, shape, bytes): same values,
    dtypes and shapes after unpickling, writable copies."""
    x = {"a": np.arange(12, dtype=np.float32).reshape(3, 4), "b": np.array([1, -2], np.int32),
         "c": np.zeros((0,), np.float64), "d": np.array([True, False]), "s": "text"}
    y = pickle.loads(S._pickle_fast(x))
    for k in "abcd":
        assert y[k].dtype == x[k].dtype and y[k].shape == x[k].shape and np.array_equal(y[k], x[k])
        assert y[k].flags.writeable
    assert y["s"] == "text"


@pytest.mark.parametrize("sizes", [[5], [0, 7, 3], [300, 1, 0, 44]])
def test_steps_pack_round_trip(sizes):
    """analyze_sharded(steps=K) gathers the K steps' blobs as one: lengths table, then blobs."""
    blobs = [bytes((i * 7 + j) % 256 for j in range(n)) for i, n in enumerate(sizes)]
    got = S._unpack_steps(memoryview(S._pack_steps(blobs)), len(blobs))
    assert [bytes(x) for x in got] == blobs
