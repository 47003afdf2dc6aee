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


def _worker(rank, world, port, names, q, fail_rank, fail_in):
    import torch.distributed as dist
    from nightcore_analyzer.engine import Params
    from nightcore_analyzer.sharded import analyze_sharded
    from sharded_oracle import OracleStages
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pairs = [make_case(synth, n)[:2] for n in names]
        st = OracleStages(pairs, fail_in=fail_in if rank == fail_rank else None)
        outs = analyze_sharded(st, Params())
        q.put((rank, "ok", [(None if o.error is None else (type(o.error).__name__, str(o.error)),
                             None if o.result is None else _norm(dataclasses.asdict(o.result)),
                             None if o.result is None else str(o.result), o.logs) for o in outs]))
    except Exception as exc:               # noqa: BLE001
        q.put((rank, "raised", (type(exc).__name__, str(exc))))
    finally:
        dist.destroy_process_group()


def _run(world, names, fail_rank=-1, fail_in=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, names, q, fail_rank, fail_in)) for r in range(world)]
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
    res = _run(2, ["sweep30"], fail_rank=1, fail_in="tempo")
    assert res[1] == ("raised", ("RuntimeError", "injected failure in tempo"))
    assert res[0][0] == "raised" and res[0][1][0] == "ShardError"
