"""RCCL on the box's one GPU: a one-rank "nccl" process group (RCCL cannot put two ranks on
one device, and the 8-GPU runs are the driver's), with sharded.Exchange.collect_at_one so
every collective of the window-sharded path is issued anyway:

* Exchange's record gather (C1a/C1b), the dB-maximum all-reduce (C2), the fail-together flag
  and the outcome byte gather, on device tensors on the split-pair stream, equal their inputs;
  a held error raises through the flag;
* run_window_sharded with gather=True through that group (the fail-together check and the
  byte all-gather of the pickled outcomes under RCCL) equals Engine.analyze field for field.

The process group lives in a spawned child so the test process keeps none.
"""
import os
import pickle
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _child(port, q):
    import torch.distributed as dist
    from nightcore_analyzer import engine as E
    from nightcore_analyzer import synth
    from nightcore_analyzer import sharded as S
    from golden.cases import make_case
    from test_gpu_sharded import _key
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    out = {}
    try:
        out["backend"] = dist.get_backend()
        out["rccl"] = ".".join(map(str, torch.cuda.nccl.version()))
        S.Exchange.collect_at_one = True
        ex = S.Exchange()
        ex.stream = torch.cuda.Stream()
        out["dev"] = str(ex.dev)
        rng = np.random.default_rng(7)
        rows = rng.standard_normal((5, 3))
        out["blocks"] = bool(np.array_equal(ex.gather_blocks(rows, [5], None), rows))
        v = rng.standard_normal(4)
        out["max"] = bool(np.array_equal(ex.allreduce_max(v, None), v))
        blob = pickle.dumps([(0, "x" * 1000), (3, list(range(50)))])
        parts = ex.gather_bytes(blob)
        out["bytes"] = len(parts) == 1 and bytes(parts[0]) == blob
        try:
            ex.check(ValueError("held"))
            out["raised"] = None
        except ValueError as e:
            out["raised"] = str(e)
        eng = E.get_engine(0)
        pairs = [make_case(synth, n)[:2] for n in ("chords80", "sweep30")] + [synth.make_pair(150.0, 1234)]
        ref = [_key(o) for o in eng.analyze(pairs, E.Params())]
        got = S.run_window_sharded(pairs, E.Params(), device=0)
        out["gathered_type"] = type(got).__name__
        out["equal"] = [_key(o) for o in got] == ref
        out["n"] = len(got)
        q.put(out)
    except Exception as exc:     # noqa: BLE001
        out["error"] = repr(exc)
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_one_rank_rccl_exchange_and_gather():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=150)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert "error" not in out, out
    assert out["backend"] == "nccl" and out["dev"] == "cuda:0", out
    assert out["blocks"] and out["max"] and out["bytes"], out
    assert out["raised"] == "held", out
    assert out["gathered_type"] == "GatheredOutcomes" and out["n"] == 3 and out["equal"], out
    print("RCCL", out["rccl"])
