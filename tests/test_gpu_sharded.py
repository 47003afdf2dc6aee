"""GPU runs of the window-sharded path (nightcore_analyzer.sharded with DeviceStages):

* one rank: every outcome equals Engine.analyze of the same batch (results, report,
  logs, per-window detail) — interior pairs through the pipelined engine;
* two ranks on the one GPU of the box (gloo for the record exchange, libncgpu for the
  stages): a single pair split over both ranks reproduces the reference's own
  pipeline.run goldens, on both ranks;
* four ranks on the one GPU over a 17-pair batch (3 golden pairs + 14 synthetic pairs of
  90-200 s) with every block boundary moved into a pair (split_offset): interior pairs
  through the engine pipeline, split pairs through the stage path and the C1a/C1b
  exchanges; every outcome equals Engine.analyze of the whole batch on one rank, field
  for field, on every rank.

The 8-GPU RCCL run is the driver's; here the exchange is the same all_gather_into_tensor
call, on CPU tensors and (exchange_device) on device tensors through gloo.
"""
import dataclasses
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from nightcore_analyzer import engine as E
from nightcore_analyzer import synth
from golden.cases import make_case

pytestmark = pytest.mark.gpu
N_LOAD_LINES = 4


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


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


@pytest.mark.parametrize("names", [["chords80", "sweep30", "sweep30_nc_tail_quiet"], ["chords60_intro"],
                                   ["sweep30_gate_all"]])
def test_sharded_single_rank_equals_engine(eng, names):
    from nightcore_analyzer.sharded import run_window_sharded
    cases = [make_case(synth, n) for n in names]
    kw = cases[0][2]
    pairs = [c[:2] for c in cases] + ([synth.make_pair(180.0, 1000)] if not kw else [])
    p = E.Params(**kw)
    ref = eng.analyze(pairs, p)
    got = run_window_sharded(pairs, p)
    assert [_key(o) for o in got] == [_key(o) for o in ref]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, names, q, split_offset=0.0, full=False, exchange_device=None):
    import torch.distributed as dist
    from nightcore_analyzer.sharded import run_window_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pairs = _batch(names)
        outs = run_window_sharded(pairs, E.Params(), device=0, split_offset=split_offset,
                                  exchange_device=exchange_device)
        if full:
            q.put((rank, [_key(o) for o in outs]))
        else:
            q.put((rank, [(None if o.error is None else str(o.error),
                           None if o.result is None else _norm(dataclasses.asdict(o.result)),
                           None if o.result is None else str(o.result), o.logs) for o in outs]))
    except Exception as exc:     # noqa: BLE001
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


def _batch(names):
    """Golden cases by name; ("syn", seconds, seed) entries are synthetic pairs."""
    return [synth.make_pair(n[1], n[2]) if isinstance(n, tuple) else make_case(synth, n)[:2] for n in names]


def _spawn(world, names, split_offset=0.0, full=False, timeout=240, exchange_device=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, names, q, split_offset, full, exchange_device))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("exchange_device", [None, "cuda:0"])
def test_sharded_two_ranks_one_pair_matches_reference(eng, golden_pipeline, exchange_device):
    """One pair split over two ranks.  With exchange_device "cuda:0" the records take the
    device-tensor path of sharded.Exchange that RCCL runs (upload on the split-pair stream,
    all_gather_into_tensor / all_reduce of device tensors, read-back), here through gloo's
    CUDA-tensor collectives, C1a, C1b and the split IBI pass's C2-C4 included."""
    names = ["chords80"]
    res = _spawn(2, names, exchange_device=exchange_device)
    g = golden_pipeline["chords80"]
    for r in (0, 1):
        assert isinstance(res[r], list), res[r]
        (err, result, text, logs), = res[r]
        assert err is None
        assert logs == g["log"][N_LOAD_LINES:]
        for k, v in g["result"].items():
            assert result[k] == v, k
        assert text == g["str"]


SEVENTEEN = ["chords80", "sweep30", "sweep30_nc_tail_quiet"] + \
    [("syn", float(s), 1100 + i) for i, s in enumerate((180, 90, 200, 120, 180, 150, 95, 180, 130, 175, 110, 160, 180,
                                                        140))]


def test_sharded_four_ranks_seventeen_pairs_equal_engine(eng):
    """four ranks (gloo) on the one GPU, split pairs at every block
    boundary; all 17 outcomes equal Engine.analyze of the batch, field for field."""
    from nightcore_analyzer.sharded import shard_plan
    pairs = _batch(SEVENTEEN)
    sp = shard_plan([len(a) for pr in pairs for a in pr], E.Params(), 4, 0.45)
    assert sp.split.sum() == 3 and len(set(sp.owner.tolist())) == 4
    ref = [_key(o) for o in eng.analyze(pairs, E.Params())]
    res = _spawn(4, SEVENTEEN, split_offset=0.45, full=True, timeout=110)
    for r in range(4):
        assert isinstance(res[r], list), res[r]
        assert len(res[r]) == len(ref)
        for i, (a, b) in enumerate(zip(res[r], ref)):
            assert _norm(list(a)) == _norm(list(b)), (r, i)


def test_split_ibi_onsets_with_loud_tail_equal_one_gpu(eng):
    """the share that ends a file computes mel rows T - 16 .. T - 1 too
    (csrc/ibi.hip ibi_range_plan_kernel), so the all-reduced dB maximum (C2) and the onsets
    split over 1..4 ranks equal the one-GPU onsets bit for bit on a file whose loudest frame
    is in its last 14 ms."""
    from nightcore_analyzer.engine import _Upload
    from nightcore_analyzer.sharded import DeviceStages, _ibi_share
    from test_sharded_cpu import _loud_tail_signal
    y = _loud_tail_signal()
    n = len(y)
    T = 1 + n // 64
    sig = eng.upload_signals([y])
    up = _Upload()
    up.add("off", sig.off, np.int64)
    up.add("len", sig.length, np.int64)
    up.add("start", [120.0], np.float64)
    d = up.commit(eng.dev)
    core = eng.ibi_core(sig.buf, d["off"], d["len"], np.array([n], np.int64), d["start"],
                        torch.zeros(1, dtype=torch.int32, device=eng.dev))
    full = core["onset"][:T].cpu().numpy()
    st = DeviceStages(eng, sig)
    for world in (1, 2, 3, 4):
        shares = [_ibi_share(T, world, q) for q in range(world)]
        mx = max(float(st.ibi_mel(sig.off, sig.length, [s[2]], [s[3]])[0]) for s in shares)
        seg = []
        for s in shares:
            st.ibi_mel(sig.off, sig.length, [s[2]], [s[3]])
            seg.append(st.ibi_onset(np.array([mx], np.float32)))
        np.testing.assert_array_equal(np.concatenate(seg), full, err_msg=f"world {world}")
