"""Multi-process (gloo, world_size 2, CPU) tests of the pair sharding and the
result gather used by bench.py / run_batch_distributed on N GPUs."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from nightcore_analyzer.distributed import shard_range


def test_shard_range_covers_exactly():
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, fail_rank=-1):
    import torch.distributed as dist
    from nightcore_analyzer.distributed import run_batch_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def fake_analyze(pairs, scale):   # stands in for the GPU engine
        if rank == fail_rank:
            raise ValueError(f"rank {rank} failed")
        return [("rank", rank, p * scale) for p in pairs]

    out = run_batch_distributed(list(range(7)), analyze_fn=fake_analyze, scale=10)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(fail_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, fail_rank)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_run_batch_distributed_gloo_world2():
    res = _spawn()
    expect = [("rank", 0 if i < 4 else 1, i * 10) for i in range(7)]
    assert res[0] == expect and res[1] == expect


def test_run_batch_distributed_failing_rank_delivers_its_exception():
    """A rank whose analysis raises still joins the result gather (no rank blocks): its
    pairs come back as the exception, the other rank's as results."""
    res = _spawn(fail_rank=1)
    for r in (0, 1):
        assert res[r][:4] == [("rank", 0, i * 10) for i in range(4)]
        assert all(isinstance(e, ValueError) and str(e) == "rank 1 failed" for e in res[r][4:])
        assert len(res[r]) == 7


def test_run_batch_distributed_rejects_unknown_arguments():
    from nightcore_analyzer.distributed import run_batch_distributed
    with pytest.raises(ValueError, match="shard must be"):
        run_batch_distributed([("a.wav", "b.wav")], shard="frames")
    with pytest.raises(TypeError, match="unexpected keyword"):
        run_batch_distributed([("a.wav", "b.wav")], shard="windows", windowsec=3.0)
    with pytest.raises(ValueError, match="pair mode only"):
        run_batch_distributed([("a.wav", "b.wav")], analyze_fn=len, shard="windows")


def _win_worker(rank, world, port, q, paths):
    import torch.distributed as dist
    from nightcore_analyzer.distributed import run_batch_distributed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = run_batch_distributed(paths, shard="windows", log=None)
        q.put((rank, [(type(e).__name__, str(e)) for e in out]))
    finally:
        dist.destroy_process_group()


def test_window_mode_run_failure_is_every_pairs_result(tmp_path):
    """Window mode: a file that does not decode (here on every rank, no device needed)
    comes back as each pair's result on every rank, not as an exception."""
    import numpy as np
    good = tmp_path / "ok.npy"
    np.save(good, np.zeros(22050 * 40, np.float32))
    paths = [(str(tmp_path / "missing.wav"), str(good)), (str(good), str(good)), (str(good), str(good))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_win_worker, args=(r, 2, port, q, paths)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    assert len(res[0]) == 3 and all(name == "FileNotFoundError" for name, _ in res[0])
