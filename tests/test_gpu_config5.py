"""GPU parity at BASELINE config 5: one 60-minute pair (src 3600 s, seed 5000,
nc = resample_poly(src, 4, 5); the pair bench.py times), against the committed
oracle fixtures of tests/golden/make_config5.py.

* run() analysis through the engine, IBI pass included: window counts, every
  per-window tempo, the nc prior, every 20 s chunk lag and the consensus ratios
  and CIs, exactly (pipeline.py:23-216);
* the hop-64 IBI pass (tempo.py:120-173): tempo lag and every beat frame of both
  files exactly, IBI ratio and bootstrap CI exactly (consensus.py:270-312);
* xcorr.estimate_speed_xcorr's search of src against nc (xcorr.py:95-162):
  slope within 1e-9, quality within 1e-5 (f64 device dots against numpy's f32 BLAS).
"""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import io as nio
from nightcore_analyzer import synth, xcorr

pytestmark = pytest.mark.gpu

FIX = Path(__file__).resolve().parent / "golden" / "config5.json"


@pytest.fixture(scope="module")
def case():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = json.loads(FIX.read_text())
    nc, src = synth.make_pair(g["seconds"], g["seed"])
    assert len(nc) == g["nc_raw_len"] and len(src) == g["src_raw_len"]
    return g, nc, src


@pytest.fixture(scope="module")
def outcome(case):
    g, nc, src = case
    o, = E.get_engine(0).analyze([(nc, src)], E.Params(ibi_beats=True))
    assert o.error is None, o.error
    return o


def test_config5_windows_and_consensus(case, outcome):
    g, _, _ = case
    r, d = outcome.result, outcome.detail
    assert (d["n_src_windows"], d["n_nc_windows"]) == (g["n_src_windows"], g["n_nc_windows"])
    assert r.src_duration * 22050 == g["src_len"] and r.nc_duration * 22050 == g["nc_len"]
    assert r.src_tempos_raw == g["src_tempos"]
    assert r.nc_tempos_raw == g["nc_tempos"]
    assert d["nc_start_bpm"] == g["nc_start_bpm"]
    assert d["chunk_lags"] == g["chunk_lags"]
    assert r.tempo_ratio == g["tempo_ratio"] and list(r.tempo_ci) == g["tempo_ci"]
    assert r.pitch_ratio == g["pitch_ratio"] and list(r.pitch_ci) == g["pitch_ci"]
    assert r.classification == g["classification"]


def test_config5_ibi_beat_frames(case, outcome):
    g, _, _ = case
    d, r = outcome.detail, outcome.result
    nc_b, src_b = d["ibi_beats"]
    assert d["ibi_lag"] == (g["ibi"]["nc"]["lag"], g["ibi"]["src"]["lag"])
    np.testing.assert_array_equal(src_b, g["ibi"]["src"]["beats"])
    np.testing.assert_array_equal(nc_b, g["ibi"]["nc"]["beats"])
    assert d["ibi_n"] == (g["ibi"]["nc"]["n_ibis"], g["ibi"]["src"]["n_ibis"])
    assert r.ibi_ratio == g["ibi"]["ratio"] and list(r.ibi_ci) == g["ibi"]["ci"]
    assert abs(r.ibi_ratio - 1.25) < 0.01


def test_config5_waveform_xcorr(case):
    g, nc, src = case
    nc_t, _, _ = nio.strip_silence(nc, 22050)
    src_t, _, _ = nio.strip_silence(src, 22050)
    ratio, quality = xcorr.estimate_speed_xcorr_arrays(src_t, nc_t)
    assert abs(ratio - g["xcorr"]["ratio"]) < 1e-9
    assert abs(quality - g["xcorr"]["quality"]) < 1e-5


def _shard_worker(rank, world, port, path, q):
    import os
    import torch.distributed as dist
    from nightcore_analyzer.sharded import run_window_sharded, shard_plan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = np.load(path)
        nc, src = d["nc"], d["src"]
        sp = shard_plan([len(nc), len(src)], E.Params(), world)
        outs = run_window_sharded([(nc, src)], E.Params(), device=0)
        o = outs[0]
        q.put((rank, bool(sp.split[0]), None if o.error is None else repr(o.error),
               None if o.result is None else (o.result.src_tempos_raw, o.result.nc_tempos_raw, o.result.tempo_ratio,
                                              list(o.result.tempo_ci), o.result.pitch_ratio, o.result.ibi_ratio,
                                              list(o.result.ibi_ci)),
               {k: o.detail.get(k) for k in ("chunk_lags", "ibi_lag", "ibi_n", "nc_start_bpm")}))
    except Exception as exc:          # noqa: BLE001
        q.put((rank, None, repr(exc), None, None))
    finally:
        dist.destroy_process_group()


def test_config5_window_sharded_two_ranks(case, tmp_path):
    """The 60-min pair split over two ranks (gloo on the one GPU): its windows and chunk
    pairs by the item plan, its hop-64 IBI pass by frames (C2 all-reduce MAX of the dB
    reference, C4 gather of the onset segments, C3 gather of the tempogram tile rows, beat
    tracking on the owner); every rank's result equals the fixtures, IBI ratio and CI exactly
    (the same IBIs as one GPU: every tile row is the one-GPU row, summed in the same order)."""
    import socket
    import torch.multiprocessing as mp
    g, nc, src = case
    path = tmp_path / "pair.npz"
    np.savez(path, nc=nc, src=src)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, str(path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=140) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, split, err, r, d in res:
        assert err is None, (rank, err)
        assert split, "the single pair must be split over the ranks"
        src_t, nc_t, tr, tci, pr, ir, ici = r
        assert src_t == g["src_tempos"] and nc_t == g["nc_tempos"]
        assert tr == g["tempo_ratio"] and tci == g["tempo_ci"] and pr == g["pitch_ratio"]
        assert d["chunk_lags"] == g["chunk_lags"] and d["nc_start_bpm"] == g["nc_start_bpm"]
        assert d["ibi_lag"] == (g["ibi"]["nc"]["lag"], g["ibi"]["src"]["lag"])
        assert d["ibi_n"] == (g["ibi"]["nc"]["n_ibis"], g["ibi"]["src"]["n_ibis"])
        assert ir == g["ibi"]["ratio"] and ici == g["ibi"]["ci"]
