"""GPU parity: CQT chroma (tuning -> 7-octave CQT -> 12-bin chroma mean) and the
cyclic cross-correlation lag against oracle/ncref.py on the same chunks."""
import numpy as np
import pytest
import torch

from oracle import ncref, refglue
from nightcore_analyzer import _dev, synth

pytestmark = pytest.mark.gpu


def _chroma_gpu(ctx, sig, chunks):
    dev = _dev.device(0)
    d_sig = _dev.to_dev(sig, dev, np.float32)
    off = np.array([c[0] for c in chunks], np.int64)
    ln = np.array([c[1] for c in chunks], np.int64)
    n = len(chunks)
    d_off, d_len = _dev.to_dev(off, dev), _dev.to_dev(ln, dev)
    out = _dev.empty(n * 12, torch.float32, dev)
    tun = _dev.empty(n, torch.float32, dev)
    tidx = _dev.empty(n, torch.int32, dev)
    wsb = ctx.lib.nc_chroma_workspace_bytes(ctx.h, n, int(ln.sum()))
    ws = _dev.workspace(wsb, dev)
    ctx.call("nc_chroma_mean", d_sig.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, int(ln.sum()),
             int(ln.max()), out.data_ptr(), tun.data_ptr(), tidx.data_ptr(), ws.data_ptr(), wsb,
             _dev.stream_handle())
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(n, 12), tun.cpu().numpy(), out, tidx.cpu().numpy()


def test_decimator_matches_oracle_response():
    """The half-band replacement for soxr_hq: flat to the top CQT filter, >= 100 dB stopband."""
    import scipy.signal
    h = ncref.halfband_taps()
    w, H = scipy.signal.freqz(h, worN=8192, fs=1.0)
    Hdb = 20 * np.log10(np.maximum(np.abs(H), 1e-300))
    assert np.max(np.abs(np.abs(H[w <= 0.11]) - 1.0)) < 1e-4
    assert np.max(Hdb[w >= 0.33]) < -100.0


@pytest.mark.parametrize("seed", [1001, 1005])
def test_chroma_mean_and_tuning_match_oracle(gpu_ctx, seed):
    nc, src = synth.make_pair(45.0, seed)
    cn = 441000
    sig = np.concatenate([src, nc]).astype(np.float32)
    chunks = [(0, cn), (cn, cn), (len(src), cn), (len(src) + cn, 7 * 22050 + 123)]
    got, tun, _, _ = _chroma_gpu(gpu_ctx, sig, chunks)
    for i, (o, L) in enumerate(chunks):
        y = sig[o:o + L]
        ref_t = ncref.estimate_tuning(y, 22050, bins_per_octave=36)
        assert abs(tun[i] - ref_t) <= 0.0100001, (i, tun[i], ref_t)
        ref_c = ncref.chroma_cqt(y, 22050, 512, 36, tuning=float(tun[i])).mean(axis=1)
        np.testing.assert_allclose(got[i], ref_c, rtol=0, atol=2e-5)


def test_chroma_ragged_chunks_across_decimator_tiles(gpu_ctx):
    """The fused octave chain (cqt.hip decimate3_kernel) owns 2048 level-0 samples per tile:
    chunk lengths one sample either side of a tile edge and at odd offsets (no aligned
    float4 path) must give the oracle's chroma like the 20 s chunks do."""
    nc, src = synth.make_pair(30.0, 1003)
    sig = np.concatenate([src, nc]).astype(np.float32)
    chunks = [(1, 2048 * 40 + 1), (3, 2048 * 41 - 1), (len(src) + 5, 2048 * 64), (len(src) + 2, 2048 * 48 + 2047)]
    got, tun, _, _ = _chroma_gpu(gpu_ctx, sig, chunks)
    for i, (o, L) in enumerate(chunks):
        y = sig[o:o + L]
        ref_c = ncref.chroma_cqt(y, 22050, 512, 36, tuning=float(tun[i])).mean(axis=1)
        np.testing.assert_allclose(got[i], ref_c, rtol=0, atol=2e-5, err_msg=f"chunk {i} len {L}")


def test_chunk_lags_match_reference_glue(gpu_ctx):
    nc, src = synth.make_pair(65.0, 1001)
    plan = refglue.chunk_plan(len(src), len(nc))
    sig = np.concatenate([src, nc]).astype(np.float32)
    chunks = []
    for a, b, c, d in plan:
        chunks += [(a, b - a), (len(src) + c, d - c)]
    _, _, d_chroma, _ = _chroma_gpu(gpu_ctx, sig, chunks)
    n = len(plan)
    dev = _dev.device(0)
    si = _dev.to_dev(np.arange(0, 2 * n, 2, dtype=np.int32), dev)
    ni = _dev.to_dev(np.arange(1, 2 * n, 2, dtype=np.int32), dev)
    lag = _dev.empty(n, torch.int32, dev)
    gpu_ctx.call("nc_chroma_lag", d_chroma.data_ptr(), si.data_ptr(), ni.data_ptr(), n, lag.data_ptr(),
                 _dev.stream_handle())
    torch.cuda.synchronize()
    ref = [refglue.chunk_lag(src[a:b], nc[c:d]) for a, b, c, d in plan]
    assert lag.cpu().numpy().tolist() == ref
    assert ref == [4] * n            # 1.25x speed-up -> +4 chroma bins (the lag/3 quirk)


def test_cyclic_xcorr_peak_golden(gpu_ctx, golden_units):
    cases = golden_units["cyclic_xcorr_peak"]
    dev = _dev.device(0)
    ch = np.array([c["src"] for c in cases] + [c["nc"] for c in cases], np.float32)
    n = len(cases)
    d = _dev.to_dev(ch.reshape(-1), dev)
    si = _dev.to_dev(np.arange(n, dtype=np.int32), dev)
    ni = _dev.to_dev(np.arange(n, 2 * n, dtype=np.int32), dev)
    lag = _dev.empty(n, torch.int32, dev)
    gpu_ctx.call("nc_chroma_lag", d.data_ptr(), si.data_ptr(), ni.data_ptr(), n, lag.data_ptr(),
                 _dev.stream_handle())
    torch.cuda.synchronize()
    assert lag.cpu().numpy().tolist() == [c["lag"] for c in cases]
