"""GPU parity: CQT chroma (tuning -> 7-octave CQT -> 12-bin chroma mean) and the
cyclic cross-correlation lag against oracle/ncref.py on the same chunks.

The tuning is an index decision (the argmax of a 100-bin residual histogram): every
chunk's tuning index and its decision margin (argmax count minus the runner-up's) must
equal the oracle's, and the chroma is compared at the ORACLE's tuning, so a flipped
tuning decision cannot hide behind a self-consistent chroma."""
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
    tmg = _dev.empty(n, torch.int32, dev)
    wsb = ctx.lib.nc_chroma_workspace_bytes(ctx.h, n, int(ln.sum()))
    ws = _dev.workspace(wsb, dev)
    ctx.call("nc_chroma_mean", d_sig.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, int(ln.sum()),
             int(ln.max()), out.data_ptr(), tun.data_ptr(), tidx.data_ptr(), tmg.data_ptr(), ws.data_ptr(), wsb,
             _dev.stream_handle())
    torch.cuda.synchronize()
    _chroma_gpu.margin = tmg.cpu().numpy()
    return out.cpu().numpy().reshape(n, 12), tun.cpu().numpy(), out, tidx.cpu().numpy()


def _check_tuning(i, y, tidx, margin):
    """The chunk's tuning decision equals the oracle's (the index exactly); its margin (the
    argmax bin's count minus the runner-up's) agrees to a peak or two -- a single piptrack
    peak whose f32 residual lands one bin over moves a count by one without moving the
    decision.  Returns the oracle's tuning, at which the chroma is then compared."""
    ref_t, ref_i, ref_m = ncref.estimate_tuning_detail(y, 22050, bins_per_octave=36)
    assert int(tidx[i]) == ref_i, ("tuning index", i, int(tidx[i]), ref_i, int(margin[i]), ref_m)
    assert abs(int(margin[i]) - ref_m) <= max(2, ref_m // 50), ("tuning margin", i, int(margin[i]), ref_m)
    return ref_t


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
    got, tun, _, tidx = _chroma_gpu(gpu_ctx, sig, chunks)
    mg = _chroma_gpu.margin
    for i, (o, L) in enumerate(chunks):
        y = sig[o:o + L]
        ref_t = _check_tuning(i, y, tidx, mg)
        assert tun[i] == np.float32(ref_t), (i, tun[i], ref_t)
        ref_c = ncref.chroma_cqt(y, 22050, 512, 36, tuning=ref_t).mean(axis=1)
        np.testing.assert_allclose(got[i], ref_c, rtol=0, atol=2e-5)


def dense_peak_chunk(n=441000, seed=7):
    """32 tones a semitone apart between 600 and 3 900 Hz, all 0.3 of a 36-per-octave bin
    off the A440 grid, in white noise: 58-91 piptrack peaks per frame (median 80), so the
    peak compaction of nc_piptrack.h takes more than one 64-peak pass on nearly every frame,
    while the common detuning keeps the tuning decision far from a tie (oracle margin 166)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 22050
    y = np.zeros(n)
    for m in range(0, 400, 3):
        f = 27.5 * 2 ** ((m + 0.3) / 36)
        if 600 <= f <= 3900:
            y += 0.03 * np.sin(2 * np.pi * f * t + rng.uniform(0, 6.28))
    return (y + rng.normal(0, 0.08, n)).astype(np.float32)


def test_tuning_with_more_than_64_peaks_per_frame(gpu_ctx):
    y = dense_peak_chunk()
    p, _ = ncref.piptrack(y)
    assert np.median((p > 0).sum(axis=0)) > 64
    got, tun, _, tidx = _chroma_gpu(gpu_ctx, y, [(0, len(y))])
    ref_t = _check_tuning(0, y, tidx, _chroma_gpu.margin)
    assert tun[0] == np.float32(ref_t), (tun[0], ref_t)
    ref_c = ncref.chroma_cqt(y, 22050, 512, 36, tuning=ref_t).mean(axis=1)
    np.testing.assert_allclose(got[0], ref_c, rtol=0, atol=2e-5)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_chroma_independent_of_chunk_alignment(gpu_ctx, shift):
    """Chunks at any sample offset (a trimmed file starts anywhere): the tuning frames load
    odd-offset pairs as two dwords, the low-octave CQT stages unaligned blocks through
    registers instead of the 16-byte LDS-DMA.  Same samples, same arithmetic: tuning and
    chroma bit-identical to the aligned chunks."""
    nc, src = synth.make_pair(45.0, 1001)
    cn = 441000
    sig = np.concatenate([src, nc]).astype(np.float32)
    chunks = [(0, cn), (len(src), cn), (len(src) + 3, cn - 7)]
    ref, rtun, _, ridx = _chroma_gpu(gpu_ctx, sig, chunks)
    sig2 = np.concatenate([np.zeros(shift, np.float32), sig])
    got, tun, _, tidx = _chroma_gpu(gpu_ctx, sig2, [(o + shift, L) for o, L in chunks])
    assert np.array_equal(tidx, ridx) and np.array_equal(tun, rtun)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("scale", [3e-7, 1e-3, 40.0, 3e4])
def test_chroma_f16_split_scaling_across_amplitudes(gpu_ctx, scale):
    """Octaves 3-6 run on the f16 matrix cores with hi/lo split operands at a per-chunk
    power-of-two scale (cqt.hip cqt_mfma_kernel, decimate3's per-tile maxima): the chroma
    must follow the oracle from quiet (-130 dB) to loud (+90 dB) chunks, and a chunk shorter
    than one 64-frame tile.  A chunk whose first half is digital silence is checked for scale
    invariance (power-of-two scaling: the GPU result at scale s equals the one at scale 1 to
    f32 rounding) and against the oracle at 2e-3 only: its frames at the silence boundary
    are ill-conditioned (a few edge samples projected on filters whose taps are ~0 there),
    where any two f32 implementations differ by ~1e-3 in the mean -- the FFT-only build
    (NC_CQ_MFMA=0) measured 7e-4 .. 1.2e-3 against the oracle on the same chunk."""
    nc, src = synth.make_pair(30.0, 1007)
    base = src[:441000].astype(np.float32)

    def run(sc):
        y = (base * sc).astype(np.float32)
        half = y.copy()
        half[:220500] = 0.0
        sig = np.concatenate([y, half, y[:25000]]).astype(np.float32)
        chunks = [(0, 441000), (441000, 441000), (882000, 25000)]
        got, tun, _, tidx = _chroma_gpu(gpu_ctx, sig, chunks)
        return sig, chunks, got, tidx

    sig, chunks, got, tidx = run(scale)
    mg = _chroma_gpu.margin
    for i, (o, L) in enumerate(chunks):
        yy = sig[o:o + L]
        ref_t = _check_tuning(i, yy, tidx, mg)
        ref_c = ncref.chroma_cqt(yy, 22050, 512, 36, tuning=ref_t).mean(axis=1)
        tol = 2e-3 if i == 1 else 2e-5
        np.testing.assert_allclose(got[i], ref_c, rtol=0, atol=tol, err_msg=f"scale {scale} chunk {i}")
    if scale >= 1e-3:  # far from f32 subnormals
        _, _, got1, _ = run(1.0)
        np.testing.assert_allclose(got[1], got1[1], rtol=0, atol=1e-5)


def test_chroma_is_deterministic_across_workspace_contents(gpu_ctx):
    """The CQT kernels stream operands by LDS-DMA with hand-counted waits (cqt.hip): a wait
    that retires the wrong DMA reads stale LDS and shows up as run-to-run differences (a
    counted vmcnt over mixed slice/block DMAs did, up to 2e-3).  Same chunks, workspaces
    pre-filled with different bytes, results must be bit-identical."""
    nc, src = synth.make_pair(60.0, 1011)
    sig = np.concatenate([src, nc]).astype(np.float32)
    chunks = [(i * 441000 // 2, 441000) for i in range(4)] + [(len(src) + 17, 441000), (len(src), 300000)]
    dev = _dev.device(0)
    d_sig = _dev.to_dev(sig, dev, np.float32)
    off = np.array([c[0] for c in chunks], np.int64)
    ln = np.array([c[1] for c in chunks], np.int64)
    n = len(chunks)
    d_off, d_len = _dev.to_dev(off, dev), _dev.to_dev(ln, dev)
    wsb = gpu_ctx.lib.nc_chroma_workspace_bytes(gpu_ctx.h, n, int(ln.sum()))
    outs = []
    for fill in (0x00, 0x7f, 0xff, 0x3c):
        ws = torch.full((wsb,), fill, dtype=torch.uint8, device=dev)
        out = torch.full((n * 12,), float("nan"), dtype=torch.float32, device=dev)
        tun = _dev.empty(n, torch.float32, dev)
        gpu_ctx.call("nc_chroma_mean", d_sig.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n, int(ln.sum()),
                     int(ln.max()), out.data_ptr(), tun.data_ptr(), None, None, ws.data_ptr(), wsb,
                     _dev.stream_handle())
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])
    assert not np.isnan(outs[0]).any()


def test_chroma_silent_chunk_is_zero(gpu_ctx):
    """All-zero chunk: decimate3's maximum is 0, the f16 scale stays 2^0 and every chroma is 0
    (librosa's inf-norm leaves an all-zero frame at zero)."""
    sig = np.zeros(441000, np.float32)
    got, _, _, _ = _chroma_gpu(gpu_ctx, sig, [(0, 441000)])
    assert np.all(got == 0.0)


def test_chroma_ragged_chunks_across_decimator_tiles(gpu_ctx):
    """The fused octave chain (cqt.hip decimate3_kernel) owns 2048 level-0 samples per tile:
    chunk lengths one sample either side of a tile edge and at odd offsets (no aligned
    float4 path) must give the oracle's chroma like the 20 s chunks do."""
    nc, src = synth.make_pair(30.0, 1003)
    sig = np.concatenate([src, nc]).astype(np.float32)
    chunks = [(1, 2048 * 40 + 1), (3, 2048 * 41 - 1), (len(src) + 5, 2048 * 64), (len(src) + 2, 2048 * 48 + 2047)]
    got, tun, _, tidx = _chroma_gpu(gpu_ctx, sig, chunks)
    mg = _chroma_gpu.margin
    for i, (o, L) in enumerate(chunks):
        y = sig[o:o + L]
        ref_t = _check_tuning(i, y, tidx, mg)
        ref_c = ncref.chroma_cqt(y, 22050, 512, 36, tuning=ref_t).mean(axis=1)
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


def _edit_pairs():
    """(name, src chunk, nc chunk) pairs of 20 s chunks with internal silence and fades:
    the regime where the f16-split CQT and the oracle's complex64 CQT differ most (frames
    next to digital silence are ill-conditioned, see test_chroma_f16_split_scaling)."""
    nc, src = synth.make_pair(100.0, 1013)
    cn = 441000
    out = []
    for k, (name, how) in enumerate((("gap", "gap"), ("fade_in", "fin"), ("fade_out", "fout"),
                                     ("half_silent", "half"), ("both_faded", "both"))):
        s = src[k * cn // 2:k * cn // 2 + cn].copy()
        n = nc[k * cn // 2:k * cn // 2 + cn].copy()
        ramp = np.linspace(0.0, 1.0, 8 * 22050, dtype=np.float32)
        if how == "gap":                     # 3 s of digital silence inside both chunks
            s[150000:216150] = 0.0
            n[200000:266150] = 0.0
        elif how == "fin":
            s[:len(ramp)] *= ramp
            n[:len(ramp)] *= ramp ** 2
        elif how == "fout":
            s[-len(ramp):] *= ramp[::-1]
            n[-len(ramp):] *= ramp[::-1] ** 3
        elif how == "half":
            s[:cn // 2] = 0.0
        else:
            s[:len(ramp)] *= ramp
            s[-len(ramp):] *= ramp[::-1]
            n[:cn // 3] = 0.0
        out.append((name, s, n))
    return out


def test_chunk_lags_with_silence_and_fades_match_oracle(gpu_ctx):
    """chunk-lag (and tuning-index) equality against the oracle on chunk
    pairs with internal silence, fade-ins and fade-outs."""
    pairs = _edit_pairs()
    sig = np.concatenate([a for _, s, n in pairs for a in (s, n)]).astype(np.float32)
    chunks = [(i * 441000, 441000) for i in range(2 * len(pairs))]
    _, _, d_chroma, tidx = _chroma_gpu(gpu_ctx, sig, chunks)
    mg = _chroma_gpu.margin
    n = len(pairs)
    dev = _dev.device(0)
    si = _dev.to_dev(np.arange(0, 2 * n, 2, dtype=np.int32), dev)
    ni = _dev.to_dev(np.arange(1, 2 * n, 2, dtype=np.int32), dev)
    lag = _dev.empty(n, torch.int32, dev)
    margin = _dev.empty(n, torch.float64, dev)
    gpu_ctx.call("nc_chroma_lag_margin", d_chroma.data_ptr(), si.data_ptr(), ni.data_ptr(), n, lag.data_ptr(),
                 margin.data_ptr(), _dev.stream_handle())
    torch.cuda.synchronize()
    got = lag.cpu().numpy().tolist()
    for i, (name, s, nn) in enumerate(pairs):
        for j, y in ((2 * i, s), (2 * i + 1, nn)):
            _check_tuning(j, y, tidx, mg)
        assert got[i] == refglue.chunk_lag(s, nn), (name, got[i], float(margin.cpu()[i]))
