"""GPU parity: per-window stage (energy, onset envelope, tempogram mean) and the
tempo/beat tracker against the CPU oracle (oracle/ncref.py) on the same inputs."""
import numpy as np
import pytest
import torch

from oracle import ncref, refglue
from nightcore_analyzer import _dev, synth

pytestmark = pytest.mark.gpu


def _windows(y, win=220500, hop=110250):
    return [s for s in range(0, len(y) - win + 1, hop)]


def _run_window_stage(ctx, sig, offs, win_len=220500):
    dev = _dev.device(0)
    d_sig = _dev.to_dev(sig, dev, np.float32)
    d_off = _dev.to_dev(np.asarray(offs, np.int64), dev)
    n = len(offs)
    T = 1 + win_len // 512
    acw = ncref.ac_win_length(22050, 512)
    onset = _dev.empty(n * T, torch.float32, dev)
    tg = _dev.empty(n * acw, torch.float64, dev)
    en = _dev.empty(n, torch.float64, dev)
    wsb = ctx.lib.nc_window_stage_workspace_bytes(ctx.h, n, win_len, 512)
    ws = _dev.workspace(wsb, dev)
    ctx.call("nc_window_stage", d_sig.data_ptr(), d_off.data_ptr(), None, n, win_len, 512,
             onset.data_ptr(), tg.data_ptr(), en.data_ptr(), ws.data_ptr(), wsb,
             _dev.stream_handle())
    torch.cuda.synchronize()
    return (onset.cpu().numpy().reshape(n, T), tg.cpu().numpy().reshape(n, acw),
            en.cpu().numpy(), (d_sig, d_off))


def test_window_stage_matches_oracle(gpu_ctx):
    nc, src = synth.make_pair(40.0, 1001)
    offs = _windows(src)
    onset, tg, en, _ = _run_window_stage(gpu_ctx, src, offs)
    for i, o in enumerate(offs):
        w = src[o:o + 220500]
        ref_on = ncref.onset_strength(w, 22050, 512)
        ref_tg = ncref.tempogram_mean(ref_on, 344)
        assert abs(en[i] - refglue.rms_db(w)) < 1e-9
        # onset: f32 FFT vs librosa's f64 FFT -> ~1e-6 relative to the envelope peak
        assert np.max(np.abs(onset[i] - ref_on)) <= 1e-4 * max(1.0, np.max(ref_on))
        assert np.max(np.abs(tg[i] - ref_tg)) < 2e-5
        # the decision the reference makes from it: identical tempo lag
        assert ncref.tempo_from_tg(tg[i])[1] == ncref.tempo_from_tg(ref_tg)[1]


def _run_beats(ctx, onset, tg, start_bpm, hop=512):
    dev = _dev.device(0)
    n, T = onset.shape
    acw = tg.shape[1]
    d_on = _dev.to_dev(onset.reshape(-1), dev, np.float32)
    d_tg = _dev.to_dev(tg.reshape(-1), dev, np.float64)
    off = _dev.to_dev(np.arange(n, dtype=np.int64) * T, dev)
    ln = _dev.to_dev(np.full(n, T, np.int32), dev)
    sb = _dev.to_dev(np.asarray(start_bpm, np.float64), dev)
    bpm = _dev.empty(n, torch.float64, dev)
    lag = _dev.empty(n, torch.int32, dev)
    nb = _dev.empty(n, torch.int32, dev)
    mg = _dev.empty(n, torch.float64, dev)
    beats = _dev.empty(n * T, torch.int32, dev)
    total = n * T
    wsb = ctx.lib.nc_tempo_beats_workspace_bytes(total)
    ws = _dev.workspace(wsb, dev)
    ctx.call("nc_tempo_beats", d_on.data_ptr(), off.data_ptr(), ln.data_ptr(), n, T, d_tg.data_ptr(),
             acw, sb.data_ptr(), None, None, hop, 1, bpm.data_ptr(), lag.data_ptr(), nb.data_ptr(),
             mg.data_ptr(), beats.data_ptr(), total, ws.data_ptr(), wsb, _dev.stream_handle())
    torch.cuda.synchronize()
    b = beats.cpu().numpy().reshape(n, T)
    nbv = nb.cpu().numpy()
    return bpm.cpu().numpy(), lag.cpu().numpy(), nbv, [b[i, :max(0, nbv[i])] for i in range(n)]


@pytest.mark.parametrize("prior", [120.0, 153.80859375])
def test_beats_match_oracle_on_same_onset(gpu_ctx, prior):
    """Same onset + tempogram inputs -> bit-identical decisions (lag, beat frames)."""
    nc, src = synth.make_pair(40.0, 1002)
    sig = nc if prior > 140 else src
    ons, tgs = [], []
    for o in _windows(sig):
        on = ncref.onset_strength(sig[o:o + 220500], 22050, 512)
        ons.append(on)
        tgs.append(ncref.tempogram_mean(on, 344))
    ons, tgs = np.stack(ons), np.stack(tgs)
    bpm, lag, nb, beats = _run_beats(gpu_ctx, ons, tgs, [prior] * len(ons))
    for i in range(len(ons)):
        rb, rbeats = ncref.beat_track(ons[i], 22050, 512, prior, tg_mean=tgs[i])
        assert bpm[i] == rb
        assert nb[i] == len(rbeats)
        np.testing.assert_array_equal(beats[i], rbeats)


def test_full_window_tempo_matches_reference_glue(gpu_ctx):
    """GPU onset -> GPU beats vs refglue.estimate_tempo on the same windows."""
    nc, src = synth.make_pair(40.0, 1003)
    for sig, prior in ((src, 120.0), (nc, 123.046875 * 1.25)):
        offs = _windows(sig)
        onset, tg, en, _ = _run_window_stage(gpu_ctx, sig, offs)
        bpm, lag, nb, beats = _run_beats(gpu_ctx, onset, tg, [prior] * len(offs))
        for i, o in enumerate(offs):
            ref = refglue.estimate_tempo(sig[o:o + 220500], 22050, prior)
            got = float(bpm[i]) if nb[i] >= 4 else None
            assert got == ref


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_window_stage_independent_of_alignment(gpu_ctx, shift):
    """A trimmed file's windows start at any sample: at an odd offset the STFT loads its sample
    pairs as two dwords (stft.hip), otherwise as one 8-byte load.  Same samples, same
    arithmetic: onsets, tempogram means and energies are bit-identical to the aligned run."""
    nc, src = synth.make_pair(40.0, 1001)
    offs = _windows(src)
    ref = _run_window_stage(gpu_ctx, src, offs)
    sig = np.concatenate([np.zeros(shift, np.float32), src])
    got = _run_window_stage(gpu_ctx, sig, [o + shift for o in offs])
    for g, r in zip(got[:3], ref[:3]):
        assert np.array_equal(g, r)
