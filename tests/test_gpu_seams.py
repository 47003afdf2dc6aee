"""GPU side of the drop-in seams: pitch._cyclic_xcorr_peak for any vector length
(pitch.py:67-85, nc_xcorr_peak) against a numpy restatement of the reference's loop,
and the engine lifetime across the sequential analysis threads of the reference's GUI
(gui/worker.py:16-56: one QThread per analysis)."""
import threading

import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import pipeline, pitch, synth

pytestmark = pytest.mark.gpu


def _ref_peak(a, b):
    """pitch.py:76-85 restated: f32 dot products (one f32 FMA chain in j order; the f32 x f32
    product is exact in f64, so the f64 sum rounded to f32 is the FMA barring a double
    rounding tie), first argmax."""
    n = len(a)
    xc = []
    for k in range(n):
        d = np.float32(0.0)
        r = np.roll(b, -k)
        for j in range(n):
            d = np.float32(np.float64(a[j]) * np.float64(r[j]) + np.float64(d))
        xc.append(d)
    lag = int(np.argmax(np.array(xc, np.float32)))
    return lag - n if lag > n // 2 else lag


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


@pytest.mark.parametrize("n", [1, 2, 3, 7, 12, 36, 37, 300, 1000])
def test_cyclic_xcorr_peak_any_length(eng, n):
    rng = np.random.default_rng(n)
    for t in range(6):
        a = rng.random(n).astype(np.float32)
        b = np.roll(a, rng.integers(n)) + np.float32(0.01) * rng.random(n).astype(np.float32) if t % 2 else \
            rng.random(n).astype(np.float32)
        b = b.astype(np.float32)
        assert pitch._cyclic_xcorr_peak(a, b) == _ref_peak(a, b), (n, t)


def test_cyclic_xcorr_peak_ties_and_nan(eng):
    a = np.ones(12, np.float32)
    assert pitch._cyclic_xcorr_peak(a, a) == 0                   # all lags tie: the first (k = 0)
    b = np.zeros(12, np.float32)
    b[5] = np.nan
    assert pitch._cyclic_xcorr_peak(a, b) == 0                   # every xcorr is NaN: np.argmax -> 0
    a2 = np.zeros(12, np.float32)
    a2[3] = 1.0
    b2 = np.zeros(12, np.float32)
    b2[10] = 1.0                                                  # peak at k = 7 -> wrapped to -5
    assert pitch._cyclic_xcorr_peak(a2, b2) == _ref_peak(a2, b2) == -5


def test_engine_released_with_its_thread():
    """pipeline.run from 20 sequential threads: one engine per live thread, released when
    the thread ends; HBM reserved by the caching allocator stays flat."""
    nc, src = synth.make_pair(40.0, 1003)
    reserved, live, errs = [], [], []
    base = E.live_engines()                            # other tests' engines on this (main) thread

    def work():
        try:
            pipeline.run(nc, src, log=None)
        except BaseException as exc:                 # noqa: BLE001 - reported below
            errs.append(exc)

    for i in range(20):
        t = threading.Thread(target=work)
        t.start()
        t.join()
        torch.cuda.synchronize()
        reserved.append(torch.cuda.memory_reserved())
        live.append(E.live_engines())
    assert not errs, errs[0]
    assert max(live) == base, (base, live)             # each thread's engine went with its thread
    assert reserved[-1] <= reserved[2], reserved      # flat after the first threads warmed the allocator


# ---- tempo seams at other sample rates: the reference passes sr through to
# librosa (tempo.py:44-50, 139-164); an engine whose mel bank and tempogram windows are built for
# the rate (nc_create_rate) equals the oracle at that rate, with no resampling
def _at(sr, seconds, seed):
    import scipy.signal
    src = synth.make_source(seconds, seed)
    from math import gcd
    g = gcd(sr, 22050)
    return scipy.signal.resample_poly(src, sr // g, 22050 // g).astype(np.float32)


@pytest.mark.parametrize("sr", [44100, 48000, 16000])
def test_estimate_tempo_at_other_rates_equals_oracle(eng, sr):
    from nightcore_analyzer import io as nio, tempo
    from oracle import refglue
    y = _at(sr, 40.0, 1012)
    wins = [nio.AudioWindow(audio=y[s:s + 10 * sr], sample_rate=sr, start_sec=s / sr, end_sec=s / sr + 10.0,
                            energy_db=0.0) for s in range(0, len(y) - 10 * sr + 1, 5 * sr)]
    for bpm in (120.0, 150.0):
        got = [tempo.estimate_tempo(w, start_bpm=bpm) for w in wins]
        ref = [refglue.estimate_tempo(w.audio, sr, bpm) for w in wins]
        assert got == ref, (sr, bpm, got, ref)
    # one call over windows of two rates: each rate on its own engine, in the caller's order
    mixed = wins[:2] + [nio.AudioWindow(audio=_at(22050, 10.0, 1013), sample_rate=22050, start_sec=0.0,
                                        end_sec=10.0, energy_db=0.0)]
    got = tempo.batch_estimate_tempo(mixed, start_bpm=120.0)
    assert got == [refglue.estimate_tempo(w.audio, w.sample_rate, 120.0) for w in mixed]
    assert E.get_engine(sr=sr) is not E.get_engine() and E.get_engine(sr=sr).sr == sr


@pytest.mark.parametrize("sr,hop", [(16000, 64), (48000, 512)])
def test_ibis_at_other_rates_equal_oracle(eng, sr, hop):
    """The IBI pass (tempo.py:120-173) at 16 kHz hop 64 and 48 kHz hop 512; 44.1 kHz raises
    ValueError: at hop 64 its 5 512-frame tempogram window exceeds the beat tracker's LDS ring,
    at hop 512 the 689-frame window is odd (the streamed tempogram pairs lags)."""
    from nightcore_analyzer import tempo
    from oracle import refglue
    y = _at(sr, 20.0, 1014)
    got = tempo.estimate_ibis_global(y, sr, hop_length=hop, start_bpm=120.0)
    ref = refglue.estimate_ibis_global(y, sr, hop_length=hop, start_bpm=120.0)
    assert (got is None) == (ref is None)
    if ref is not None:
        assert len(got) == len(ref) and np.array_equal(got, ref)
    y44 = _at(44100, 12.0, 1015)
    with pytest.raises(ValueError, match="use hop_length=512"):
        tempo.estimate_ibis_global(y44, 44100, hop_length=64)
    with pytest.raises(ValueError, match="689 frames"):
        tempo.estimate_ibis_global(y44, 44100, hop_length=512)


def test_chroma_needs_the_22k_context(eng):
    from nightcore_analyzer import ops, _native
    e44 = E.get_engine(sr=44100)
    with pytest.raises(_native.NativeError, match="22050"):
        ops.chroma_means(e44, [np.zeros(441000, np.float32)])
