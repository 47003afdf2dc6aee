"""GPU load-time resampler (io.py:44-55 -> nc_resample_poly) against
scipy.signal.resample_poly — bit-identical f32 outputs (the CPU tests pin the term
order to scipy itself, tests/test_resample_cpu.py) — and through io.load_audio."""
import wave

import numpy as np
import pytest
import scipy.signal
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import io as nio
from nightcore_analyzer import ops, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


@pytest.mark.parametrize("up,down", [(1, 2), (147, 320), (147, 160), (2, 1), (4, 5), (441, 480)])
def test_resample_bit_identical_to_scipy(eng, up, down):
    rng = np.random.default_rng(up * 1000 + down)
    arrays = [rng.standard_normal(n).astype(np.float32) for n in (1, 7, 513, 44_100, 300_007)]
    got = ops.resample_poly(eng, arrays, up, down)
    for a, g in zip(arrays, got):
        want = scipy.signal.resample_poly(a.astype(np.float64), up, down).astype(np.float32)
        assert g.shape == want.shape
        assert np.array_equal(g, want)


def test_resample_full_size_3min_44k(eng):
    """A 3-min 44.1 kHz file (BASELINE config-2 length at the CD rate) -> 3 969 000 samples,
    bit-identical to scipy."""
    src = synth.make_source(180.0, 1234).astype(np.float64)
    x = scipy.signal.resample_poly(src, 2, 1).astype(np.float32)
    g, = ops.resample_poly(eng, [x], 1, 2)
    want = scipy.signal.resample_poly(x.astype(np.float64), 1, 2).astype(np.float32)
    assert len(g) == 3_969_000 and np.array_equal(g, want)


def test_load_audio_resamples_on_device(eng, tmp_path):
    src = synth.make_source(12.0, 77)
    x = scipy.signal.resample_poly(src.astype(np.float64), 320, 147)          # a 48 kHz file
    pcm = np.clip(np.round(x * 32767.0), -32768, 32767).astype("<i2")
    p = tmp_path / "a48k.wav"
    with wave.open(str(p), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(48000)
        w.writeframes(pcm.tobytes())
    y, sr = nio.load_audio(str(p))
    want = scipy.signal.resample_poly((pcm.astype(np.float32) / 32768.0).astype(np.float64), 147, 320)
    assert sr == 22050 and np.array_equal(y, want.astype(np.float32))
    y2, sr2 = nio.load_audio(str(p), sr=None)
    assert sr2 == 48000 and len(y2) == len(pcm)
