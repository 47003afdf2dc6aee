"""16-bit PCM sources uploaded at their stored width: io.load_audio's
keep_pcm16 path returns the WAV's int16 samples (io.Pcm16), Engine.upload_signals copies the
2-byte samples host -> HBM and nc_pcm16_to_f32 widens them (k / 32768, exact), so every
result equals the float32 path's bit for bit (io.py:44-55: soundfile's scaling)."""
import struct

import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import io as nio
from nightcore_analyzer import pipeline, synth

pytestmark = pytest.mark.gpu


def _wav16(path, x: np.ndarray, sr: int = 22050):
    raw = x.astype("<i2").tobytes()
    fmt = struct.pack("<HHIIHH", 1, 1, sr, sr * 2, 2, 16)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(raw)) + raw
    path.write_bytes(b"RIFF" + struct.pack("<I", len(body)) + body)


def _pcm(y: np.ndarray) -> np.ndarray:
    return np.clip(np.round(y * 32768.0), -32768, 32767).astype(np.int16)


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


def test_pcm16_upload_equals_float_upload(eng):
    rng = np.random.default_rng(3)
    lens = [1, 7, 8, 9, 63, 64, 65, 1000, 22050 * 3 + 5]
    ints = [rng.integers(-32768, 32768, n).astype(np.int16) for n in lens]
    ints[-1][:3] = [-32768, 32767, 0]
    a = eng.upload_signals([x.view(nio.Pcm16) for x in ints])
    b = eng.upload_signals([x.astype(np.float32) / np.float32(32768.0) for x in ints])
    torch.cuda.synchronize()
    assert np.array_equal(a.off, b.off) and np.array_equal(a.length, b.length)
    assert a.buf.dtype == torch.float32 and torch.equal(a.buf.view(torch.int32), b.buf.view(torch.int32))


def test_run_on_16bit_wavs_equals_the_float_arrays(eng, tmp_path):
    """pipeline.run on two mono 16-bit WAVs (the int16 upload) against run on the float32
    arrays load_audio returns: the same AnalysisResult, report and log lines."""
    nc, src = synth.make_pair(45.0, 1011)
    fn, fs = tmp_path / "nc.wav", tmp_path / "src.wav"
    _wav16(fn, _pcm(nc))
    _wav16(fs, _pcm(src))
    y_nc, _ = nio.load_audio(str(fn))
    y_src, _ = nio.load_audio(str(fs))
    assert isinstance(nio.load_audio(str(fn), keep_pcm16=True)[0], nio.Pcm16)
    la, lb = [], []
    ra = pipeline.run(str(fn), str(fs), log=la.append)
    rb = pipeline.run(y_nc, y_src, log=lb.append)
    assert str(ra) == str(rb) and repr(ra) == repr(rb)
    assert la[4:] == lb[4:]                       # past the load lines (path vs array)
    assert [l for l in la[:4] if "samples" in l] == [l for l in lb[:4] if "samples" in l]
