"""io._read_wav (the decode half of io.load_audio, io.py:44-55): PCM 8/16/24/32-bit and
IEEE float, plain and WAVE_FORMAT_EXTENSIBLE, scaled to [-1, 1) and down-mixed to mono
the way soundfile + librosa.load(mono=True) do.  Host code only."""
import struct

import numpy as np
import pytest
import scipy.io.wavfile

from nightcore_analyzer import io as nio


def _wav_bytes(samples_int: np.ndarray, bits: int, sr: int, extensible: bool, tag: int = 1) -> bytes:
    ch = samples_int.shape[1]
    width = bits // 8
    if bits == 24:
        v = samples_int.astype(np.int64) & 0xFFFFFF
        raw = np.stack([(v >> (8 * k)) & 0xFF for k in range(3)], axis=-1).astype(np.uint8).tobytes()
    else:
        raw = samples_int.astype({8: np.uint8, 16: "<i2", 32: "<i4"}[bits] if tag == 1 else "<f4").tobytes()
    if extensible:
        guid = struct.pack("<H", tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        fmt = struct.pack("<HHIIHHHHI", 0xFFFE, ch, sr, sr * ch * width, ch * width, bits, 22, bits, 3) + guid
    else:
        fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * ch * width, ch * width, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"LIST" + struct.pack("<I", 3) + b"abc\x00" \
        + b"data" + struct.pack("<I", len(raw)) + raw
    return b"RIFF" + struct.pack("<I", len(body)) + body


@pytest.mark.parametrize("extensible", [False, True])
@pytest.mark.parametrize("bits", [8, 16, 24, 32])
def test_pcm_wav_scaled_and_downmixed(tmp_path, bits, extensible):
    rng = np.random.default_rng(bits)
    full = 1 << (bits - 1)
    if bits == 8:
        x = rng.integers(0, 256, size=(1000, 2))
        expect = ((x.astype(np.float32) - 128.0) / 128.0).mean(axis=1)
    else:
        x = rng.integers(-full, full, size=(1000, 2))
        expect = (x.astype(np.float64) / full).astype(np.float32).mean(axis=1)
    p = tmp_path / "a.wav"
    p.write_bytes(_wav_bytes(x, bits, 44100, extensible))
    y, sr = nio._read_wav(p)
    assert sr == 44100 and y.dtype == np.float32
    np.testing.assert_allclose(y, expect.astype(np.float32), rtol=0, atol=1e-7)
    assert np.max(np.abs(y)) <= 1.0


@pytest.mark.parametrize("extensible", [False, True])
def test_float_wav(tmp_path, extensible):
    x = np.random.default_rng(0).standard_normal((500, 1)).astype(np.float32) * 0.3
    p = tmp_path / "f.wav"
    p.write_bytes(_wav_bytes(x, 32, 48000, extensible, tag=3))
    y, sr = nio._read_wav(p)
    assert sr == 48000
    np.testing.assert_array_equal(y, x[:, 0])


def test_scipy_written_wavs(tmp_path):
    x = (np.sin(np.arange(2000) * 0.05) * 0.5).astype(np.float32)
    for dt, scale in ((np.int16, 32767), (np.int32, 2 ** 31 - 1), (np.float32, 1.0)):
        p = tmp_path / f"s_{np.dtype(dt).name}.wav"
        scipy.io.wavfile.write(p, 22050, (x * scale).astype(dt))
        y, sr = nio._read_wav(p)
        assert sr == 22050
        np.testing.assert_allclose(y, x, atol=1e-4)


def test_not_a_wav(tmp_path):
    p = tmp_path / "x.wav"
    p.write_bytes(b"fLaC\x00\x00\x00\x22")
    with pytest.raises(ValueError):
        nio._read_wav(p)


@pytest.mark.parametrize("extensible", [False, True])
def test_keep_pcm16_returns_the_stored_samples(tmp_path, extensible):
    """load_audio(keep_pcm16=True) on a mono 16-bit WAV at the requested rate: the stored
    samples (io.Pcm16), whose float32 view is exactly what load_audio returns by default (the
    engine uploads the 2-byte samples and widens them on the device, nc_pcm16_to_f32)."""
    x = np.random.default_rng(7).integers(-32768, 32768, size=(5000, 1))
    x[:4, 0] = [-32768, 32767, 0, -1]
    f = tmp_path / "m16.wav"
    f.write_bytes(_wav_bytes(x, 16, 22050, extensible))
    y, sr = nio.load_audio(str(f), keep_pcm16=True)
    ref, sr0 = nio.load_audio(str(f))
    assert isinstance(y, nio.Pcm16) and y.dtype == np.int16 and sr == sr0 == 22050
    assert np.array_equal(y.view(np.ndarray), x[:, 0].astype(np.int16))
    f32 = nio.as_f32(y)
    assert f32.dtype == np.float32 and np.array_equal(f32, ref) and not isinstance(f32, nio.Pcm16)
    assert isinstance(y[10:20], nio.Pcm16) and np.array_equal(nio.as_f32(y[10:20]), ref[10:20])
    assert np.array_equal(nio.as_f32(ref), ref)


def test_keep_pcm16_only_for_mono_16bit_at_the_rate(tmp_path):
    """Stereo, other widths and files that need the load-time resample stay float32."""
    rng = np.random.default_rng(8)
    st = tmp_path / "s16.wav"
    st.write_bytes(_wav_bytes(rng.integers(-32768, 32768, size=(800, 2)), 16, 22050, False))
    m24 = tmp_path / "m24.wav"
    m24.write_bytes(_wav_bytes(rng.integers(-(1 << 23), 1 << 23, size=(800, 1)), 24, 22050, False))
    for f in (st, m24):
        y, _ = nio.load_audio(str(f), keep_pcm16=True)
        assert type(y) is np.ndarray and y.dtype == np.float32
        assert np.array_equal(y, nio.load_audio(str(f))[0])
    m16 = tmp_path / "m16_48k.wav"
    m16.write_bytes(_wav_bytes(rng.integers(-32768, 32768, size=(800, 1)), 16, 48000, False))
    y, sr = nio.load_audio(str(m16), sr=None, keep_pcm16=True)     # its own rate: kept
    assert isinstance(y, nio.Pcm16) and sr == 48000
