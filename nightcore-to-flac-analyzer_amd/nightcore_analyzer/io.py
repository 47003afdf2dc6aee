"""Audio I/O, windowing, energy gating and silence stripping
(drop-in for the reference's nightcore_analyzer/io.py).

* ``load_audio`` (io.py:44-55) decodes on the CPU — file decode is out of the
  engine's scope (north_star); WAV (PCM 8/16/24/32-bit, IEEE float, plain or
  WAVE_FORMAT_EXTENSIBLE) and ``.npy`` are parsed with numpy, down-mixed to mono float32 and, if
  the file is not at 22 050 Hz, resampled on the GPU by ``nc_resample_poly``
  (bit-identical to scipy.signal.resample_poly; the reference uses librosa.load's
  soxr_hq, which is absent here — see DESIGN.md).
* ``strip_silence`` (io.py:58-79) runs ``nc_trim_bounds`` on the GPU.
* ``slice_windows`` (io.py:82-112) returns views like the reference, with the
  window energies computed by ``nc_window_energy`` on the GPU.
* ``energy_gate`` (io.py:115-126) is the same list filter.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional

import numpy as np

SAMPLE_RATE: int = 22050
WINDOW_SEC: float = 10.0
HOP_SEC: float = 5.0
ENERGY_GATE_DB: float = -40.0
SILENCE_STRIP_DB: float = 60.0


@dataclass
class AudioWindow:
    """One time slice of an audio file (io.py:27-34)."""
    audio: np.ndarray
    sample_rate: int
    start_sec: float
    end_sec: float
    energy_db: float


def _rms_db(audio: np.ndarray) -> float:
    """20 log10(max(rms, 1e-10)) with float64 accumulation (io.py:38-40), on the GPU."""
    from .engine import get_engine
    from .ops import window_energies
    return float(window_energies(get_engine(), audio, np.array([0]), len(audio))[0])


_WAVE_PCM, _WAVE_FLOAT, _WAVE_EXTENSIBLE = 1, 3, 0xFFFE


class Pcm16(np.ndarray):
    """Mono 16-bit PCM as the file stores it: int16 sample k stands for k / 32768 (soundfile's
    scaling, exact in float32).  ``load_audio(..., keep_pcm16=True)`` returns one for a mono
    16-bit WAV at the requested rate; the engine uploads its 2-byte samples (half the host ->
    HBM bytes of float32) and widens them on the device (``nc_pcm16_to_f32``), so the analysis
    sees exactly the float32 array ``load_audio`` would have returned.  Slices stay Pcm16."""

    def f32(self) -> np.ndarray:
        return self.view(np.ndarray).astype(np.float32) / np.float32(32768.0)


def as_f32(a) -> np.ndarray:
    """The float32 samples of ``a``: a Pcm16 scaled by 1 / 32768, anything else as float32."""
    if isinstance(a, Pcm16):
        return a.f32()
    return np.asarray(a, dtype=np.float32)


def _read_wav(path: Path, keep_pcm16: bool = False):
    """RIFF/WAVE -> (mono float32, rate): PCM 8 (unsigned) / 16 / 24 / 32-bit and IEEE float
    32 / 64-bit, plain or WAVE_FORMAT_EXTENSIBLE (the sub-format GUID's first two bytes
    carry the format tag), scaled to [-1, 1) as soundfile does and averaged over channels
    (librosa.load(mono=True)).  ``keep_pcm16``: a mono 16-bit PCM file comes back as its
    stored samples (Pcm16)."""
    data = Path(path).read_bytes()
    if len(data) < 12 or data[:4] not in (b"RIFF", b"RF64") or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    fmt = raw = None
    pos = 12
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], int.from_bytes(data[pos + 4:pos + 8], "little")
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            raw = body
        pos += 8 + size + (size & 1)
    if fmt is None or raw is None or len(fmt) < 16:
        raise ValueError(f"{path}: WAVE file without fmt/data chunks")
    tag, ch = int.from_bytes(fmt[0:2], "little"), int.from_bytes(fmt[2:4], "little")
    sr, bits = int.from_bytes(fmt[4:8], "little"), int.from_bytes(fmt[14:16], "little")
    if tag == _WAVE_EXTENSIBLE and len(fmt) >= 26:
        tag = int.from_bytes(fmt[24:26], "little")          # SubFormat GUID data1 (low 16 bits)
    block_align = int.from_bytes(fmt[12:14], "little")
    if ch <= 0 or block_align <= 0 or block_align % ch:
        raise ValueError(f"{path}: invalid WAVE header (channels={ch}, block_align={block_align})")
    # the container width, not bits // 8: 12- or 20-bit samples sit left-justified in 2 or 3
    # bytes, so the bytes split into samples at block_align / channels
    width = block_align // ch
    n = len(raw) // (width * ch) * width * ch
    raw = raw[:n]
    if tag == _WAVE_FLOAT and width in (4, 8):
        x = np.frombuffer(raw, "<f4" if width == 4 else "<f8").astype(np.float32)
    elif tag == _WAVE_PCM and width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif tag == _WAVE_PCM and width == 2:
        if keep_pcm16 and ch == 1:
            return np.frombuffer(raw, "<i2").astype(np.int16).view(Pcm16), sr
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif tag == _WAVE_PCM and width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif tag == _WAVE_PCM and width == 4:
        x = (np.frombuffer(raw, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    else:
        raise ValueError(f"{path}: unsupported WAVE format tag {tag} with {bits}-bit samples")
    return x.reshape(-1, ch).mean(axis=1).astype(np.float32), sr


def load_audio(path: str, sr: Optional[int] = SAMPLE_RATE, *, keep_pcm16: bool = False) -> tuple[np.ndarray, int]:
    """Decode *path* to mono float32 at *sr* Hz (io.py:44-55; decode stays on the CPU).
    ``sr=None`` keeps the file's own rate (librosa.load(sr=None), spectral.py:52); a .npy
    file carries no rate and is taken to be at SAMPLE_RATE.  ``keep_pcm16`` (the engine's
    loaders, pipeline.run): a mono 16-bit WAV already at *sr* is returned as its stored
    samples (``Pcm16``: the same values as float32 once scaled by 1 / 32768, on the device)."""
    p = Path(path)
    if p.suffix.lower() == ".npy":
        y, file_sr = np.load(p, allow_pickle=False).astype(np.float32), sr or SAMPLE_RATE
        if y.ndim > 1:
            y = y.mean(axis=0).astype(np.float32)
    elif p.suffix.lower() == ".wav":
        y, file_sr = _read_wav(p, keep_pcm16)
        if isinstance(y, Pcm16):
            if sr is None or file_sr == sr:
                return y, file_sr
            y = y.f32()
    else:
        raise NotImplementedError(
            f"{p.suffix} decoding is outside the engine (the reference uses librosa.load/soundfile, "
            "not installed here); convert to WAV or .npy first")
    if sr is None:
        sr = file_sr
    if file_sr != sr:                   # io.py:54 resamples at load: on the GPU (nc_resample_poly)
        import math
        from .engine import get_engine
        from .ops import resample_poly
        g = math.gcd(int(sr), int(file_sr))
        y, = resample_poly(get_engine(), [y], int(sr) // g, int(file_sr) // g)
    return np.ascontiguousarray(y, dtype=np.float32), sr


def decoded_length(x, sr: int = SAMPLE_RATE) -> int:
    """Samples ``load_audio(x, sr)`` returns, read from the file header alone (a decoded
    array: its length): the window-sharded runs plan every rank's items from the lengths
    of all files before each rank decodes only the files it touches."""
    if isinstance(x, np.ndarray):
        return len(x)
    p = Path(x)
    if p.suffix.lower() == ".npy":
        a = np.load(p, mmap_mode="r", allow_pickle=False)
        return int(a.shape[1] if a.ndim > 1 else a.shape[0])
    if p.suffix.lower() != ".wav":
        return len(load_audio(x, sr)[0])          # raises the same NotImplementedError
    size = p.stat().st_size
    fmt = None
    frames = None
    with open(p, "rb") as fh:
        head = fh.read(12)
        if len(head) < 12 or head[:4] not in (b"RIFF", b"RF64") or head[8:12] != b"WAVE":
            raise ValueError(f"{p}: not a RIFF/WAVE file")
        pos = 12
        while pos + 8 <= size:
            fh.seek(pos)
            ck = fh.read(8)
            cid, n = ck[:4], int.from_bytes(ck[4:8], "little")
            if cid == b"fmt ":
                fmt = fh.read(n)
            elif cid == b"data":
                frames = min(n, size - pos - 8)
            pos += 8 + n + (n & 1)
    if fmt is None or frames is None or len(fmt) < 16:
        raise ValueError(f"{p}: WAVE file without fmt/data chunks")
    ch, block_align = int.from_bytes(fmt[2:4], "little"), int.from_bytes(fmt[12:14], "little")
    if ch <= 0 or block_align <= 0 or block_align % ch:
        raise ValueError(f"{p}: invalid WAVE header (channels={ch}, block_align={block_align})")
    n = frames // block_align
    file_sr = int.from_bytes(fmt[4:8], "little")
    if sr is None or file_sr == sr:
        return n
    import math
    g = math.gcd(int(sr), file_sr)
    up, down = int(sr) // g, file_sr // g
    return -(-n * up // down)                   # resample_poly's output length


def strip_silence(audio: np.ndarray, sr: int, top_db: float = SILENCE_STRIP_DB) -> tuple[np.ndarray, float, float]:
    """(trimmed view, leading_sec, trailing_sec) — librosa.effects.trim on the GPU."""
    from .engine import get_engine
    from .ops import trim_bounds
    (start, end), = trim_bounds(get_engine(), [audio], top_db)
    return audio[start:end], start / sr, (len(audio) - end) / sr


def slice_windows(audio: np.ndarray, sr: int, window_sec: float = WINDOW_SEC,
                  hop_sec: float = HOP_SEC) -> List[AudioWindow]:
    win_n, hop_n = int(window_sec * sr), int(hop_sec * sr)
    starts = []
    s = 0
    while s + win_n <= len(audio):
        starts.append(s)
        s += hop_n
    if not starts:
        return []
    from .engine import get_engine
    from .ops import window_energies
    en = window_energies(get_engine(), audio, np.asarray(starts, np.int64), win_n)
    return [AudioWindow(audio[s:s + win_n], sr, s / sr, (s + win_n) / sr, float(e)) for s, e in zip(starts, en)]


def energy_gate(windows: List[AudioWindow], threshold_db: float = ENERGY_GATE_DB) -> List[AudioWindow]:
    if not windows:
        return windows
    peak = max(w.energy_db for w in windows)
    return [w for w in windows if w.energy_db >= peak + threshold_db]
