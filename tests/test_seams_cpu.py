"""The drop-in seams called with the reference's own signatures, on the CPU (no device
work reaches the engine): the pitch seams raise ValueError for a sample rate other than
io.SAMPLE_RATE instead of being analysed with the 22 050 Hz CQT tables (pitch.py:55-62), the
tempo seams for a rate outside the 8-48 kHz their per-rate tables cover (tempo.py:41-44,158;
44.1 kHz runs on the device: tests/test_gpu_seams.py),
session.set_many takes the reference's dict (session.py:37-41), and MELODIA runs
essentia's algorithm when essentia is importable (pitch.py:187-241; a stand-in module
here, since essentia is absent: parity unpinned)."""
import json
import math
import sys
import types

import numpy as np
import pytest

from nightcore_analyzer import io as nio, pitch, session, tempo

SR44 = 44100


def _window(sr):
    return nio.AudioWindow(audio=np.zeros(10 * sr, np.float32), sample_rate=sr, start_sec=0.0, end_sec=10.0,
                           energy_db=-100.0)


@pytest.mark.parametrize("call", [
    lambda: pitch._mean_chroma(np.zeros(SR44 * 20, np.float32), SR44),
    lambda: pitch._chroma_shift_for_chunk(np.zeros(SR44 * 20, np.float32), np.zeros(SR44 * 20, np.float32), SR44),
    lambda: pitch.estimate_pitch_chroma(np.zeros(SR44 * 60, np.float32), np.zeros(SR44 * 60, np.float32), SR44,
                                        log=None),
    lambda: pitch.estimate_pitch_combined(np.zeros(SR44 * 60, np.float32), np.zeros(SR44 * 60, np.float32), SR44,
                                          log=None),
])
def test_other_sample_rates_raise_value_error(call):
    with pytest.raises(ValueError, match="44100 Hz"):
        call()


@pytest.mark.parametrize("sr", [4000, 96000])
@pytest.mark.parametrize("call", [
    lambda sr: tempo.estimate_tempo(_window(sr)),
    lambda sr: tempo.batch_estimate_tempo([_window(sr)], log=None, start_bpm=120.0),
    lambda sr: tempo.estimate_ibis_global(np.zeros(sr * 20, np.float32), sr, hop_length=64, min_ibis=4,
                                          start_bpm=120.0),
])
def test_tempo_seams_outside_the_table_rates_raise(call, sr):
    with pytest.raises(ValueError, match=f"{sr} Hz is outside"):
        call(sr)


def test_session_set_many_takes_a_dict(tmp_path, monkeypatch):
    f = tmp_path / "s.json"
    monkeypatch.setattr(session, "_SESSION_FILE", f)
    session.set("a", 1)
    session.set_many({"window": 12.0, "hop": 6.0})        # gui/main_window.py:201's call
    assert json.loads(f.read_text()) == {"a": 1, "window": 12.0, "hop": 6.0}
    assert session.get("hop") == 6.0 and session.get("missing", 7) == 7


class _FakeMelodia:
    """essentia.standard.PredominantPitchMelodia stand-in: the F0 track of a known tone."""
    calls = []

    def __init__(self, frameSize, hopSize, sampleRate):
        _FakeMelodia.calls.append((frameSize, hopSize, sampleRate))
        self.hop = hopSize

    def __call__(self, audio):
        assert audio.dtype == np.float32
        n = 1 + len(audio) // self.hop
        f0 = np.full(n, float(audio[0]), np.float32)   # the "pitch" is carried by the first sample
        f0[::3] = 0.0                                  # unvoiced frames
        return f0, np.ones(n, np.float32)


@pytest.fixture
def fake_essentia(monkeypatch):
    es = types.ModuleType("essentia.standard")
    es.PredominantPitchMelodia = _FakeMelodia
    pkg = types.ModuleType("essentia")
    pkg.standard = es
    monkeypatch.setitem(sys.modules, "essentia", pkg)
    monkeypatch.setitem(sys.modules, "essentia.standard", es)
    _FakeMelodia.calls.clear()
    return es


def test_melodia_runs_when_essentia_is_importable(fake_essentia):
    src = np.full(22050 * 30, 440.0, np.float32)
    nc = np.full(22050 * 24, 440.0 * 2 ** (4 / 12), np.float32)
    lines = []
    out = pitch.estimate_pitch_melodia(src, nc, 22050, log=lines.append)
    assert out is not None
    s, n = out
    assert _FakeMelodia.calls == [(2048, 128, 22050.0)] * 2
    assert len(s) <= 2 * pitch.MAX_MELODIA_FRAMES and len(n) <= 2 * pitch.MAX_MELODIA_FRAMES
    assert all(v == 440.0 for v in s)
    # f32 Hz values: the logged shift is 4 st to f32 rounding; 3445 voiced frames thin by a
    # stride of 3445 // 2000 = 1, i.e. not at all (the reference's own rule, pitch.py:214-217)
    st = float(lines[0].split()[1])
    assert lines[0].startswith("    MELODIA: +") and abs(st - 4.0) < 1e-5 and "(3445 src / 2756 nc voiced frames)" in lines[0]
    assert len(s) == 3445
    # acceptance rule of estimate_pitch_combined: within 1.5 st of the chroma shift; the
    # chroma path reports 4/3 st for this +4 st pair (the lag / 3 quirk), so MELODIA's +4 st
    # is rejected, as the reference would
    assert pitch.melodia_choice(out, 3.0) is not None
    msgs = []
    assert pitch.melodia_choice(out, 4.0 / 3.0, msgs.append) is None
    assert "disagrees with chroma" in msgs[0]


def test_melodia_failure_is_logged_not_raised(fake_essentia, monkeypatch):
    def boom(self, audio):
        raise RuntimeError("bad audio")
    monkeypatch.setattr(_FakeMelodia, "__call__", boom)
    lines = []
    assert pitch.estimate_pitch_melodia(np.ones(4096, np.float32), np.ones(4096, np.float32), 22050,
                                        log=lines.append) is None
    assert lines[0] == "    MELODIA extraction failed: bad audio"


def test_melodia_absent_is_skipped():
    if pitch._try_import_essentia() is not None:
        pytest.skip("essentia is installed here")
    lines = []
    assert pitch.estimate_pitch_melodia(np.ones(10), np.ones(10), 22050, log=lines.append) is None
    assert lines == ["    essentia not available — skipping MELODIA refinement"]
    from nightcore_analyzer.pipeline import _melodia_hook
    assert _melodia_hook([(np.ones(4), np.ones(4))]) is None


def test_wav_header_width_from_block_align(tmp_path):
    """12-bit samples in 2-byte containers: read at the container width."""
    vals = np.array([0, 1024 << 4, -2048 << 4, 32752], np.int16)   # left-justified 12-bit
    fmt = (1).to_bytes(2, "little") + (1).to_bytes(2, "little") + (22050).to_bytes(4, "little") + \
        (44100).to_bytes(4, "little") + (2).to_bytes(2, "little") + (12).to_bytes(2, "little")
    data = vals.tobytes()
    body = b"WAVE" + b"fmt " + len(fmt).to_bytes(4, "little") + fmt + b"data" + len(data).to_bytes(4, "little") + data
    p = tmp_path / "t12.wav"
    p.write_bytes(b"RIFF" + len(body).to_bytes(4, "little") + body)
    y, sr = nio._read_wav(p)
    assert sr == 22050 and np.array_equal(y, vals.astype(np.float32) / 32768.0)
    bad = bytearray(p.read_bytes())
    bad[22:24] = (0).to_bytes(2, "little")            # channels = 0
    p.write_bytes(bytes(bad))
    with pytest.raises(ValueError, match="invalid WAVE header"):
        nio._read_wav(p)


def test_window_limit_matches_the_kernel_formula():
    from nightcore_analyzer import engine as E
    # csrc/window_stage.hip: (2 T + 3 acw) doubles within 160 KiB - 1 KiB
    T = E.MAX_WINDOW_FRAMES
    assert (2 * T + 3 * 344) * 8 <= 160 * 1024 - 1024 < (2 * (T + 1) + 3 * 344) * 8
    assert math.isclose((T - 1) * 512 / 22050, 224.3, abs_tol=0.1)
