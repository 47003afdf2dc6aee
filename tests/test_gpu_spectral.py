"""GPU parity of spectral.analyze (spectral.py:38-103, nc_spectral_stats) against the
CPU oracle (oracle/refglue.spectral_analyze) and the reference's own goldens
(tests/golden/spectral.json, made by running the reference's spectral module).

Tolerances (f32 FFT on the device, f64 FFT rounded to complex64 in librosa):
  * centroid, rms mean / variance: relative 2e-5;
  * band means: relative 2e-5 plus an absolute floor of 1e-6 x the file's largest band
    mean (the f32 FFT's error floor; a band 90 dB below the bass, as in the low-passed
    case, sits on it);
  * rolloff: the per-frame bin is the first crossing of an f32 running sum whose
    summation order differs (numpy: sequential) over |S| values that differ by ~1e-7
    (f32 vs f64 FFT), so a frame moves by one bin at a near-tie.  Where the spectrum
    is thin at the crossing (a brick-wall cutoff) the increments are ~1e-5 of the
    total and about 0.1 % of frames tie: |mean difference| <= bin_hz * max(3, T/500) / T;
  * decay_rate = mean(diff(loud frame RMS)) telescopes to (last - first) / (n - 1)
    of f32 frame RMS values: absolute 1e-6 * max(rms) + relative 1e-3;
  * duration and effective bandwidth (a bin frequency): exact;
  * frame RMS: relative 2e-6; per-bin dB means: 2e-3 dB.
"""
import contextlib
import io
import json
import wave
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import refglue
from nightcore_analyzer import engine as E
from nightcore_analyzer import spectral, synth
import golden.cases as cases

pytestmark = pytest.mark.gpu
GOLD = json.loads((Path(__file__).parent / "golden" / "spectral.json").read_text())


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


def _check(got: dict, want: dict, y: np.ndarray, sr: int, rms_max: float):
    T = 1 + len(y) // 512
    hz = np.fft.rfftfreq(2048, 1.0 / sr)[1]
    bands = ("sub_bass", "bass", "midrange", "presence", "brilliance")
    floor = 1e-6 * max(want[k] for k in bands)
    for k in ("centroid", "rms_mean", "rms_variance") + bands:
        assert got[k] == pytest.approx(want[k], rel=2e-5, abs=floor if k in bands else 1e-12), k
    assert abs(got["rolloff"] - want["rolloff"]) <= hz * max(3.0, T / 500.0) / T + 1e-9
    assert abs(got["decay_rate"] - want["decay_rate"]) <= 1e-6 * rms_max + 1e-3 * abs(want["decay_rate"])
    assert got["duration"] == want["duration"]
    assert got["effective_bandwidth_hz"] == want["effective_bandwidth_hz"]


@pytest.mark.parametrize("name", [c[0] for c in cases.SPECTRAL_CASES])
def test_spectral_matches_golden_and_oracle(eng, name):
    y, sr = cases.make_spectral_signal(synth, name)
    sig = eng.upload_signals([y])
    ev, h, keep = eng.spectral_frames(sig.buf, sig.off, sig.length, [sr], frame_rms=True)
    ev.synchronize()
    got = eng.spectral_finish(h)[0]
    ref, det = refglue.spectral_analyze(y, sr, detail=True)
    rms_max = float(det["rms"].max())
    np.testing.assert_allclose(h["rms"], det["rms"], rtol=2e-6, atol=1e-12)
    T = len(det["rms"])
    np.testing.assert_allclose(h["bins"][:1025] / T, det["bin_db_mean"], atol=2e-3)
    rms = det["rms"]                       # the device percentile follows numpy's rule exactly
    assert h["stats"][10] == np.percentile(h["rms"], 75)
    assert got["rms_mean"] == pytest.approx(float(np.mean(rms)), rel=2e-6, abs=1e-12)
    _check(got, ref, y, sr, rms_max)
    _check(got, GOLD["cases"][name]["stats"], y, sr, rms_max)


def test_spectral_batch_mixed_rates_equals_single(eng):
    names = ["chords30_44k_lp16k", "tone20_22k", "sweep20_48k", "silence", "short"]
    sigs = [cases.make_spectral_signal(synth, n) for n in names]
    batch = spectral.analyze_batch(sigs)
    for (y, sr), b in zip(sigs, batch):
        assert b == spectral.analyze_arrays(y, sr)


_NUM = __import__("re").compile(r"[-+]?\d+(?:\.\d+)?")


def _same_report(got: str, want: str) -> bool:
    """Identical text except printed numbers, which may differ in the last printed digit
    (or by 1e-3 relative): a percentage of a band 90 dB below the bass (the low-passed
    case's brilliance) carries the f32 FFT floor into its first decimal."""
    if _NUM.sub("#", got) != _NUM.sub("#", want):
        return False
    for a, b in zip(_NUM.findall(got), _NUM.findall(want)):
        if a != b and abs(float(a) - float(b)) > max(0.1 + 1e-9, 1e-3 * abs(float(b))):
            return False
    return True


def test_compare_report_from_device_stats(eng):
    stats = {}
    names = sorted({c["ref"] for c in GOLD["compare"]} | {c["other"] for c in GOLD["compare"]})
    for n, st in zip(names, spectral.analyze_batch([cases.make_spectral_signal(synth, n) for n in names])):
        stats[n] = st
    exact = 0
    for c in GOLD["compare"]:
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            spectral.compare_and_print(stats[c["ref"]], stats[c["other"]], c["label_ref"], c["label_other"],
                                       c["ref_path"], c["other_path"])
        assert _same_report(buf.getvalue(), c["text"]), (buf.getvalue(), c["text"])
        exact += buf.getvalue() == c["text"]
    assert exact >= len(GOLD["compare"]) - 1


def test_analyze_path_native_rate(eng, tmp_path):
    y, sr = cases.make_spectral_signal(synth, "chords30_44k_lp16k")
    p = tmp_path / "ncog.wav"
    with wave.open(str(p), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(np.clip(np.round(y * 32767.0), -32768, 32767).astype("<i2").tobytes())
    q = (np.frombuffer(p.read_bytes()[44:], "<i2").astype(np.float32) / 32768.0)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        got = spectral.analyze(str(p), label="NCOG")
    assert buf.getvalue() == "  Loading NCOG…\n"
    want = refglue.spectral_analyze(q, sr)
    assert got.duration == want["duration"] and got.effective_bandwidth_hz == want["effective_bandwidth_hz"]
    assert got.centroid == pytest.approx(want["centroid"], rel=2e-5)


def test_spectral_full_size_3min_44k(eng):
    """BASELINE config-2 length at 44.1 kHz (15 504 frames): the MP3-like cutoff is found
    and the device result is independent of the batch it runs in."""
    src = synth._chords(180 * 22050, np.random.default_rng(77)).astype(np.float64)
    from scipy.signal import resample_poly
    y = resample_poly(src, 2, 1)
    y = y + np.random.default_rng(78).standard_normal(len(y)) * 0.003
    X = np.fft.rfft(y)
    X[np.fft.rfftfreq(len(y), 1 / 44100) >= 16000] = 0
    y = np.fft.irfft(X, len(y)).astype(np.float32)
    a, = spectral.analyze_batch([(y, 44100)])
    b = spectral.analyze_batch([(y[:44100 * 20], 44100), (y, 44100)])[1]
    assert a == b
    assert 15_900 < a.effective_bandwidth_hz < 16_100
    ref = refglue.spectral_analyze(y, 44100)
    _check(a.__dict__, ref, y, 44100, 1.0)
