"""CPU checks of the spectral row (spectral.py:38-359): the oracle against the
reference's own goldens, known answers from first principles, and the host-side
report against the reference's printed text.  No GPU needed."""
import contextlib
import io
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import ncref, refglue
from nightcore_analyzer import spectral, synth
import golden.cases as cases

GOLD = json.loads((Path(__file__).parent / "golden" / "spectral.json").read_text())


@pytest.mark.parametrize("name", [c[0] for c in cases.SPECTRAL_CASES])
def test_oracle_equals_reference_golden(name):
    y, sr = cases.make_spectral_signal(synth, name)
    g = GOLD["cases"][name]
    assert (len(y), sr) == (g["n"], g["sr"])
    assert refglue.spectral_analyze(y, sr) == g["stats"]


def test_known_answers_bin_centred_tone():
    """A periodic-Hann frame of a bin-centred tone leaks into exactly k0-1, k0, k0+1 with
    magnitudes 1/2 : 1 : 1/2, so interior frames have centroid f(k0), rolloff f(k0+1)
    (running sum 1/4, 3/4, 1 of the total vs 0.85) and the rms of a sine is A/sqrt(2)."""
    sr, k0, A = 22050, 93, 0.5
    y = (A * np.sin(2 * np.pi * k0 * sr / 2048 * np.arange(30 * sr) / sr)).astype(np.float32)
    S = ncref.stft_mag(y)
    freqs = ncref.fft_frequencies(sr)
    cen = ncref.spectral_centroid(S=S, sr=sr)[0]
    rol = ncref.spectral_rolloff(S=S, sr=sr)[0]
    mid = slice(8, S.shape[1] - 8)
    np.testing.assert_allclose(cen[mid], freqs[k0], rtol=1e-5)
    assert np.all(rol[mid] == freqs[k0 + 1])
    np.testing.assert_allclose(ncref.rms_frames(y)[mid], A / np.sqrt(2), rtol=1e-3)
    out = refglue.spectral_analyze(y, sr)
    assert out["effective_bandwidth_hz"] == freqs[k0 + 1]
    assert out["sub_bass"] < 1e-2 * out["midrange"]


def test_known_answers_silence_and_db_floor():
    out = refglue.spectral_analyze(np.zeros(4096, np.float32), 44100)
    assert out["centroid"] == out["rolloff"] == out["rms_mean"] == out["decay_rate"] == 0.0
    assert out["effective_bandwidth_hz"] == 22050.0          # every bin ties at 0 dB -> last bin
    db = ncref.amplitude_to_db(np.array([[1.0, 1e-6], [0.5, 0.0]], np.float32), ref=np.max)
    np.testing.assert_allclose(db, [[0.0, -80.0], [20 * np.log10(0.5), -80.0]], atol=1e-5)


def test_rolloff_first_crossing_matches_definition():
    rng = np.random.default_rng(3)
    S = rng.random((1025, 50)).astype(np.float32)
    got = ncref.spectral_rolloff(S=S, sr=22050)[0]
    freqs = ncref.fft_frequencies(22050)
    for t in range(50):
        c = np.cumsum(S[:, t])
        assert got[t] == freqs[np.argmax(c >= 0.85 * c[-1])]


def test_report_text_matches_reference():
    for c in GOLD["compare"]:
        a = spectral.SpectralStats(**GOLD["cases"][c["ref"]]["stats"])
        b = spectral.SpectralStats(**GOLD["cases"][c["other"]]["stats"])
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            spectral.compare_and_print(a, b, c["label_ref"], c["label_other"], c["ref_path"], c["other_path"])
        assert buf.getvalue() == c["text"]


def test_quality_note_grades_and_same_label_quirk():
    assert [spectral._transcode_grade(b) for b in (None, 16_000, 18_000, 19_999, 20_000)] == \
        [None, "MP3 ~128 kbps", "MP3 ~192 kbps", "MP3 ~320 kbps", None]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        spectral._format_quality_note("a.wav", "b.flac", 1.0, 1.0, "X", "X", 16000.0, 17000.0)
    lines = buf.getvalue().splitlines()
    # the reference picks the container name by label, so equal labels show the first file's twice
    assert lines[5].startswith("  ! X (WAV) — spectral content cuts off at ~17.0 kHz")
    assert spectral._pct(0.0, 5.0) == 0.0
