"""MELODIA restatement (opt-in, PARITY UNPINNED: essentia, which the reference calls at
pitch.py:210-215, is not installed, so no essentia output pins any of this) without a GPU:

* the CPU oracle of the frame front end (oracle/melodia_ref.py) on tones whose answer is known
  from first principles: the salience peak of a harmonic tone sits at its fundamental's bin;
* the host contour stage (nightcore_analyzer/melodia.py: PitchContours, PitchContoursMelody) on
  synthetic salience peaks and on the oracle's front end: one steady peak gives one contour at its
  pitch, an octave duplicate is removed, a short blip is not a contour, unvoiced frames read 0;
* the backend switch: the default keeps the reference's skip/essentia behaviour."""
import numpy as np
import pytest

from nightcore_analyzer import melodia as M
from oracle import melodia_ref as R


def _peaks(T, rows):
    """SaliencePeaks from rows[t] = [(bin, sal), ...]."""
    c = np.zeros(T, np.int32)
    b = np.zeros((T, M.SALPK), np.int32)
    s = np.zeros((T, M.SALPK), np.float32)
    for t, r in enumerate(rows):
        r = sorted(r, key=lambda x: (-x[1], x[0]))
        c[t] = len(r)
        for i, (bb, ss) in enumerate(r):
            b[t, i], s[t, i] = bb, ss
    return M.SaliencePeaks(c, b, s)


def test_window_and_frames_agree_with_oracle():
    np.testing.assert_array_equal(M.window(), R.window())
    assert M.window().dtype == np.float32 and abs(float(M.window().sum()) - 2.0) < 1e-5
    for n in (0, 1, 127, 128, 2048, 661500):
        assert M.n_frames(n) == R.n_frames(n) == -(-(n + 1024) // 128)
    assert M.cent_bin(55.0) == 0 and M.cent_bin(110.0) == 120 and M.cent_bin(80.0) == 65


def _tone(f0, seconds=1.0, sr=22050, nh=6, seed=0):
    t = np.arange(int(seconds * sr)) / sr
    y = sum((0.6 ** h) * np.sin(2 * np.pi * f0 * (h + 1) * t) for h in range(nh))
    y += 1e-4 * np.random.default_rng(seed).standard_normal(len(t))
    return (0.2 * y).astype(np.float32)


@pytest.mark.parametrize("f0", [110.0, 220.0, 330.0])
def test_oracle_salience_peak_at_the_fundamental(f0):
    y = _tone(f0)
    for t in (40, 80, 120):
        bins, sal = R.frame_salience_peaks(y, t)
        assert len(bins) and abs(int(bins[0]) - M.cent_bin(f0)) <= 1, (f0, t, bins[:3])


def test_one_steady_peak_is_one_contour_at_its_pitch():
    T = 200
    p = _peaks(T, [[(300, 1.0)] for _ in range(T)])
    cs = M.pitch_contours(p)
    assert len(cs) == 1 and cs[0].start == 0 and len(cs[0].bins) == T
    hz = M.contours_melody(cs, T)
    np.testing.assert_allclose(hz, 55.0 * 2 ** 2.5)


def test_short_blip_is_not_a_contour_and_reads_unvoiced():
    T = 100
    rows = [[(300, 1.0)] if 40 <= t < 45 else [] for t in range(T)]   # 5 frames < 100 ms
    cs = M.pitch_contours(_peaks(T, rows))
    assert cs == []
    assert not M.contours_melody(cs, T).any()


def test_octave_duplicate_removed():
    T = 400
    rng = np.random.default_rng(3)
    rows = []
    for t in range(T):
        a = 0.95 + 0.05 * rng.random()
        rows.append([(300, a), (420, a - 0.02)])     # the fundamental a little stronger
    cs = M.pitch_contours(_peaks(T, rows))
    assert len(cs) == 2
    hz = M.contours_melody(cs, T)
    assert np.all(hz == hz[0]) and abs(hz[0] - 55.0 * 2 ** 2.5) < 1e-9


def test_contour_follows_a_glide_and_breaks_at_a_jump():
    T = 300
    rows = []
    for t in range(T):
        b = 250 + t // 10 if t < 150 else 450          # a slow glide, then a jump of > 16 bins
        rows.append([(b, 1.0)])
    cs = M.pitch_contours(_peaks(T, rows))
    assert [(c.start, len(c.bins)) for c in cs] == [(0, 150), (150, 150)]


def test_oracle_front_end_to_melody_on_a_tone():
    y = _tone(220.0, seconds=0.6)
    T = R.n_frames(len(y))
    rows = []
    for t in range(T):
        b, s = R.frame_salience_peaks(y, t)
        rows.append(list(zip(b.tolist(), s.tolist())))
    hz = M.melody_from_peaks(_peaks(T, rows))
    voiced = hz[hz > 0]
    assert len(voiced) > 0.6 * T
    assert abs(12 * np.log2(np.median(voiced) / 220.0)) < 0.1


def test_backend_default_keeps_the_reference_skip(monkeypatch):
    from nightcore_analyzer import pitch
    monkeypatch.delenv("NC_MELODIA", raising=False)
    if pitch._try_import_essentia() is not None:
        pytest.skip("essentia is installed here")
    assert pitch.melodia_backend() is None
    monkeypatch.setenv("NC_MELODIA", "device")
    assert pitch.melodia_backend() == "device"
    assert pitch.melodia_backend("essentia") is None      # an explicit backend wins over the env


@pytest.mark.slow
def test_oracle_melody_shift_of_a_nightcore_pair():
    """Oracle front end + host contours on a 1.25x melody pair: the voiced-median shift is the
    true 3.86 st within the 10-cent grid (about 10 s of numpy)."""
    from nightcore_analyzer import synth
    nc, src = synth.make_melody_pair(6.0, 7)
    med = []
    for y in (src, nc):
        T = R.n_frames(len(y))
        rows = []
        for t in range(T):
            b, s = R.frame_salience_peaks(y, t)
            rows.append(list(zip(b.tolist(), s.tolist())))
        hz = M.melody_from_peaks(_peaks(T, rows))
        assert (hz > 0).sum() > 0.3 * T
        med.append(np.median(hz[hz > 0]))
    assert abs(12 * np.log2(med[1] / med[0]) - 12 * np.log2(1.25)) < 0.15


# ---- the host stage against the oracle's independent restatement (oracle/melodia_ref.py)
def _rows_of(p):
    return [p.frame(t) for t in range(len(p.counts))]


def _ref_contours(p):
    return R.contours_ref(_rows_of(p))


def _same_contours(cs, ref):
    assert len(cs) == len(ref), (len(cs), len(ref))
    for c, (start, bins, sals) in zip(cs, ref):
        assert c.start == start
        np.testing.assert_array_equal(c.bins, np.array(bins))
        np.testing.assert_array_equal(c.sal, np.array(sals))


def _same_melody(hz, ref):
    """Same voicing and the same bin per frame (Hz from numpy's vectorised power and Python's
    scalar one may differ in the last bit)."""
    np.testing.assert_array_equal(hz > 0, ref > 0)
    np.testing.assert_allclose(hz, ref, rtol=1e-12, atol=0)


@pytest.mark.parametrize("seed", range(4))
def test_contours_and_melody_equal_the_oracle_on_random_peaks(seed):
    """Random salience peaks with notes, glides, octave copies, gaps and noise peaks: the host's
    contours and melody equal the restatement's exactly (decisions and values)."""
    rng = np.random.default_rng(seed)
    T = 900
    rows = []
    note, left = 300, 0
    for t in range(T):
        if left == 0:
            note, left = int(rng.integers(200, 420)), int(rng.integers(20, 120))
        left -= 1
        r = []
        if rng.random() > 0.08:                                    # the melody, with dropouts
            r.append((note + int(rng.integers(-2, 3)), float(0.8 + 0.2 * rng.random())))
        if rng.random() < 0.5:                                     # its octave copy, weaker
            r.append((note + 120, float(0.5 + 0.3 * rng.random())))
        for _ in range(int(rng.integers(0, 4))):                   # noise peaks
            r.append((int(rng.integers(65, 600)), float(0.05 + 0.6 * rng.random())))
        seen = {}
        for b, s in r:
            seen[b] = max(s, seen.get(b, 0.0))
        rows.append(list(seen.items()))
    p = _peaks(T, rows)
    cs = M.pitch_contours(p)
    ref = _ref_contours(p)
    assert len(cs) > 5
    _same_contours(cs, ref)
    _same_melody(M.contours_melody(cs, T), R.melody_ref(ref, T))


@pytest.mark.slow
def test_host_stage_equals_oracle_on_a_melody_pair_front_end():
    """The oracle's front end of a 1.25x melody pair feeds both host stages: identical contours,
    identical melody (about 10 s of numpy)."""
    from nightcore_analyzer import synth
    nc, src = synth.make_melody_pair(4.0, 7)
    for y in (src, nc):
        T = R.n_frames(len(y))
        rows = []
        for t in range(T):
            b, s = R.frame_salience_peaks(y, t)
            rows.append(list(zip(b.tolist(), s.tolist())))
        p = _peaks(T, rows)
        cs = M.pitch_contours(p)
        _same_contours(cs, _ref_contours(p))
        hz = M.contours_melody(cs, T)
        _same_melody(hz, R.melody_ref(_ref_contours(p), T))
        assert (hz > 0).sum() > 0.3 * T
