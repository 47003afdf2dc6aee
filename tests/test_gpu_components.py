"""GPU parity of the remaining components against the CPU oracle, through the
drop-in module functions (io / tempo / pitch / xcorr), plus full-size (3-min,
BASELINE config 2) properties."""
import numpy as np
import pytest
import scipy.signal
import torch

from oracle import ncref, refglue
from nightcore_analyzer import engine as E
from nightcore_analyzer import io as nio
from nightcore_analyzer import ops, pitch, synth, tempo, xcorr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


def _silence_cases():
    nc, src = synth.make_pair(12.0, 1007)
    z = np.zeros
    return [src, np.concatenate([z(33_333, np.float32), src, z(7_777, np.float32)]),
            np.concatenate([z(1000, np.float32), src[:50_000] * np.float32(1e-4), src]),
            z(40_000, np.float32), src[:1500].copy()]


def test_trim_matches_oracle(eng):
    cases = _silence_cases()
    got = ops.trim_bounds(eng, cases, 60.0)
    for y, g in zip(cases, got):
        assert g == ncref.trim(y, 60.0)[1]
    y = cases[1]
    t, lead, trail = nio.strip_silence(y, 22050, 60.0)
    rt, rlead, rtrail = refglue.strip_silence(y, 22050, 60.0)
    assert len(t) == len(rt) and lead == rlead and trail == rtrail


def test_slice_windows_energies(eng):
    nc, src = synth.make_pair(40.0, 1008)
    wins = nio.slice_windows(src, 22050)
    ref = refglue.slice_windows(src, 22050)
    assert [w.start_sec for w in wins] == [w.start_sec for w in ref]
    assert np.max(np.abs(np.array([w.energy_db for w in wins]) - [w.energy_db for w in ref])) < 1e-9
    assert [w.start_sec for w in nio.energy_gate(wins)] == [w.start_sec for w in refglue.energy_gate(ref)]


def test_window_energy_from_trim_blocks(eng):
    """nc_window_energy_blocks (round 6): io._rms_db of windows at any sample offset of their
    (untrimmed) file, from the silence trim's f64 512-sample block sums plus the partial blocks
    at the window ends, equals the direct f64 sum of the window's samples (nc_window_energy) and
    the oracle to 1e-9 dB; the engine's pipelined groups take their energies from it."""
    cases = _silence_cases()[:3] + [synth.make_pair(45.0, 1010)[0]]
    sig = eng.upload_signals(cases)
    start, end, tb = eng._trim_all(sig, E.Params())
    assert tb is not None and (tb.f0, tb.f1) == (0, len(cases))
    rng = np.random.default_rng(4)
    win_off, win_file, ref = [], [], []
    L = 22050 * 2 + 333
    for f, y in enumerate(cases):
        if len(y) < L:
            continue
        for s in sorted({0, 1, 511, 512, 513, len(y) - L, *rng.integers(0, len(y) - L, 6).tolist()}):
            win_off.append(int(sig.off[f]) + s)
            win_file.append(f)
            ref.append(refglue.rms_db(y[s:s + L]))
    n = len(win_off)
    d_off = torch.tensor(win_off, dtype=torch.int64, device=eng.dev)
    d_file = torch.tensor(win_file, dtype=torch.int32, device=eng.dev)
    out = torch.empty(n, dtype=torch.float64, device=eng.dev)
    eng.call("nc_window_energy_blocks", sig.buf.data_ptr(), tb.ws.data_ptr(), tb.f1 - tb.f0, tb.off.data_ptr(),
             d_off.data_ptr(), d_file.data_ptr(), n, L, out.data_ptr(), eng.stream())
    got = out.cpu().numpy()
    assert np.max(np.abs(got - np.array(ref))) < 1e-9
    # the same windows through nc_window_energy (direct f64 sums over the samples)
    for f in sorted(set(win_file)):
        idx = [i for i in range(n) if win_file[i] == f]
        d = ops.window_energies(eng, cases[f], np.array([win_off[i] - int(sig.off[f]) for i in idx]), L)
        assert np.max(np.abs(np.asarray(d) - got[idx])) < 1e-9


def test_batch_estimate_tempo_and_logs(eng):
    nc, src = synth.make_pair(40.0, 1009)
    wins = nio.slice_windows(nc, 22050)
    logs = []
    got = tempo.batch_estimate_tempo(wins, log=logs.append, start_bpm=153.80859375)
    ref = [refglue.estimate_tempo(w.audio, 22050, 153.80859375) for w in wins]
    assert got == ref
    assert logs[-1] == f"    {sum(r is not None for r in ref)}/{len(ref)} windows yielded a confident tempo estimate"


def test_estimate_ibis_global_matches_oracle(eng):
    nc, src = synth.make_pair(35.0, 1010)
    for y, prior in ((src, 120.0), (nc, 153.80859375)):
        got = tempo.estimate_ibis_global(y, 22050, start_bpm=prior)
        ref = refglue.estimate_ibis_global(y, 22050, start_bpm=prior)
        assert (got is None) == (ref is None)
        np.testing.assert_array_equal(got, ref)


def test_estimate_pitch_chroma_matches_oracle(eng):
    nc, src = synth.make_pair(70.0, 1011)
    logs = []
    s_hz, n_hz, pt, ci, n = pitch.estimate_pitch_chroma(src, nc, 22050, log=logs.append)
    r = refglue.estimate_pitch_chroma(src, nc, 22050)
    assert (s_hz, n_hz, pt, ci, n) == r[:5]
    assert pitch.estimate_pitch_combined(src, nc, 22050)[2] == "chroma_xcorr"


@pytest.mark.parametrize("speed", [1.0, 1.01])
def test_xcorr_speed_matches_oracle(eng, speed):
    nc, src = synth.make_pair(60.0, 1012)
    if speed == 1.0:
        yb = src.copy()
    else:
        yb = scipy.signal.resample_poly(src.astype(np.float64), 100, 101).astype(np.float32)
    g = xcorr.estimate_speed_xcorr_arrays(src, yb)
    r = refglue.estimate_speed_xcorr_arrays(src, yb)
    assert abs(g[0] - r[0]) < 1e-9 and abs(g[1] - r[1]) < 1e-5
    assert xcorr.estimate_speed_xcorr_arrays(np.zeros(500_000, np.float32), yb) == (1.0, 0.0)


def test_find_content_offset_matches_reference(eng, golden_units):
    """The device intro search reproduces the reference's find_content_offset goldens, one
    pair at a time (the drop-in) and as one batch (the engine path of run(auto_align))."""
    from golden.cases import make_align_pair
    pairs, exp = [], []
    for c in golden_units["find_content_offset"]:
        nc, src = make_align_pair(synth, c["seconds"], c["seed"], c["intro"], c["up"], c["down"])
        assert xcorr.find_content_offset(src, nc, 22050) == (c["offset"], c["speed"])
        pairs.append((src, nc))
        exp.append((c["offset"], c["speed"]))
    sig = eng.upload_signals([a for p in pairs for a in p])
    got = eng.align_offsets(sig.buf, sig.off[0::2], sig.length[0::2], sig.off[1::2], sig.length[1::2])
    assert got == exp
    # a 60-min source against a 48-min nightcore: the device search matches the oracle
    rng = np.random.default_rng(5)
    g = np.repeat(rng.uniform(0.25, 1.0, 3601), 22050).astype(np.float32)
    src = (np.resize(synth.make_source(60.0, 1013), 3600 * 22050) * g[:3600 * 22050]).astype(np.float32)
    nc = scipy.signal.resample_poly(src[30 * 22050:], 4, 5).astype(np.float32)
    assert xcorr.find_content_offset(src, nc, 22050) == refglue.find_content_offset(src, nc, 22050)


def test_full_size_pair_properties(eng):
    """BASELINE config 2 (one 3-min pair): exact window counts and duration ratio,
    tempo on the expected grid lags (21 / 17), chroma lag +4 on every chunk, IBI ~1.25."""
    nc, src = synth.make_pair(180.0, 1000)
    out, = eng.analyze([(nc, src)], E.Params())
    r, d = out.result, out.detail
    assert len(d["energy_src"]) == 35 and len(d["energy_nc"]) == 27
    assert r.src_duration / r.nc_duration == 1.25
    assert all(t == 2583.984375 / 21 for t in r.src_tempos_raw)
    assert all(t == 2583.984375 / 17 for t in r.nc_tempos_raw)
    # 12-bin chroma lags sit near 4 (3.86 st), with near-ties the oracle reproduces
    ref_lags = [refglue.chunk_lag(src[a:b], nc[c:dd]) for a, b, c, dd in refglue.chunk_plan(len(src), len(nc))]
    assert d["chunk_lags"] == ref_lags
    assert abs(r.pitch_ratio - 2 ** (float(np.median(ref_lags)) / 36)) < 1e-12
    assert r.classification == "time_stretch_only"
    assert abs(r.ibi_ratio - 1.25) < 0.01


@pytest.mark.parametrize("window_sec,hop_sec", [(25.0, 12.5), (90.0, 45.0)])
def test_long_windows_match_oracle(eng, window_sec, hop_sec):
    """--window 25 / 90 (cli.py:37): 1 077-frame windows run the correlation window_tg at one
    workgroup per CU (~110 KB LDS); 3 876-frame windows take the sliding-sum window_tg
    (above the correlation kernel's LDS) and the beat tracker's global-workspace path.
    Tempos equal the oracle's."""
    nc, src = synth.make_pair(300.0, 1014)
    p = E.Params(window_sec=window_sec, hop_sec=hop_sec, compute_ibi=False)
    out, = eng.analyze([(nc, src)], p)
    ref = refglue.run_arrays(nc, src, window_sec=window_sec, hop_sec=hop_sec, compute_ibi=False)
    assert out.error is None, out.error
    assert out.result.src_tempos_raw == ref["src_tempos"] and out.result.nc_tempos_raw == ref["nc_tempos"]
    assert out.result.tempo_ratio == ref["tempo_ratio"]
    with pytest.raises(ValueError):
        eng.analyze([(nc, src)], E.Params(window_sec=240.0, hop_sec=60.0))


def test_profile_modes_time_what_they_say(eng):
    """nc_profile_enable: 1 events + spans on every kernel, 2 spans only, 3 events on the
    roofline kernels + spans, 4 events on the roofline kernels only (the bench's timed region);
    results identical whichever mode is on (timing never changes the arithmetic)."""
    nc, src = synth.make_pair(40.0, 1011)
    p = E.Params(compute_ibi=False)
    roof = {"stft_mel", "cqt_low", "cqt_high", "window_tg"}
    ref = eng.analyze([(nc, src)], p)[0].result
    for mode in (1, 2, 3, 4):
        eng.kernel_profile(mode)
        out = eng.analyze([(nc, src)], p)[0].result
        ev, sp = eng.kernel_times(), eng.kernel_spans()
        eng.kernel_profile(0)
        assert (out.tempo_ratio, out.pitch_ratio, out.tempo_ci, out.pitch_ci) == \
               (ref.tempo_ratio, ref.pitch_ratio, ref.tempo_ci, ref.pitch_ci)
        ev_k = set(ev) - {"cqt_chroma"}
        sp_k = set(sp) - {"cqt_chroma"}
        if mode == 1:
            assert roof <= ev_k and roof <= sp_k and "decimate" in ev_k and "decimate" in sp_k
        elif mode == 2:
            assert not ev_k and roof <= sp_k
        elif mode == 3:
            assert ev_k == roof and roof <= sp_k and "decimate" in sp_k
        else:
            assert ev_k == roof and not sp_k
        assert all(ms > 0 and n > 0 for ms, n in ev.values())


def test_profile_marker_spans(eng):
    """Profile mode 5: the timed kernels' spans plus marker spans around the small entry points
    (bootstraps, gate, valid-tempo collection, prior, chroma plan / tail / lag, trim bounds,
    window energies); results unchanged, and the markers leave modes 2 and 4 alone."""
    nc, src = synth.make_pair(40.0, 1013)
    p = E.Params(compute_ibi=False)
    ref = eng.analyze([(nc, src)], p)[0].result
    eng.kernel_profile(5)
    out = eng.analyze([(nc, src)], p)[0].result
    spans = eng.device_spans()
    eng.kernel_profile(2)
    eng.analyze([(nc, src)], p)
    spans2 = eng.device_spans()
    eng.kernel_profile(0)
    assert (out.tempo_ratio, out.pitch_ratio, out.tempo_ci, out.pitch_ci) == \
           (ref.tempo_ratio, ref.pitch_ratio, ref.tempo_ci, ref.pitch_ci)
    tags = {t for t, _, _ in spans}
    small = {"bootstrap", "energy_gate", "collect_valid", "tempo_prior", "chroma_plan", "cqt_tail", "chroma_lag",
             "trim_bounds", "window_energy"}
    assert small <= tags and {"stft_mel", "cqt_low", "cqt_high"} <= tags, tags
    assert all(0.0 <= a <= b for _, a, b in spans)
    assert not small & {t for t, _, _ in spans2}      # mode 2 records no markers


def test_profile_span_dump_and_busy_agree(eng):
    """nc_profile_dump_spans (mode 2): every timed launch of one analysis with its tag, start
    <= end, inside one extent; the union of the dumped spans equals what nc_profile_read_busy
    reports for a second, identical call (same kernels, same union semantics)."""
    nc, src = synth.make_pair(40.0, 1012)
    p = E.Params(compute_ibi=False)
    eng.analyze([(nc, src)], p)
    eng.kernel_profile(2)
    eng.analyze([(nc, src)], p)
    spans = eng.device_spans()
    eng.analyze([(nc, src)], p)
    busy, extent, n = eng.device_busy()
    eng.kernel_profile(0)
    tags = {t for t, _, _ in spans}
    assert {"stft_mel", "window_tg", "cqt_low", "cqt_high", "decimate", "tuning_peaks"} <= tags
    assert all(0.0 <= a <= b for _, a, b in spans) and min(a for _, a, _ in spans) == 0.0
    assert n == len(spans) and extent > 0.0 and 0.0 < busy <= extent * (1 + 1e-9)
    iv, u, cur = sorted((a, b) for _, a, b in spans), 0.0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            u += 0.0 if cur is None else cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    u += cur[1] - cur[0]
    assert 0.5 < u / busy < 2.0          # two runs of the same call: the same order of magnitude
    assert eng.device_spans() == []      # the dump and the busy read both clear the spans
