"""Pin the CPU oracle (oracle/refglue.py on oracle/ncref.py) against the golden
fixtures produced by the REFERENCE's own modules (tests/golden/make_golden.py).
No GPU needed."""
import hashlib
import math

import numpy as np
import pytest

from oracle import ncref, refglue
from nightcore_analyzer import synth
from golden.cases import make_case


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def test_slice_windows_and_gate(golden_units):
    rng = np.random.default_rng(golden_units["slice_windows_rng_seed"])
    for c in golden_units["slice_windows"]:
        y = (rng.standard_normal(c["n"]) * 0.1).astype(np.float32)
        if c["n"] > 400000:
            y[100000:400000] *= np.float32(1e-3)
        assert _sha(y) == c["seed_sha"]
        wins = refglue.slice_windows(y, 22050, c["window_sec"], c["hop_sec"])
        assert [w.start_sec for w in wins] == c["starts"]
        assert [w.end_sec for w in wins] == c["ends"]
        assert [w.energy_db for w in wins] == pytest.approx(c["energy_db"], rel=0, abs=1e-12)
        assert [w.start_sec for w in refglue.energy_gate(wins, -40.0)] == c["gated_starts"]


def test_cyclic_xcorr_peak(golden_units):
    for c in golden_units["cyclic_xcorr_peak"]:
        assert refglue.cyclic_xcorr_peak(np.array(c["src"], np.float32), np.array(c["nc"], np.float32)) == c["lag"]


def test_bootstraps_exact(golden_units):
    for c in golden_units["bootstrap"]:
        a, b = np.array(c["a"]), np.array(c["b"])
        p, ci = refglue.bootstrap_ratio(a, b)
        assert p == c["point"] and list(ci) == c["ci"]
        p, ci = refglue.compute_ibi_ratio(a, b)
        assert p == c["ibi_point"] and list(ci) == c["ibi_ci"]


def test_choice_streams_are_numpy(golden_units):
    for s in golden_units["choice_streams"]:
        r = np.random.default_rng(s["seed"])
        assert [r.integers(0, n, size=n).tolist() for n in s["sizes"]] == s["draws"]


def _num(xs):
    """fixtures store non-finite floats as their repr ('nan', 'inf')"""
    return [float(x) if isinstance(x, str) else x for x in xs]


def test_build_result_numbers(golden_units):
    for c in golden_units["build_result"]:
        args = tuple(_num(c[k]) for k in ("src_p", "nc_p", "src_t", "nc_t"))
        if "error" in c:
            with pytest.raises(ValueError) as ei:
                refglue.build_result(*args, nc_duration=c["nc_duration"], src_duration=c["src_duration"])
            assert str(ei.value) == c["error"]["message"]
            continue
        r = refglue.build_result(*args, nc_duration=c["nc_duration"], src_duration=c["src_duration"])
        e = c["result"]
        for k in ("tempo_ratio", "pitch_ratio", "classification", "n_source_pitch_windows",
                  "n_nc_pitch_windows", "n_source_tempo_windows", "n_nc_tempo_windows",
                  "nc_median_bpm", "src_median_bpm"):
            assert r[k] == e[k], (c["name"], k)
        assert list(r["tempo_ci"]) == e["tempo_ci"] and list(r["pitch_ci"]) == e["pitch_ci"]


def test_classify_grid(golden_units):
    for c in golden_units["classify"]:
        assert refglue.classify(c["tr"], c["pr"], tuple(c["tci"]), tuple(c["pci"])) == c["cls"]


def test_find_content_offset_matches_reference(golden_units):
    """xcorr.find_content_offset (xcorr.py:165-259) of the reference, run on the same
    primitives: identical (offset, speed) on every intro / no-intro / too-short case."""
    from golden.cases import make_align_pair
    for c in golden_units["find_content_offset"]:
        nc, src = make_align_pair(synth, c["seconds"], c["seed"], c["intro"], c["up"], c["down"])
        assert _sha(src) == c["src_sha256"] and _sha(nc) == c["nc_sha256"]
        assert refglue.find_content_offset(src, nc, 22050) == (c["offset"], c["speed"])


@pytest.mark.parametrize("name,ibi", [("sweep30", True), ("chords60_gate", False), ("chords75_silence", False),
                                      ("chords60_intro", False)])
def test_run_arrays_matches_reference_pipeline(golden_pipeline, name, ibi):
    """The oracle's pipeline restatement reproduces the reference's pipeline.run
    (run with the same primitives) on every decision and number."""
    g = golden_pipeline[name]
    nc, src, kw = make_case(synth, name)
    assert _sha(nc) == g["nc_sha256"] and _sha(src) == g["src_sha256"]
    res = refglue.run_arrays(nc, src, compute_ibi=ibi, **kw)
    e = g["result"]
    assert res["src_tempos"] == e["src_tempos_raw"]
    assert res["nc_tempos"] == e["nc_tempos_raw"]
    assert res["src_pitches"] == e["src_pitches_raw"]
    assert res["nc_pitches"] == e["nc_pitches_raw"]
    for k in ("tempo_ratio", "pitch_ratio", "classification", "nc_duration", "src_duration",
              "nc_median_bpm", "src_median_bpm", "intro_offset_sec"):
        assert res[k] == e[k], k
    assert list(res["tempo_ci"]) == e["tempo_ci"] and list(res["pitch_ci"]) == e["pitch_ci"]
    if ibi:
        assert res["ibi_ratio"] == e["ibi_ratio"] and list(res["ibi_ci"]) == e["ibi_ci"]


@pytest.mark.parametrize("name", ["sweep30_gate_all", "sweep30_nc_tail_quiet"])
def test_run_arrays_failure_paths_match_reference(golden_pipeline, name):
    """The reference's two failure exits (pipeline.py:142-146 RuntimeError, consensus.py:544-548
    ValueError): the oracle raises the same type with the same message."""
    g = golden_pipeline[name]
    nc, src, kw = make_case(synth, name)
    assert _sha(nc) == g["nc_sha256"] and _sha(src) == g["src_sha256"]
    with pytest.raises(Exception) as ei:
        refglue.run_arrays(nc, src, compute_ibi=False, **kw)
    assert type(ei.value).__name__ == g["error"]["type"] and str(ei.value) == g["error"]["message"]
