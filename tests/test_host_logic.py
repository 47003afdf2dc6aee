"""The product's host-side logic (no GPU): result assembly, classification,
Rubber Band parameters, warnings and report text, export/CLI schemas, the
bootstrap seeding / percentile parameters and the window/chunk planning —
against the reference's own outputs (tests/golden/units.json)."""
import math

import numpy as np
import pytest

from nightcore_analyzer import consensus as C
from nightcore_analyzer import export
from nightcore_analyzer.engine import percentile_params, seed_state
from nightcore_analyzer.pitch import _chunk_plan
from oracle import refglue


def _num(xs):
    return [float(x) if isinstance(x, str) else x for x in xs]


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, float) and not math.isfinite(x):
        return repr(x)
    return x


def test_assemble_matches_reference_build_result(golden_units):
    """Given the bootstrap numbers (here from numpy, on the device in the product),
    consensus.assemble reproduces every field and the report of build_result."""
    for c in golden_units["build_result"]:
        sp, npch, st, nt = (_num(c[k]) for k in ("src_p", "nc_p", "src_t", "nc_t"))
        vs, vn, ts, tn = (refglue.valid(x) for x in (sp, npch, st, nt))
        if "error" in c:
            with pytest.raises(ValueError) as ei:
                C.assemble(sp, npch, st, nt, nc_duration=c["nc_duration"], src_duration=c["src_duration"],
                           pitch_boot=None, tempo_boot=(1.0, (1.0, 1.0)))
            assert str(ei.value) == c["error"]["message"]
            continue
        pb = refglue.bootstrap_ratio(vn, vs) if len(vs) >= 3 and len(vn) >= 3 else None
        tb = refglue.bootstrap_ratio(tn, ts)
        r = C.assemble(sp, npch, st, nt, nc_duration=c["nc_duration"], src_duration=c["src_duration"],
                       pitch_boot=pb, tempo_boot=tb)
        got = _norm({k: getattr(r, k) for k in c["result"]})
        assert got == c["result"], c["name"]
        assert str(r) == c["str"], c["name"]


def test_classify_and_rubberband(golden_units):
    for c in golden_units["classify"]:
        assert C._classify(c["tr"], c["pr"], tuple(c["tci"]), tuple(c["pci"])) == c["cls"]
    for c in golden_units["rubberband"]:
        assert C._rubberband_params(c["tr"], c["pr"], c["ncd"], c["srd"]) == c["rb"]


def test_valid_filter():
    assert C._valid([None, float("nan"), -1.0, 0.0, 2.0, float("inf"), 3.5]).tolist() == [2.0, 3.5]


def test_seed_state_is_numpy_pcg64():
    for seed in (0, 42, 12345):
        s = np.random.PCG64(seed).state["state"]
        hi, lo, ihi, ilo = seed_state(seed)
        assert (hi << 64 | lo) == s["state"] and (ihi << 64 | ilo) == s["inc"]


def test_percentile_params_reproduce_numpy_linear():
    rng = np.random.default_rng(5)
    x = np.sort(rng.random(2000))
    il, gl, ih, gh = percentile_params(2000, 0.95)

    def lerp(a, b, t):
        d = b - a
        return b - d * (1 - t) if t >= 0.5 else a + d * t
    alpha = (1.0 - 0.95) / 2.0          # consensus.py:263-265 computes the quantiles this way
    assert lerp(x[int(il)], x[int(il) + 1], gl) == np.percentile(x, alpha * 100)
    assert lerp(x[int(ih)], x[int(ih) + 1], gh) == np.percentile(x, (1.0 - alpha) * 100)


@pytest.mark.parametrize("ns,nn", [(3969000, 3175200), (441000, 441000), (441000 * 3 + 5, 441000 * 2),
                                   (300000, 3175200), (0, 100)])
def test_chunk_plan_matches_reference_glue(ns, nn):
    assert _chunk_plan(ns, nn, 22050) == refglue.chunk_plan(ns, nn)


def test_export_schema_roundtrip(tmp_path, golden_units):
    c = next(x for x in golden_units["build_result"] if x["name"] == "normal")
    sp, npch, st, nt = (_num(c[k]) for k in ("src_p", "nc_p", "src_t", "nc_t"))
    vs, vn, ts, tn = (refglue.valid(x) for x in (sp, npch, st, nt))
    r = C.assemble(sp, npch, st, nt, nc_duration=c["nc_duration"], src_duration=c["src_duration"],
                   pitch_boot=refglue.bootstrap_ratio(vn, vs), tempo_boot=refglue.bootstrap_ratio(tn, ts))
    d = export.to_dict(r)
    assert set(d) == {"classification", "warnings", "tempo_ratio", "pitch_ratio", "tempo_ci_95", "pitch_ci_95",
                      "windows_used", "rubberband", "durations", "median_bpms"}
    export.export_csv(r, tmp_path / "r.csv")
    header = (tmp_path / "r.csv").read_text().splitlines()[0].split(",")
    assert header[0] == "classification" and header[-1] == "warnings" and len(header) == 24


def test_median_is_numpy_median_bit_for_bit():
    rng = np.random.default_rng(3)
    for n in range(1, 80):
        x = rng.random(n) * 300.0
        assert C._median(x.tolist()) == float(np.median(x))
    assert C._median([2583.984375 / 21] * 4) == 2583.984375 / 21


def test_pair_groups_cover_the_batch_in_order():
    from nightcore_analyzer.engine import _group_bounds
    for B in (1, 7, 16, 17, 40, 64, 100):
        g = _group_bounds(B, 16)
        assert g[0][0] == 0 and g[-1][1] == B
        assert all(a1 == b0 for (a0, a1), (b0, b1) in zip(g, g[1:]))
        assert all(b > a for a, b in g)


def test_default_pair_group_schedule():
    """The engine's default schedule (groups of 32, the last two evened out) covers any batch in
    order with no empty or small stragglers; the config-3 batch gets 32/32."""
    from nightcore_analyzer.engine import _group_bounds
    assert [b - a for a, b in _group_bounds(64, None)] == [32, 32]
    assert [b - a for a, b in _group_bounds(70, None)] == [32, 19, 19]
    assert [b - a for a, b in _group_bounds(17, None)] == [17]
    assert [b - a for a, b in _group_bounds(33, None)] == [17, 16]
    assert _group_bounds(0, None) == []
    for B in range(1, 200):
        g = _group_bounds(B, None)
        sizes = [b - a for a, b in g]
        assert g[0][0] == 0 and g[-1][1] == B and sum(sizes) == B
        assert all(a1 == b0 for (a0, a1), (b0, b1) in zip(g, g[1:]))
        assert min(sizes) >= min(B, 16) and max(sizes) <= 32
    assert [b - a for a, b in _group_bounds(10, [3, 4])] == [3, 4, 3]
