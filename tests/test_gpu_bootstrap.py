"""GPU parity: the bootstrap kernel against numpy's Generator (the reference's
own RNG) — bit-exact points, CIs and every one of the 2000 resample ratios."""
import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


def test_bootstrap_golden_reference_consensus(eng, golden_units):
    """consensus._bootstrap_ratio / compute_ibi_ratio outputs of the reference itself."""
    cases = golden_units["bootstrap"]
    outs = eng.bootstrap([(np.array(c["a"]), np.array(c["b"])) for c in cases], seed=42)
    ibis = eng.bootstrap([(np.array(c["b"]), np.array(c["a"])) for c in cases], seed=42)
    for c, (p, ci), (ip, ici) in zip(cases, outs, ibis):
        assert p == c["point"]
        assert list(ci) == c["ci"]
        assert ip == c["ibi_point"]
        assert list(ici) == c["ibi_ci"]


def _numpy_boots(a, b, seed, n_boot=2000):
    rng = np.random.default_rng(seed)
    out = np.empty(n_boot)
    for i in range(n_boot):
        x = np.median(rng.choice(a, size=len(a), replace=True))
        out[i] = x / np.median(rng.choice(b, size=len(b), replace=True)) if b is not None else x
    return out


def _device_boots(eng, a, b, seed, ctl_out=None):
    """Run nc_bootstrap_ratio with boot_out to compare every resample."""
    from nightcore_analyzer.engine import _Upload, percentile_params, seed_state
    vals = np.concatenate([a, b]) if b is not None else a
    cap = len(vals)
    up = _Upload()
    up.add("vals", vals, np.float64)
    up.add("a_off", [0], np.int64)
    up.add("a_n", [len(a)], np.int32)
    up.add("b_off", [len(a)], np.int64)
    up.add("b_n", [len(b) if b is not None else 0], np.int32)
    up.add("seed", seed_state(seed), np.uint64)
    up.add("wsoff", [0], np.int64)
    up.add("cap", [cap], np.int32)
    d = up.commit(eng.dev)
    out = torch.zeros(3, dtype=torch.float64, device=eng.dev)
    boots = torch.zeros(2000, dtype=torch.float64, device=eng.dev)
    ws = eng.workspace("t_boot", eng.ctx.lib.nc_bootstrap_job_bytes(cap, 2000))
    il, gl, ih, gh = percentile_params(2000, 0.95)
    eng.call("nc_bootstrap_ratio", d["vals"].data_ptr(), d["a_off"].data_ptr(), d["a_n"].data_ptr(),
             d["b_off"].data_ptr() if b is not None else None, d["b_n"].data_ptr() if b is not None else None,
             1, 2000, d["seed"].data_ptr(), il, gl, ih, gh, 1, out[0:1].data_ptr(), out[1:2].data_ptr(),
             out[2:3].data_ptr(), boots.data_ptr(), d["wsoff"].data_ptr(), d["cap"].data_ptr(), ws.data_ptr(),
             ws.numel(), eng.stream())
    if ctl_out is not None:  # JobCtl (bootstrap.hip): after rank/sorted/start/boot
        o = ((cap * 4 + 15) & ~15) + cap * 8 + 2000 * 16
        ctl_out.extend(ws[o:o + 24].cpu().numpy().view(np.int32)[:4].tolist())
        ctl_out.append(int(ws[o + 16:o + 24].cpu().numpy().view(np.int64)[0]))
    return boots.cpu().numpy(), out.cpu().numpy()


@pytest.mark.parametrize("na,nb,seed", [(27, 35, 42), (1, 5, 42), (2, 1, 42), (3000, 2500, 42),
                                        (4097, 1, 7), (9, None, 0)])
def test_every_resample_bit_exact(eng, na, nb, seed):
    """Covers n == 1 (no draws), the low/high half-word carry and Lemire rejections (large n)."""
    rng = np.random.default_rng(na * 7 + 1)
    a = np.round(rng.random(na) * 100 + 50, 1)        # ties on purpose
    b = None if nb is None else np.round(rng.random(nb) * 100 + 50, 1)
    got, pt = _device_boots(eng, a, b, seed)
    ref = _numpy_boots(a, b, seed)
    np.testing.assert_array_equal(got, ref)
    assert pt[1] == np.percentile(ref, 2.5) and pt[2] == np.percentile(ref, 97.5)


def test_rejections_resolved_by_exact_starts(eng):
    """A large job meets Lemire rejections (flag set); the sparse rejection scan + walk gives
    exact starts (status 0: no fix-point fallback) and every resample stays bit-exact."""
    rng = np.random.default_rng(5)
    a = np.round(rng.random(3000) * 100 + 50, 1)
    b = np.round(rng.random(2500) * 100 + 50, 1)
    ctl = []
    got, _ = _device_boots(eng, a, b, 42, ctl)
    flag, nrej_a, nrej_b, status, end = ctl
    assert flag == 1 and status == 0
    assert nrej_a + nrej_b > 0 and end > 2000 * 5500
    np.testing.assert_array_equal(got, _numpy_boots(a, b, 42))


@pytest.mark.parametrize("a,b", [([3.0] * 7, [2.0] * 5),             # every resample equal (no digit pass)
                                 ([1.0, 2.0] * 4, [1.0] * 3),         # two values, heavy ties at both ranks
                                 ([-0.5, 0.25, 7.0], None),           # signs and a single array
                                 ([1e-300, 1e300, 1.0, 2.0, 3.0], [1.0, 1e-300])])
def test_percentiles_on_tied_and_extreme_boots(eng, a, b):
    """The order statistics behind the CI (ranks il, il + 1, ih, ih + 1 of the 2000 resample
    ratios, boot_order_stats) on ties, a constant set, signs and a 600-decade spread."""
    a = np.array(a)
    b = None if b is None else np.array(b)
    got, pt = _device_boots(eng, a, b, 3)
    ref = _numpy_boots(a, b, 3)
    np.testing.assert_array_equal(got, ref)
    assert pt[1] == np.percentile(ref, 2.5) and pt[2] == np.percentile(ref, 97.5)
