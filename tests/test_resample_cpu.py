"""CPU pinning of the load-time resampler (io.py:44-55).

librosa.load resamples with libsoxr soxr_hq, which is absent here and cannot be
bit-matched (documented deviation); the engine's resampler is
scipy.signal.resample_poly, reproduced on the GPU bit for bit.  These tests pin the
restated term order (oracle.ncref.resample_poly_terms) and the host filter plan
(ops.poly_plan) to scipy itself, so the GPU test only has to match the restatement."""
import numpy as np
import pytest
import scipy.signal

from oracle import ncref
from nightcore_analyzer.ops import poly_plan

RATIOS = [(1, 2), (147, 320), (147, 160), (2, 1), (4, 5), (3, 7), (441, 480)]   # 44.1k, 48k, 24k -> 22.05k, ...


@pytest.mark.parametrize("up,down", RATIOS)
@pytest.mark.parametrize("n", [0, 1, 5, 63, 1000, 20_011])
def test_terms_bit_identical_to_scipy(up, down, n):
    if n == 0:
        return                               # scipy returns an empty array; the engine never launches
    x = np.random.default_rng(n + up).standard_normal(n).astype(np.float32)
    want = scipy.signal.resample_poly(x.astype(np.float64), up, down)
    u, d, h, pre = poly_plan(up, down, n)
    n_out = -(-n * u // d)
    got = ncref.resample_poly_terms(x, u, d, h, pre, n_out)
    assert len(want) == n_out
    assert np.array_equal(got.astype(np.float32), want.astype(np.float32))
    assert np.array_equal(got, want)


def test_longer_filter_plan_is_harmless():
    """A batch shares the plan of its longest file: the extra trailing zero taps leave a
    shorter file's output bit-identical."""
    x = np.random.default_rng(1).standard_normal(3001).astype(np.float32)
    want = scipy.signal.resample_poly(x.astype(np.float64), 147, 320)
    u, d, h, pre = poly_plan(147, 320, 10 * len(x))
    got = ncref.resample_poly_terms(x, u, d, h, pre, len(want))
    assert np.array_equal(got, want)
