"""The leading tuning frames of a 20 s chunk that starts where a 10 s window starts are
computed inside the window STFT (nc_window_stage_tuning + nc_chroma_mean_shared).  They
are the same samples through the same FFT and the same piptrack code (nc_piptrack.h),
so the fused path must give BIT-IDENTICAL tuning, chroma and results to the unfused one
(and both match the oracle: tests/test_gpu_chroma.py, tests/test_gpu_pipeline.py)."""
import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


def _run(eng, pairs, share, **kw):
    old = eng.share_tuning
    eng.share_tuning = share
    try:
        return eng.analyze(pairs, E.Params(compute_ibi=False, **kw))
    finally:
        eng.share_tuning = old


def test_shared_tuning_frames_are_bit_identical(eng):
    pairs = [synth.make_pair(65.0, 1001), synth.make_pair(130.0, 1005), synth.make_pair(31.0, 1006),
             synth.make_pair(12.0, 1007)]
    a = _run(eng, pairs, False)
    b = _run(eng, pairs, True)
    for x, y in zip(a, b):
        assert repr(x.error) == repr(y.error)
        if x.error is not None:
            continue
        assert np.array_equal(x.detail["tuning"], y.detail["tuning"])
        assert np.array_equal(x.detail["chroma"], y.detail["chroma"])
        assert list(x.detail["chunk_lags"]) == list(y.detail["chunk_lags"])
        assert str(x.result) == str(y.result)


def test_shared_tuning_bit_identical_with_dense_peaks(eng):
    """Frames with more than 64 piptrack peaks (two compaction passes) through the window
    STFT's piptrack and through tuning_peaks_kernel."""
    import scipy.signal
    from test_gpu_chroma import dense_peak_chunk
    src = dense_peak_chunk(45 * 22050, 11)
    nc = scipy.signal.resample_poly(src, 4, 5).astype(np.float32)
    a = _run(eng, [(nc, src)], False)[0]
    b = _run(eng, [(nc, src)], True)[0]
    assert repr(a.error) == repr(b.error)
    assert np.array_equal(a.detail["tuning"], b.detail["tuning"])
    assert np.array_equal(a.detail["chroma"], b.detail["chroma"])


def test_shared_tuning_with_trim_and_offsets(eng):
    """Windows and chunks start at the trimmed file start (silence strip, src_trim_sec)."""
    nc, src = synth.make_pair(70.0, 1002)
    src = np.concatenate([np.zeros(50_000, np.float32), src, np.zeros(30_001, np.float32)])
    pairs = [(nc, src)]
    for kw in ({}, {"src_trim_sec": 1.5}):
        a = _run(eng, pairs, False, **kw)[0]
        b = _run(eng, pairs, True, **kw)[0]
        assert np.array_equal(a.detail["tuning"], b.detail["tuning"])
        assert str(a.result) == str(b.result)


def test_analyze_leaves_no_reference_cycles(eng):
    """analyze() pauses the cyclic collector; everything it allocates must be freed by
    reference counting, or garbage would pile up between collections."""
    import gc
    pairs = [synth.make_pair(45.0, 1001), synth.make_pair(12.0, 1007)]
    eng.analyze(pairs, E.Params(compute_ibi=True))
    gc.collect()
    gc.disable()
    try:
        outs = eng.analyze(pairs, E.Params(compute_ibi=True))
        _ = [str(o.result) for o in outs if o.result is not None] + [o.logs for o in outs]
        del outs, _
        found = gc.collect()
    finally:
        gc.enable()
    assert found == 0, f"{found} objects in reference cycles"
