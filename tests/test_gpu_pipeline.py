"""GPU parity of the whole drop-in: nightcore_analyzer.pipeline.run (MI355X
engine) against the golden fixtures produced by running the REFERENCE's own
pipeline.run (tests/golden/make_golden.py) on the same synthetic inputs."""
import hashlib
import math

import numpy as np
import pytest
import torch

import nightcore_analyzer as NA
from nightcore_analyzer import export, synth
from nightcore_analyzer.cli import output_dict

from golden.cases import PIPELINE_CASES, make_case

pytestmark = pytest.mark.gpu


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, float) and not math.isfinite(x):
        return repr(x)
    return x


@pytest.mark.parametrize("name", [c[0] for c in PIPELINE_CASES])
def test_run_matches_reference_golden(name, golden_pipeline):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = golden_pipeline[name]
    nc, src, kw = make_case(synth, name)
    assert _sha(nc) == g["nc_sha256"] and _sha(src) == g["src_sha256"], "synthetic input drifted"
    logs = []
    if "error" in g:
        with pytest.raises(Exception) as ei:
            NA.run(nc, src, log=logs.append, **kw)
        assert type(ei.value).__name__ == g["error"]["type"]
        assert str(ei.value) == g["error"]["message"]
        assert logs == g["log"]          # every line the reference logged before raising
        return
    r = NA.run(nc, src, log=logs.append, **kw)
    exp = g["result"]
    # decisions first (most informative failure messages)
    assert r.src_tempos_raw == exp["src_tempos_raw"]
    assert r.nc_tempos_raw == exp["nc_tempos_raw"]
    assert r.nc_pitches_raw == exp["nc_pitches_raw"]
    assert r.src_pitches_raw == exp["src_pitches_raw"]
    got = _norm({k: getattr(r, k) for k in exp})
    for k in exp:
        assert got[k] == exp[k], k
    assert str(r) == g["str"]
    assert _norm(export.to_dict(r)) == g["export_dict"]
    assert logs == g["log"]
    if "cli_json" in g:
        assert _norm(output_dict(r)) == g["cli_json"]
