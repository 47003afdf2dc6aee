"""NC_CU_SPLIT's CU masks (engine.cu_masks; the measurement of VERDICT r5 item 3): the window
and chroma chains get complementary, non-empty CU sets of the requested sizes."""
import pytest

from nightcore_analyzer.engine import cu_masks


@pytest.mark.parametrize("spec,k", [("128", 128), ("160", 160), ("96", 96), ("128:low", 128), ("100", 100)])
def test_masks_complementary(spec, k):
    win, chroma = cu_masks(spec, 256)
    assert len(win) == len(chroma) == 8
    assert sum(bin(w).count("1") for w in win) == k
    assert sum(bin(c).count("1") for c in chroma) == 256 - k
    assert all((w & c) == 0 and (w | c) == 0xFFFFFFFF for w, c in zip(win, chroma))
    if ":low" not in spec:            # every 32-CU word keeps CUs for both chains
        assert all(w and c for w, c in zip(win, chroma))
