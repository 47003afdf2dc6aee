#!/usr/bin/env python3
"""Which objects of one analyze() call end up in reference cycles (gc.DEBUG_SAVEALL)."""
import gc
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))

from nightcore_analyzer import engine as E, synth  # noqa: E402

eng = E.get_engine(0)
pairs = [synth.make_pair(45.0, 1001), synth.make_pair(12.0, 1007)]
for ibi in (False, True):
    eng.analyze(pairs, E.Params(compute_ibi=ibi))
    gc.collect()
    gc.set_debug(gc.DEBUG_SAVEALL)
    gc.disable()
    outs = eng.analyze(pairs, E.Params(compute_ibi=ibi))
    _ = [str(o.result) for o in outs if o.result is not None] + [o.logs for o in outs]
    del outs, _
    n = gc.collect()
    print("ibi", ibi, "cycle objects", n)
    for o in gc.garbage[:12]:
        r = repr(o)
        print("  ", type(o).__name__, r[:200])
    gc.garbage.clear()
    gc.set_debug(0)
    gc.enable()
