#!/usr/bin/env python3
"""Saves one config-3 batch's 64 outcomes (unrendered, as the window-sharded gather pickles
them) to gpurun_out/outcomes.pkl, for host-side profiling of the gather's pickling on the CPU.
    python3 tools/dump_outcomes.py"""
import pickle
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    import bench
    from nightcore_analyzer import engine as E
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    outs = eng.analyze(signals=sig, params=E.Params(compute_ibi=False))
    (REPO / "gpurun_out").mkdir(exist_ok=True)
    with open(REPO / "gpurun_out" / "outcomes.pkl", "wb") as f:
        pickle.dump(list(enumerate(outs)), f, protocol=pickle.HIGHEST_PROTOCOL)
    print("saved", len(outs))


if __name__ == "__main__":
    main()
