#!/usr/bin/env python3
"""Kernel-isolation driver for rocprofv3 counter passes: runs one entry point of
the engine a few times on synthetic data (no oracle, no bench harness).

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/prof_kernels.py chroma
    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/prof_kernels.py windows
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from nightcore_analyzer import engine as E, ops, synth  # noqa: E402


def main(which: str, reps: int = 3) -> None:
    eng = E.get_engine(0)
    rng = np.random.default_rng(0)
    src = synth.make_source(180.0, 1000)
    if which == "chroma":
        chunks = [src[i * 441000:(i + 1) * 441000] for i in range(8)] * 14   # 112 x 20 s
        for _ in range(reps):
            ops.chroma_means(eng, chunks)
    elif which == "windows":
        wins = [src[i * 110250:i * 110250 + 220500] for i in range(35)] * 16  # 560 x 10 s
        for _ in range(reps):
            ops.window_tempos(eng, wins, [120.0] * len(wins))
    else:
        raise SystemExit(f"unknown target {which}")
    torch.cuda.synchronize()
    print("done", which, rng.integers(1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "chroma")
