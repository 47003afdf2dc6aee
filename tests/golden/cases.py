"""Input definitions shared by make_golden.py (fixture generation) and the
parity tests: the synthetic pairs are regenerated from seeds, never stored."""
import numpy as np

PIPELINE_CASES = [
    # name, seconds, seed, kind, run() kwargs, edit
    ("sweep30", 30.0, 1000, "sweep", {}, None),
    ("chords80", 80.0, 1001, "chords", {}, None),
    ("chords80_nopitch", 80.0, 1001, "chords", {"compute_pitch": False}, None),
    ("chords75_silence", 75.0, 1002, "chords", {"src_trim_sec": 1.5}, "silence"),
    ("chords60_gate", 60.0, 1003, "chords", {"energy_gate_db": -20.0}, "quiet"),
]


def edit(nc, src, how, seed):
    if how == "silence":
        src = np.concatenate([np.zeros(50_000, np.float32), src, np.zeros(30_001, np.float32)])
        nc = np.concatenate([np.zeros(12_345, np.float32), nc])
    elif how == "quiet":
        a, b = 300_000, 300_000 + 12 * 22050
        src = src.copy()
        src[a:b] *= np.float32(10 ** (-30 / 20))
        nc = nc.copy()
        nc[:200_000] *= np.float32(10 ** (-25 / 20))
    return nc, src


def make_case(synth, name):
    for n, secs, seed, kind, kw, ed in PIPELINE_CASES:
        if n == name:
            nc, src = synth.make_pair(secs, seed, kind)
            if ed:
                nc, src = edit(nc, src, ed, seed)
            return nc, src, kw
    raise KeyError(name)
