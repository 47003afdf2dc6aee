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
    ("chords60_intro", 60.0, 1005, "chords", {"auto_align": True}, "intro"),
]

# xcorr.find_content_offset cases: (seconds, seed, intro seconds, resample_poly up, down)
ALIGN_CASES = [(60.0, 1005, 7.3, 4, 5), (90.0, 1006, 15.0, 10, 11), (45.0, 1007, 0.0, 4, 5),
               (8.0, 1008, 0.0, 4, 5)]


def make_align_pair(synth, seconds, seed, intro_sec, up, down):
    """(src with a quiet intro of intro_sec, nc = src content sped up by down/up): the
    source content carries a 1 s step gain so its RMS envelope has a unique alignment."""
    from scipy.signal import resample_poly
    src = synth.make_source(seconds, seed)
    rng = np.random.default_rng(seed + 99)
    g = np.repeat(rng.uniform(0.25, 1.0, int(len(src) // 22050) + 1), 22050)[:len(src)].astype(np.float32)
    srcm = (src * g).astype(np.float32)
    nc = resample_poly(srcm, up, down).astype(np.float32)
    if intro_sec > 0:
        intro = (synth.make_source(intro_sec, seed + 500) * np.float32(0.3)).astype(np.float32)
        srcm = np.concatenate([intro, srcm]).astype(np.float32)
    return nc, srcm


def edit(nc, src, how, seed, synth=None, seconds=None):
    if how == "intro":
        return make_align_pair(synth, seconds, seed, 7.3, 4, 5)
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
                nc, src = edit(nc, src, ed, seed, synth, secs)
            return nc, src, kw
    raise KeyError(name)
