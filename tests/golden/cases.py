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
    # the reference's two failure paths (pipeline.py:142-146, consensus.py:544-548): logs up to the raise
    ("sweep30_gate_all", 30.0, 1000, "sweep", {"energy_gate_db": 1.0}, None),
    ("sweep30_nc_tail_quiet", 30.0, 1000, "sweep", {}, "nc_tail_quiet"),
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
    elif how == "nc_tail_quiet":
        # nc windows [10, 20) s at -50 dB: kept by the -60 dB silence trim, dropped by the
        # -40 dB energy gate, leaving 2 nightcore tempo windows (< MIN_VALID = 3)
        nc = nc.copy()
        nc[10 * 22050:] *= np.float32(10 ** (-50 / 20))
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


# spectral.analyze cases (spectral.py:38-103): name -> (seconds, seed, native sample rate, edit)
SPECTRAL_CASES = [
    ("chords30_22k", 30.0, 1000, 22050, "plain"),
    ("chords30_44k", 30.0, 1001, 44100, "full"),          # broadband content up to 22 kHz
    ("chords30_44k_lp16k", 30.0, 1001, 44100, "lp16k"),   # same content, MP3-128k-like cutoff
    ("chords30_44k_dark", 30.0, 1001, 44100, "dark"),     # low-passed + compressed + reverb tail
    ("sweep20_48k", 20.0, 1002, 48000, "sweep"),
    ("tone20_22k", 20.0, 1003, 22050, "tone"),
    ("intro25_22k", 25.0, 1004, 22050, "intro"),
    ("silence", 0.25, 1005, 22050, "zeros"),
    ("short", 0.07, 1006, 22050, "noise"),
]

# compare_and_print pairs: (ref case, other case, label_ref, label_other, ref_path, other_path)
SPECTRAL_COMPARE = [
    ("chords30_44k", "chords30_44k_lp16k", "HQ", "NCOG", "hq.flac", "ncog.flac"),
    ("chords30_44k", "chords30_44k_dark", "REFERENCE", "OTHER", "a.wav", "b.mp3"),
    ("chords30_44k_dark", "chords30_44k", "HQNC", "NCOG", "x.mp3", "y.flac"),
    ("chords30_22k", "intro25_22k", "REFERENCE", "OTHER", None, None),
    ("chords30_44k_lp16k", "chords30_44k_lp16k", "A", "B", "a.aiff", "b.wav"),
    ("sweep20_48k", "chords30_44k", "S", "C", "s.mp3", "c.ogg"),
]


def make_spectral_signal(synth, name):
    """(mono f32 signal, native sample rate) of a SPECTRAL_CASES entry."""
    from scipy.signal import butter, resample_poly, sosfilt
    for n, secs, seed, sr, how in SPECTRAL_CASES:
        if n != name:
            continue
        rng = np.random.default_rng(seed)
        if how == "zeros":
            return np.zeros(int(secs * sr), np.float32), sr
        if how == "noise":
            return (rng.standard_normal(int(secs * sr)) * 0.1).astype(np.float32), sr
        if how == "tone":
            k0 = 93
            t = np.arange(int(secs * sr))
            return (0.5 * np.sin(2 * np.pi * k0 * sr / 2048 * t / sr)).astype(np.float32), sr
        if how == "sweep":
            src = synth.make_pair(secs, seed, "sweep")[1].astype(np.float64)
        elif how in ("full", "lp16k", "dark"):                        # sustained chords, no kick
            src = synth._chords(int(secs * 22050), np.random.default_rng(seed)).astype(np.float64)
        else:
            src = synth.make_source(secs, seed).astype(np.float64)
        if sr != 22050:
            g = np.gcd(sr, 22050)
            src = resample_poly(src, sr // g, 22050 // g)
        if how in ("full", "lp16k"):                                  # mastered: limited peaks
            src = np.tanh(3.0 * src) / 3.0
        if how in ("full", "lp16k", "dark", "sweep"):
            hiss = rng.standard_normal(len(src)) * 0.01               # broadband air / cymbal noise
            src = src + sosfilt(butter(4, 5000, "highpass", fs=sr, output="sos"), hiss)
        if how == "lp16k":                                            # brick-wall, as an MP3 encoder
            X = np.fft.rfft(src)
            X[np.fft.rfftfreq(len(src), 1.0 / sr) >= 16000.0] = 0.0
            src = np.fft.irfft(X, len(src))
        elif how == "dark":
            src = sosfilt(butter(6, 3000, "lowpass", fs=sr, output="sos"), src)
            src = np.tanh(4.0 * src) / 4.0
            tail = np.exp(-np.arange(int(0.4 * sr)) / (0.12 * sr)) * rng.standard_normal(int(0.4 * sr)) * 0.02
            src = np.convolve(src, np.concatenate([[1.0], tail]))[:len(src)]
        elif how == "intro":
            src[:5 * sr] *= 10 ** (-30 / 20)
        return src.astype(np.float32), sr
    raise KeyError(name)
