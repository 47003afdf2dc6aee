"""Deterministic synthetic nightcore/source pairs.

There is no network and the reference ships no audio, so every benchmark and
parity case runs on these signals:

* source  = equal-tempered triad sequence (A4 = 440 Hz, 4 harmonics, amplitude
  0.2, chord change every 4 beats, roots drawn by the rng)
          + a click/kick every 10 752 samples (= 168 hop-64 frames = 21 hop-512
  frames -> 123.046875 BPM, exactly on both tempo grids; 30 ms decaying noise +
  60 Hz burst, amplitude 0.5)
          + white noise at -50 dBFS;
* nightcore = ``scipy.signal.resample_poly(src, 4, 5)`` (an exact 1.25x
  speed-up: pitch and tempo together).

``kind="sweep"`` replaces the chords by a log sine sweep 100 Hz -> 4 kHz (config
1 of BASELINE.json).
"""
from __future__ import annotations

import numpy as np
import scipy.signal

SR = 22050
BEAT_SAMPLES = 10752


def _clicks(n: int, rng: np.random.Generator, period: int = BEAT_SAMPLES) -> np.ndarray:
    y = np.zeros(n, dtype=np.float64)
    L = int(0.030 * SR)
    Lk = int(0.080 * SR)
    t = np.arange(max(L, Lk)) / SR
    env_n = np.exp(-t[:L] / 0.006)
    kick = np.sin(2 * np.pi * 60.0 * t[:Lk]) * np.exp(-t[:Lk] / 0.025)
    for b in range(0, n, period):
        noise = rng.standard_normal(L) * env_n
        e = min(n, b + L)
        y[b:e] += 0.5 * 0.5 * noise[:e - b]
        e = min(n, b + Lk)
        y[b:e] += 0.5 * kick[:e - b]
    return y


def _chords(n: int, rng: np.random.Generator) -> np.ndarray:
    y = np.zeros(n, dtype=np.float64)
    seg = 4 * BEAT_SAMPLES
    harm = np.array([1.0, 0.5, 1.0 / 3.0, 0.25])
    harm = harm / harm.sum()
    t = np.arange(seg) / SR
    ramp = np.minimum(1.0, np.minimum(np.arange(seg), seg - 1 - np.arange(seg)) / 256.0)
    for s in range(0, n, seg):
        root = int(rng.integers(48, 60))
        third = 3 if rng.random() < 0.5 else 4
        notes = [root, root + third, root + 7]
        chunk = np.zeros(seg)
        for m in notes:
            f0 = 440.0 * 2.0 ** ((m - 69) / 12.0)
            for h, a in enumerate(harm, start=1):
                chunk += a * np.sin(2 * np.pi * f0 * h * t + rng.random() * 2 * np.pi)
        e = min(n, s + seg)
        y[s:e] += (0.2 / 3.0) * (chunk * ramp)[:e - s]
    return y


def _sweep(n: int) -> np.ndarray:
    t = np.arange(n) / SR
    T = n / SR
    f0, f1 = 100.0, 4000.0
    k = np.log(f1 / f0)
    phase = 2 * np.pi * f0 * T / k * (np.exp(t / T * k) - 1.0)
    return 0.2 * np.sin(phase)


def make_source(seconds: float, seed: int, kind: str = "chords") -> np.ndarray:
    n = int(round(seconds * SR))
    rng = np.random.default_rng(seed)
    tonal = _chords(n, rng) if kind == "chords" else _sweep(n)
    y = tonal + _clicks(n, rng) + rng.standard_normal(n) * 10 ** (-50 / 20)
    return y.astype(np.float32)


def make_pair(seconds: float = 180.0, seed: int = 1000, kind: str = "chords",
              up: int = 4, down: int = 5):
    """Return (nightcore, source) float32 arrays; nc = resample_poly(src, up, down)."""
    src = make_source(seconds, seed, kind)
    nc = scipy.signal.resample_poly(src.astype(np.float64), up, down).astype(np.float32)
    return nc, src


def make_melody_pair(seconds: float = 6.0, seed: int = 7, up: int = 4, down: int = 5):
    """(nightcore, source) with one clear melody line (MELODIA cases): 0.5 s notes drawn from
    MIDI 57-71, 6 harmonics at 0.5^h, 20 ms ramps, amplitude 0.3, over white noise at 0.02;
    nc = resample_poly(src, up, down)."""
    rng = np.random.default_rng(seed)
    n = int(round(seconds * SR))
    y = np.zeros(n)
    t = np.arange(int(0.5 * SR)) / SR
    env = np.minimum(1.0, np.minimum(t, t[-1] - t) / 0.02)
    for s in range(0, n, len(t)):
        f0 = 440.0 * 2 ** ((int(rng.integers(57, 72)) - 69) / 12)
        note = sum((0.5 ** h) * np.sin(2 * np.pi * f0 * (h + 1) * t) for h in range(6)) * env
        e = min(n, s + len(t))
        y[s:e] += 0.3 * note[:e - s]
    y += 0.02 * rng.standard_normal(n)
    src = y.astype(np.float32)
    nc = scipy.signal.resample_poly(src.astype(np.float64), up, down).astype(np.float32)
    return nc, src


def pair_lengths(seconds: float = 180.0, up: int = 4, down: int = 5):
    """(nightcore, source) lengths of make_pair(seconds, ...) without making the pair."""
    n = int(round(seconds * SR))
    return -(-n * up // down), n


def make_batch(n_pairs: int, seconds: float = 180.0, base_seed: int = 1000, kind: str = "chords"):
    """Config-3/4 style batch: pair i uses seed base_seed + i."""
    return [make_pair(seconds, base_seed + i, kind) for i in range(n_pairs)]
