"""Spectral comparison of two files (drop-in for the reference's
nightcore_analyzer/spectral.py).

``analyze`` (spectral.py:38-103) decodes on the CPU at the file's native rate
and computes every statistic on the MI355X: one |STFT| pass feeds the centroid,
the 85 % rolloff, the frame RMS, the five band means and the per-bin
``amplitude_to_db`` means (``nc_spectral_stats``, csrc/spectral.hip).  The host
keeps only O(frames) numpy glue that the reference itself runs on those arrays
(mean / var / percentile / diff of the frame RMS).  ``analyze_batch`` does any
number of files in one launch.

``compare_and_print`` / ``_format_quality_note`` (spectral.py:113-359) are
host-side report formatting; the text is the reference's, line for line.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np


@dataclass
class SpectralStats:
    """spectral.py:20-33 (same fields, same order)."""
    centroid: float
    rolloff: float
    rms_mean: float
    rms_variance: float
    sub_bass: float
    bass: float
    midrange: float
    presence: float
    brilliance: float
    decay_rate: float
    duration: float
    effective_bandwidth_hz: float


def analyze_batch(signals: Sequence[Tuple[np.ndarray, int]]) -> List[SpectralStats]:
    """SpectralStats of decoded (mono f32 signal, native sample rate) pairs, one device batch."""
    from .engine import get_engine
    return [SpectralStats(**d) for d in get_engine().spectral(list(signals))]


def analyze_arrays(y: np.ndarray, sr: int) -> SpectralStats:
    return analyze_batch([(y, sr)])[0]


def analyze(path: str, label: Optional[str] = None) -> SpectralStats:
    """Load *path* at its own sample rate and return its spectral statistics (spectral.py:38-103)."""
    from .io import load_audio
    if label:
        print(f"  Loading {label}…")
    y, sr = load_audio(path, sr=None)
    return analyze_arrays(y, sr)


# ---------------------------------------------------------------------------- report
def _pct(a: float, b: float) -> float:
    """Percentage change from a to b (spectral.py:108-110)."""
    return ((b - a) / a) * 100 if a != 0 else 0.0


_RULE = "=" * 57
_BANDS = (("Sub-bass  (20–80 Hz)", "sub_bass"), ("Bass      (80–250 Hz)", "bass"),
          ("Midrange  (250–2 kHz)", "midrange"), ("Presence  (2–6 kHz)", "presence"),
          ("Brilliance (6–20 kHz)", "brilliance"))


def _verdicts(ref: SpectralStats, other: SpectralStats):
    """The percentage changes every section and the summary share."""
    return {"bd": _pct(ref.centroid, other.centroid), "rd": _pct(ref.rolloff, other.rolloff),
            "vd": _pct(ref.rms_variance, other.rms_variance), "dd": _pct(ref.decay_rate, other.decay_rate),
            "brill": _pct(ref.brilliance, other.brilliance), "dur": abs(other.duration - ref.duration),
            "reverb": other.decay_rate > ref.decay_rate * 0.8}


def _report_lines(ref, other, lr, lo):
    v = _verdicts(ref, other)
    bd, rd, vd, dd = v["bd"], v["rd"], v["vd"], v["dd"]
    slow_decay = v["reverb"] and abs(dd) > 20
    yield from ("", _RULE, "SPECTRAL COMPARISON RESULTS", f"  Reference : {lr}", f"  Other     : {lo}", _RULE)

    yield "\nBRIGHTNESS (Spectral Centroid)"
    yield f"  {lr}: {ref.centroid:.1f} Hz  |  {lo}: {other.centroid:.1f} Hz"
    yield (f"  ! {lo} is {abs(bd):.1f}% DARKER  -> likely low-pass filter applied" if bd < -10 else
           f"  ! {lo} is {bd:.1f}% BRIGHTER  -> likely high-pass or treble boost" if bd > 10 else
           f"  OK  Similar brightness ({bd:+.1f}%)")

    yield "\nHIGH FREQUENCY ROLLOFF"
    yield f"  {lr}: {ref.rolloff:.1f} Hz  |  {lo}: {other.rolloff:.1f} Hz"
    yield (f"  ! {lo} has {abs(rd):.1f}% less high-frequency energy  -> treble cut confirmed" if rd < -10 else
           f"  ! {lo} has {rd:.1f}% more high-frequency energy  -> treble boost" if rd > 10 else
           f"  OK  Similar high-frequency content ({rd:+.1f}%)")

    yield "\nDYNAMIC RANGE (Compression)"
    yield f"  {lr} variance: {ref.rms_variance:.6f}  |  {lo}: {other.rms_variance:.6f}"
    yield (f"  ! {lo} is {abs(vd):.1f}% more compressed  -> heavy limiting/compression" if vd < -30 else
           f"  ! {lo} is {abs(vd):.1f}% more compressed  -> moderate compression" if vd < -10 else
           f"  ! {lo} has {vd:.1f}% MORE dynamic range  -> less compressed than reference" if vd > 30 else
           f"  OK  Similar dynamic range ({vd:+.1f}%)")

    yield "\nFREQUENCY BAND BREAKDOWN"
    for title, field in _BANDS:
        diff = _pct(getattr(ref, field), getattr(other, field))
        tag = "OK" if abs(diff) < 10 else "! "
        yield f"  {tag}  {title}: {diff:+.1f}% ({'more' if diff > 0 else 'less'} in {lo})"

    yield "\nREVERB / DECAY"
    yield (f"  ! {lo} decays more slowly ({dd:+.1f}%)  -> possible reverb added" if slow_decay else
           f"  OK  Similar decay characteristics ({dd:+.1f}%)")

    if v["dur"] > 1.0:
        yield "\nDURATION NOTE"
        yield f"  {lr}: {ref.duration:.1f} s  |  {lo}: {other.duration:.1f} s"
        yield f"  ! Files differ by {v['dur']:.1f} s  -> different edits, fade-in/out, or intro/outro"

    yield from ("", _RULE, "SUMMARY", _RULE)
    issues = []
    if bd < -10:
        issues.append(f"low-pass filter ({abs(bd):.0f}% darker)")
    elif bd > 10:
        issues.append(f"treble boost ({bd:.0f}% brighter)")
    if rd < -10:
        issues.append(f"treble cut ({abs(rd):.0f}% rolloff reduction)")
    if vd < -10:
        kind = "heavy" if vd < -30 else "moderate"
        issues.append(f"{kind} compression ({abs(vd):.0f}% less dynamic range)")
    if v["brill"] < -20:
        issues.append(f"reduced high-frequency content ({abs(v['brill']):.0f}% less brilliance"
                      " — consistent with MP3 compression)")
    if slow_decay:
        issues.append("slower decay (possible reverb)")
    if v["dur"] > 1.0:
        issues.append(f"duration mismatch ({v['dur']:.1f} s — different edits)")
    if issues:
        yield f"Detected differences in {lo}:"
        yield from (f"  - {item}" for item in issues)
    else:
        yield "No significant spectral differences detected."


def compare_and_print(ref: SpectralStats, other: SpectralStats, label_ref: str = "REFERENCE",
                      label_other: str = "OTHER", ref_path: Optional[str] = None,
                      other_path: Optional[str] = None) -> None:
    """Print the plain-English spectral comparison report (spectral.py:113-249)."""
    for line in _report_lines(ref, other, label_ref, label_other):
        print(line)
    _format_quality_note(ref_path, other_path, ref.brilliance, other.brilliance, label_ref, label_other,
                         ref_bandwidth=ref.effective_bandwidth_hz, other_bandwidth=other.effective_bandwidth_hz)


_LOSSLESS = frozenset({"flac", "wav", "aiff", "aif", "pcm"})
# lossy-transcode grades by effective bandwidth (spectral.py:286-298): MP3 128k cuts near 16 kHz,
# 192k near 18 kHz, 320k near 20 kHz; at or above 20 kHz the content looks genuinely lossless
_GRADES = ((16_500, "MP3 ~128 kbps"), (18_500, "MP3 ~192 kbps"), (20_000, "MP3 ~320 kbps"))


def _transcode_grade(bw: Optional[float]) -> Optional[str]:
    if bw is None:
        return None
    return next((name for edge, name in _GRADES if bw < edge), None)


def _format_quality_note(ref_path: Optional[str], other_path: Optional[str], ref_brilliance: float,
                         other_brilliance: float, label_ref: str, label_other: str,
                         ref_bandwidth: Optional[float] = None,
                         other_bandwidth: Optional[float] = None) -> None:
    """Container + measured-bandwidth quality note (spectral.py:252-359)."""
    if not ref_path or not other_path:
        return

    def ext(p) -> str:
        return str(p).rsplit(".", 1)[-1].lower() if "." in str(p) else "?"

    sides = []
    for label, path, bw in ((label_ref, ref_path, ref_bandwidth), (label_other, other_path, other_bandwidth)):
        fmt = ext(path)
        lossless = fmt in _LOSSLESS
        grade = _transcode_grade(bw) if lossless else None
        sides.append({"label": label, "fmt": fmt, "container": lossless, "grade": grade, "bw": bw,
                      "true": lossless and grade is None})
    r, o = sides
    print()
    print("FORMAT / QUALITY NOTE")
    print(f"  Container: {label_ref} → {r['fmt'].upper()}   |   {label_other} → {o['fmt'].upper()}")
    if ref_bandwidth and other_bandwidth:
        print(f"  Effective bandwidth: {label_ref} → {ref_bandwidth/1000:.1f} kHz   |   "
              f"{label_other} → {other_bandwidth/1000:.1f} kHz")
    for s in sides:
        if s["container"] and s["grade"] and s["bw"]:
            shown = r["fmt"] if s["label"] == label_ref else o["fmt"]     # the reference keys this on the label
            print(f"  ! {s['label']} ({shown.upper()}) — spectral content cuts off at ~{s['bw']/1000:.1f} kHz, "
                  f"consistent with {s['grade']} encoding. This file appears to be a lossy-to-lossless "
                  f"transcode; the lossless container does NOT guarantee lossless audio.")
    if r["true"] and not o["true"]:
        print(f"  Verdict: {label_ref} is genuinely lossless — {label_other} is lower quality.")
    elif o["true"] and not r["true"]:
        print(f"  Verdict: {label_other} is genuinely lossless but {label_ref} is not — "
              f"check that files are in the correct order.")
    elif not r["true"] and not o["true"]:
        print("  Verdict: Neither file appears to be a genuine lossless master.")
    else:
        print("  Verdict: Both files appear to be genuinely lossless.")
    if r["true"] and not o["true"] and _pct(ref_brilliance, other_brilliance) > 20:
        print(f"  Warning: {label_other} (lower quality by format) has more high-frequency "
              f"content than {label_ref}. The files may be in the wrong order.")
