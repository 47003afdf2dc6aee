"""Consensus: result schema, bootstrap ratios (on the MI355X), classification,
Rubber Band parameters and sanity warnings.

Drop-in for the reference's ``nightcore_analyzer/consensus.py``:

* ``AnalysisResult`` — same fields, order, defaults and ``__str__`` report
  (consensus.py:66-232);
* ``_valid`` (:236-240), ``_classify`` (:315-336), ``_rubberband_params``
  (:339-381), ``_check_sanity`` (:384-515) — host logic, same decisions/strings;
* ``_bootstrap_ratio`` (:243-267) and ``compute_ibi_ratio`` (:270-312) — run
  by ``libncgpu`` (``nc_bootstrap_ratio``): numpy's PCG64 stream, draw order,
  medians and 'linear' percentiles reproduced bit-exactly on the device;
* ``build_result`` (:519-608) — same gates, half-time flip and outputs.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

N_BOOTSTRAP: int = 2000
CI_LEVEL: float = 0.95
PURE_NC_TOLERANCE: float = 0.02
MIN_VALID: int = 3

NIGHTCORE_RATIO_MIN: float = 1.05
NIGHTCORE_RATIO_MAX: float = 1.50
NEAR_UNITY_TOLERANCE: float = 0.05
WIDE_CI_RELATIVE: float = 2.0
DURATION_TEMPO_MISMATCH_TOLERANCE: float = 0.08


@dataclass
class AnalysisResult:
    """Full output of the windowed consensus pipeline (schema of consensus.py:66-156)."""

    tempo_ratio: float
    pitch_ratio: float
    tempo_ci: Tuple[float, float]
    pitch_ci: Tuple[float, float]
    classification: str
    n_source_pitch_windows: int
    n_nc_pitch_windows: int
    n_source_tempo_windows: int
    n_nc_tempo_windows: int
    rubberband: dict = field(default_factory=dict)
    src_pitches_raw: Optional[List[Optional[float]]] = None
    nc_pitches_raw: Optional[List[Optional[float]]] = None
    src_tempos_raw: Optional[List[Optional[float]]] = None
    nc_tempos_raw: Optional[List[Optional[float]]] = None
    nc_duration: Optional[float] = None
    src_duration: Optional[float] = None
    nc_median_bpm: Optional[float] = None
    src_median_bpm: Optional[float] = None
    warnings: List[str] = field(default_factory=list)
    pitch_method: Optional[str] = None
    ibi_ratio: Optional[float] = None
    ibi_ci: Optional[Tuple[float, float]] = None
    xcorr_ratio: Optional[float] = None
    xcorr_quality: Optional[float] = None
    intro_offset_sec: Optional[float] = None

    def __str__(self) -> str:  # report text of consensus.py:158-232
        out: List[str] = [f"WARNING  : {w}" for w in self.warnings]
        if self.warnings:
            out.append("")
        out.append(f"Classification  : {self.classification}")
        dur = ""
        if self.nc_duration and self.src_duration:
            dur = (f"  |  duration ratio {self.src_duration / self.nc_duration:.6f}×"
                   f" ({self.src_duration:.1f} s / {self.nc_duration:.1f} s)")
        lo, hi = self.tempo_ci
        out.append(f"Tempo ratio     : {self.tempo_ratio:.6f}  95% CI [{lo:.6f}, {hi:.6f}]"
                   f"  (from {self.n_source_tempo_windows} src / {self.n_nc_tempo_windows} nc windows)"
                   + dur)
        if self.n_source_pitch_windows > 0 or self.n_nc_pitch_windows > 0:
            plo, phi = self.pitch_ci
            out.append(f"Pitch ratio     : {self.pitch_ratio:.6f}  95% CI [{plo:.6f}, {phi:.6f}]"
                       f"  (from {self.n_source_pitch_windows} src / {self.n_nc_pitch_windows} nc samples)")
            if self.pitch_method:
                out.append(f"Pitch method    : {self.pitch_method}")
        else:
            out.append("Pitch ratio     : not computed in this step")
        tr = self.tempo_ratio
        if tr > 0:
            out += ["",
                    f"Speed summary   : nightcore is {tr:.4f}× the source speed",
                    f"                  to hear original tempo → play nightcore at {1.0 / tr:.4f}× speed",
                    f"                  (source was sped up by {tr:.4f}× to create the nightcore)"]
        if self.nc_median_bpm is not None and self.src_median_bpm is not None:
            out.append(f"Median BPMs     : nightcore {self.nc_median_bpm:.2f}  |"
                       f"  source {self.src_median_bpm:.2f}"
                       f"  (raw detected; ratio = {self.nc_median_bpm / self.src_median_bpm:.6f})")
        rb = self.rubberband
        out += ["",
                f"Rubber Band     : --time {rb.get('time_ratio', '?'):.6f}"
                f"  --pitch {rb.get('pitch_semitones', '?'):.4f} st  (beat-detected ratio)",
                f"CLI (detected)  : {rb.get('cli_command', '')}"]
        if rb.get("duration_time_ratio"):
            out += [f"Duration-based  : --time {rb['duration_time_ratio']:.6f}"
                    f"  --pitch {rb['duration_pitch_semitones']:.4f} st"
                    "  (uses file-length ratio — prefer this when CI is degenerate)",
                    f"CLI (duration)  : {rb.get('duration_cli_command', '')}"]
        return "\n".join(out)


# --------------------------------------------------------------------------- host decisions
def _median(values) -> float:
    """np.median of a non-empty sequence of finite floats, bit for bit: the middle
    element, or (a + b) / 2 of the two middle ones (numpy's mean of two values)."""
    v = sorted(values)
    m = len(v) // 2
    return float(v[m]) if len(v) & 1 else (float(v[m - 1]) + float(v[m])) / 2.0


def _valid(values: List[Optional[float]]) -> np.ndarray:
    """consensus.py:236-240: drop None / NaN / inf / non-positive."""
    return np.array([v for v in values if v is not None and math.isfinite(v) and v > 0],
                    dtype=np.float64)


def _valid_list(values) -> list:
    """``_valid`` as a list (same elements, same order): what ``assemble`` needs (counts and
    medians) without building four small arrays per pair on the host's assembly path."""
    isf = math.isfinite
    return [v for v in values if v is not None and isf(v) and v > 0]


def _classify(tempo_ratio: float, pitch_ratio: float, tempo_ci: Tuple[float, float],
              pitch_ci: Tuple[float, float], tol: float = PURE_NC_TOLERANCE) -> str:
    diff = pitch_ratio - tempo_ratio
    overlap = tempo_ci[0] <= pitch_ci[1] and pitch_ci[0] <= tempo_ci[1]
    if abs(diff) <= tol or (overlap and abs(diff) <= 2 * tol):
        return "pure_nightcore"
    if diff > tol:
        return "independent_pitch_shift"
    if tempo_ratio > 1.0 + tol and diff < -tol:
        return "time_stretch_only"
    return "ambiguous"


def _rb_cli(time_ratio: float, pitch_st: float) -> str:
    return f"rubberband --time {time_ratio:.6f} --pitch {pitch_st:.4f} nightcore.flac reconstructed.flac"


def _rubberband_params(tempo_ratio: float, pitch_ratio: float, nc_duration: Optional[float] = None,
                       src_duration: Optional[float] = None) -> dict:
    pitch_st = -12.0 * math.log2(pitch_ratio)
    rb = {
        "time_ratio": round(tempo_ratio, 6),
        "pitch_semitones": round(pitch_st, 4),
        "nc_to_source_speed": round(1.0 / tempo_ratio, 6) if tempo_ratio != 0 else None,
        "cli_command": _rb_cli(tempo_ratio, pitch_st),
    }
    if nc_duration and src_duration and nc_duration > 0:
        dr = src_duration / nc_duration
        dst = -12.0 * math.log2(dr)
        rb["duration_time_ratio"] = round(dr, 6)
        rb["duration_pitch_semitones"] = round(dst, 4)
        rb["duration_cli_command"] = _rb_cli(dr, dst)
    return rb


def _check_sanity(tempo_ratio: float, pitch_ratio: float, tempo_ci: Tuple[float, float],
                  pitch_ci: Tuple[float, float], nc_duration: Optional[float] = None,
                  src_duration: Optional[float] = None, tempo_was_corrected: bool = False) -> List[str]:
    """consensus.py:384-515 — the same checks, in the same order, same wording."""
    w: List[str] = []
    have_dur = nc_duration is not None and src_duration is not None
    if tempo_was_corrected:
        w.append(
            "Beat-tracker half-time artefact corrected: librosa returned a raw tempo "
            "ratio < 1 (nightcore beat-detected at half-time), but the nightcore file "
            f"({nc_duration:.1f} s) is shorter than the source ({src_duration:.1f} s), "
            "confirming the nightcore IS faster. The ratio has been inverted "
            f"to {tempo_ratio:.4f}× automatically. This is a known librosa artefact "
            "for high-BPM music (>~130 BPM).")
    elif have_dur:
        if abs(nc_duration / src_duration - 1.0) < NEAR_UNITY_TOLERANCE:
            w.append(
                f"Both files are nearly the same duration ({nc_duration:.1f} s vs {src_duration:.1f} s). "
                "Did you accidentally provide two nightcore files, or two originals? "
                "A real nightcore should be ~10–35 % shorter than the source.")
    else:
        if abs(tempo_ratio - 1.0) < NEAR_UNITY_TOLERANCE:
            w.append(
                f"Tempo ratio is {tempo_ratio:.4f} — both files appear to be at the "
                "same speed. Did you accidentally provide two nightcore files, or two "
                "originals? A real nightcore should be 1.05–1.50× faster than the source.")
        elif tempo_ratio < 1.0:
            w.append(
                f"Tempo ratio is {tempo_ratio:.4f} < 1.0. Two possible causes: "
                "(1) librosa half-time detection artefact — the true ratio may be "
                f"{round(1.0 / tempo_ratio, 4):.4f}× (the inverse); or (2) the files are in the wrong order. "
                "Re-run with the correct original FLAC as --source to disambiguate.")
        elif tempo_ratio > NIGHTCORE_RATIO_MAX:
            w.append(
                f"Tempo ratio is {tempo_ratio:.4f}, above the typical nightcore range "
                f"({NIGHTCORE_RATIO_MIN}–{NIGHTCORE_RATIO_MAX}×). Verify the input files.")

    if have_dur:
        dsr = src_duration / nc_duration
        disc = abs(dsr - tempo_ratio) / tempo_ratio
        if disc > DURATION_TEMPO_MISMATCH_TOLERANCE:
            w.append(
                f"Duration ratio ({dsr:.4f}×) and detected tempo ratio "
                f"({tempo_ratio:.4f}×) differ by {disc * 100:.1f}%. For a pure "
                "speed-up these should be nearly equal. Most likely cause: the two files "
                "are different edits or versions of the same song (e.g. radio edit vs. "
                "extended mix). Find the exact version used to create the nightcore, or "
                f"use the duration ratio ({dsr:.4f}×) directly as the "
                "rubberband --time factor.")

    if abs(tempo_ci[1] - tempo_ci[0]) < 0.001:
        if have_dur and nc_duration > 0:
            dsr = src_duration / nc_duration
            mism = abs(tempo_ratio - dsr) / dsr
            if mism < DURATION_TEMPO_MISMATCH_TOLERANCE:
                w.append(
                    f"Tempo CI is degenerate [lo = hi = {tempo_ci[0]:.6f}]: every "
                    "analysis window returned the same BPM. This is expected for "
                    "constant-tempo music (drum machine / eurodance). The detected "
                    f"ratio ({tempo_ratio:.4f}×) agrees with the duration ratio "
                    f"({dsr:.4f}×) — result is reliable.")
            else:
                w.append(
                    f"Tempo CI is degenerate [lo = hi = {tempo_ci[0]:.6f}] and the "
                    f"detected ratio ({tempo_ratio:.4f}×) disagrees with the duration "
                    f"ratio ({dsr:.4f}×) by {mism * 100:.1f}%. "
                    "This is a librosa BPM quantisation artefact — the beat tracker "
                    "snapped all windows to the same wrong grid BPM. "
                    "Use the 'Duration-based' CLI command instead of 'CLI (detected)'.")
        else:
            w.append(
                f"Tempo CI is degenerate [lo = hi = {tempo_ci[0]:.6f}]: every "
                "analysis window returned the same BPM from librosa. This may be a "
                "quantisation artefact (beat tracker snapped to a fixed grid BPM) or "
                "simply a constant-tempo track. Provide both file durations to "
                "distinguish the two cases.")

    if pitch_ratio > 0 and (pitch_ci[1] - pitch_ci[0]) > WIDE_CI_RELATIVE * pitch_ratio:
        w.append(
            f"Pitch CI is very wide ({pitch_ci[0]:.3f}–{pitch_ci[1]:.3f}) relative "
            f"to the point estimate ({pitch_ratio:.4f}). The pitch estimator could "
            "not reliably determine a consistent pitch ratio — this is common with "
            "polyphonic or heavily processed audio. "
            "Trust the tempo ratio; treat the pitch ratio and classification as "
            "approximate.")
    return w


def insufficient_tempo_error(n_src: int, n_nc: int) -> ValueError:
    return ValueError(f"Insufficient valid tempo windows (source: {n_src}, "
                      f"nightcore: {n_nc}).  Need ≥ {MIN_VALID} each.")


def assemble(src_pitches, nc_pitches, src_tempos, nc_tempos, *, nc_duration, src_duration,
             pitch_boot: Optional[Tuple[float, Tuple[float, float]]],
             tempo_boot: Tuple[float, Tuple[float, float]]) -> AnalysisResult:
    """build_result (consensus.py:519-608) after the bootstraps: gates, half-time
    flip, medians, classification, Rubber Band parameters, warnings."""
    src_p, nc_p, src_t, nc_t = (_valid_list(src_pitches), _valid_list(nc_pitches), _valid_list(src_tempos),
                                _valid_list(nc_tempos))
    if len(src_t) < MIN_VALID or len(nc_t) < MIN_VALID:
        raise insufficient_tempo_error(len(src_t), len(nc_t))
    if len(src_p) >= MIN_VALID and len(nc_p) >= MIN_VALID:
        pitch_ratio, pitch_ci = pitch_boot
        n_sp, n_np = len(src_p), len(nc_p)
    else:
        pitch_ratio, pitch_ci, n_sp, n_np = 1.0, (1.0, 1.0), 0, 0
    tempo_ratio, tempo_ci = tempo_boot
    corrected = False
    if (nc_duration is not None and src_duration is not None
            and nc_duration < src_duration * 0.99 and tempo_ratio < 1.0):
        tempo_ratio = 1.0 / tempo_ratio
        tempo_ci = (1.0 / tempo_ci[1], 1.0 / tempo_ci[0])
        corrected = True
    nc_med = _median(nc_t) if len(nc_t) > 0 else None
    src_med = _median(src_t) if len(src_t) > 0 else None
    return AnalysisResult(
        tempo_ratio=tempo_ratio, pitch_ratio=pitch_ratio, tempo_ci=tempo_ci, pitch_ci=pitch_ci,
        classification=_classify(tempo_ratio, pitch_ratio, tempo_ci, pitch_ci),
        n_source_pitch_windows=n_sp, n_nc_pitch_windows=n_np,
        n_source_tempo_windows=len(src_t), n_nc_tempo_windows=len(nc_t),
        rubberband=_rubberband_params(tempo_ratio, pitch_ratio, nc_duration, src_duration),
        nc_duration=nc_duration, src_duration=src_duration,
        nc_median_bpm=nc_med, src_median_bpm=src_med,
        warnings=_check_sanity(tempo_ratio, pitch_ratio, tempo_ci, pitch_ci, nc_duration,
                               src_duration, corrected),
        src_pitches_raw=list(src_pitches), nc_pitches_raw=list(nc_pitches),
        src_tempos_raw=list(src_tempos), nc_tempos_raw=list(nc_tempos))


# --------------------------------------------------------------------------- GPU-backed entry points
def _bootstrap_ratio(nc_vals: np.ndarray, src_vals: np.ndarray, n_boot: int = N_BOOTSTRAP,
                     ci: float = CI_LEVEL) -> Tuple[float, Tuple[float, float]]:
    """consensus.py:243-267 on the device (draw order nc then src, seed 42)."""
    from .engine import get_engine
    return get_engine().bootstrap([(np.asarray(nc_vals, np.float64), np.asarray(src_vals, np.float64))],
                                  seed=42, n_boot=n_boot, ci=ci)[0]


def compute_ibi_ratio(nc_ibis: np.ndarray, src_ibis: np.ndarray, n_boot: int = N_BOOTSTRAP,
                      ci: float = CI_LEVEL) -> Tuple[float, Tuple[float, float]]:
    """consensus.py:270-312 on the device (draw order src then nc, seed 42)."""
    from .engine import get_engine
    return get_engine().bootstrap([(np.asarray(src_ibis, np.float64), np.asarray(nc_ibis, np.float64))],
                                  seed=42, n_boot=n_boot, ci=ci)[0]


def build_result(src_pitches: List[Optional[float]], nc_pitches: List[Optional[float]],
                 src_tempos: List[Optional[float]], nc_tempos: List[Optional[float]], *,
                 nc_duration: Optional[float] = None,
                 src_duration: Optional[float] = None) -> AnalysisResult:
    """consensus.py:519-608 (bootstraps on the device)."""
    src_p, nc_p, src_t, nc_t = (_valid(src_pitches), _valid(nc_pitches), _valid(src_tempos),
                                _valid(nc_tempos))
    if len(src_t) < MIN_VALID or len(nc_t) < MIN_VALID:
        raise insufficient_tempo_error(len(src_t), len(nc_t))
    from .engine import get_engine
    jobs = [(nc_t, src_t)]
    do_pitch = len(src_p) >= MIN_VALID and len(nc_p) >= MIN_VALID
    if do_pitch:
        jobs.insert(0, (nc_p, src_p))
    outs = get_engine().bootstrap(jobs, seed=42)
    pitch_boot = outs[0] if do_pitch else None
    return assemble(src_pitches, nc_pitches, src_tempos, nc_tempos, nc_duration=nc_duration,
                    src_duration=src_duration, pitch_boot=pitch_boot, tempo_boot=outs[-1])
