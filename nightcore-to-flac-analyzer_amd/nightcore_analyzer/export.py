"""JSON / CSV export of an AnalysisResult (same schema as the reference's
export.py:20-98; JSON mirrors the CLI output plus warnings/durations/BPMs)."""
from __future__ import annotations

import csv
import json
from pathlib import Path
from typing import Union

from .consensus import AnalysisResult

PathLike = Union[str, Path]


def _r(x, nd):
    return round(x, nd) if x else None


def to_dict(result: AnalysisResult) -> dict:
    r = result
    both = bool(r.nc_duration and r.src_duration)
    return {
        "classification": r.classification,
        "warnings": r.warnings,
        "tempo_ratio": round(r.tempo_ratio, 8),
        "pitch_ratio": round(r.pitch_ratio, 8),
        "tempo_ci_95": [round(r.tempo_ci[0], 8), round(r.tempo_ci[1], 8)],
        "pitch_ci_95": [round(r.pitch_ci[0], 8), round(r.pitch_ci[1], 8)],
        "windows_used": {
            "source_pitch": r.n_source_pitch_windows,
            "nightcore_pitch": r.n_nc_pitch_windows,
            "source_tempo": r.n_source_tempo_windows,
            "nightcore_tempo": r.n_nc_tempo_windows,
        },
        "rubberband": r.rubberband,
        "durations": {
            "nightcore_sec": _r(r.nc_duration, 3),
            "source_sec": _r(r.src_duration, 3),
            "duration_ratio": round(r.src_duration / r.nc_duration, 8) if both else None,
        },
        "median_bpms": {
            "nightcore": _r(r.nc_median_bpm, 2),
            "source": _r(r.src_median_bpm, 2),
        },
    }


def export_json(result: AnalysisResult, path: PathLike) -> None:
    Path(path).write_text(json.dumps(to_dict(result), indent=2), encoding="utf-8")


def export_csv(result: AnalysisResult, path: PathLike) -> None:
    r, rb = result, result.rubberband
    both = bool(r.nc_duration and r.src_duration)

    def opt(x, nd):
        return round(x, nd) if x else ""

    row = {
        "classification": r.classification,
        "tempo_ratio": round(r.tempo_ratio, 8),
        "pitch_ratio": round(r.pitch_ratio, 8),
        "tempo_ci_95_lo": round(r.tempo_ci[0], 8),
        "tempo_ci_95_hi": round(r.tempo_ci[1], 8),
        "pitch_ci_95_lo": round(r.pitch_ci[0], 8),
        "pitch_ci_95_hi": round(r.pitch_ci[1], 8),
        "source_pitch_windows": r.n_source_pitch_windows,
        "nightcore_pitch_windows": r.n_nc_pitch_windows,
        "source_tempo_windows": r.n_source_tempo_windows,
        "nightcore_tempo_windows": r.n_nc_tempo_windows,
        "rb_time_ratio": rb.get("time_ratio", ""),
        "rb_pitch_semitones": rb.get("pitch_semitones", ""),
        "rb_nc_to_source_speed": rb.get("nc_to_source_speed", ""),
        "rb_cli_command": rb.get("cli_command", ""),
        "rb_dur_time_ratio": rb.get("duration_time_ratio", ""),
        "rb_dur_pitch_semitones": rb.get("duration_pitch_semitones", ""),
        "rb_dur_cli_command": rb.get("duration_cli_command", ""),
        "nc_median_bpm": opt(r.nc_median_bpm, 2),
        "src_median_bpm": opt(r.src_median_bpm, 2),
        "nc_duration_sec": opt(r.nc_duration, 3),
        "src_duration_sec": opt(r.src_duration, 3),
        "duration_ratio": round(r.src_duration / r.nc_duration, 8) if both else "",
        "warnings": " | ".join(r.warnings),
    }
    with open(path, "w", newline="", encoding="utf-8") as fh:
        w = csv.DictWriter(fh, fieldnames=list(row.keys()))
        w.writeheader()
        w.writerow(row)
