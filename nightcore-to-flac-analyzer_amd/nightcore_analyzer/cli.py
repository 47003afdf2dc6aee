"""Command-line interface (same flags, exit codes and JSON as the reference's
cli.py:25-202).

    python -m nightcore_analyzer.cli --nightcore nc.wav --source src.wav -o results.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

from . import pipeline
from .io import ENERGY_GATE_DB, HOP_SEC, SILENCE_STRIP_DB, WINDOW_SEC


def _build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        prog="python -m nightcore_analyzer.cli",
        description=("Extract the precise tempo ratio and pitch ratio between a nightcore track and its "
                     "FLAC source, then emit the Rubber Band parameters needed to reconstruct the original."),
        formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--nightcore", "-n", required=True, metavar="FILE", help="Nightcore audio file")
    p.add_argument("--source", "-s", required=True, metavar="FILE", help="Source (original) audio file")
    p.add_argument("--output", "-o", metavar="FILE", help="Write JSON results to this file (default: stdout)")
    p.add_argument("--window", type=float, default=WINDOW_SEC, metavar="SEC",
                   help="Analysis window duration in seconds")
    p.add_argument("--hop", type=float, default=HOP_SEC, metavar="SEC",
                   help="Hop between consecutive windows in seconds (< --window for overlap)")
    p.add_argument("--energy-gate", type=float, default=ENERGY_GATE_DB, metavar="DB",
                   help="Discard windows whose RMS energy is below peak + ENERGY_GATE dB")
    p.add_argument("--silence-strip-db", type=float, default=SILENCE_STRIP_DB, metavar="DB",
                   help="Top-dB threshold for trimming leading/trailing silence")
    p.add_argument("--no-silence-strip", action="store_true", help="Disable silence stripping entirely.")
    p.add_argument("--src-trim-sec", type=float, default=0.0, metavar="SEC",
                   help="Manually trim this many seconds from the start of the source")
    p.add_argument("--auto-align", action="store_true", default=False,
                   help="Attempt automatic intro-offset detection (RMS envelope correlation)")
    p.add_argument("--quiet", "-q", action="store_true", help="Suppress progress output")
    return p


def output_dict(result) -> dict:
    """cli.py:171-184 output schema (8-dp rounding; no IBI/xcorr/pitch_method)."""
    return {
        "classification": result.classification,
        "tempo_ratio": round(result.tempo_ratio, 8),
        "pitch_ratio": round(result.pitch_ratio, 8),
        "tempo_ci_95": [round(result.tempo_ci[0], 8), round(result.tempo_ci[1], 8)],
        "pitch_ci_95": [round(result.pitch_ci[0], 8), round(result.pitch_ci[1], 8)],
        "windows_used": {
            "source_pitch": result.n_source_pitch_windows,
            "nightcore_pitch": result.n_nc_pitch_windows,
            "source_tempo": result.n_source_tempo_windows,
            "nightcore_tempo": result.n_nc_tempo_windows,
        },
        "rubberband": result.rubberband,
    }


def main(argv: list[str] | None = None) -> int:
    args = _build_parser().parse_args(argv)
    nc_path, src_path = Path(args.nightcore), Path(args.source)
    errors = []
    if not nc_path.exists():
        errors.append(f"Nightcore file not found: {nc_path}")
    if not src_path.exists():
        errors.append(f"Source file not found:    {src_path}")
    if args.hop >= args.window:
        errors.append("--hop must be less than --window for overlapping windows")
    if errors:
        for e in errors:
            print(f"ERROR: {e}", file=sys.stderr)
        return 2
    log = None if args.quiet else print
    try:
        result = pipeline.run(str(nc_path), str(src_path), window_sec=args.window, hop_sec=args.hop,
                              energy_gate_db=args.energy_gate,
                              silence_strip_db=None if args.no_silence_strip else args.silence_strip_db,
                              src_trim_sec=args.src_trim_sec,
                              auto_align=args.auto_align and args.src_trim_sec == 0.0, log=log)
    except Exception as exc:
        print(f"\nERROR: {exc}", file=sys.stderr)
        return 1
    text = json.dumps(output_dict(result), indent=2)
    if args.output:
        out = Path(args.output)
        out.write_text(text, encoding="utf-8")
        if not args.quiet:
            print(f"\nResults written to: {out}")
    else:
        print()
        print(text)
    if not args.quiet:
        print()
        print(result)
    return 0


if __name__ == "__main__":
    sys.exit(main())
