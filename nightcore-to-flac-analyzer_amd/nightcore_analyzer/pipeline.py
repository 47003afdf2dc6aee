"""Full windowed consensus pipeline (drop-in for the reference's
nightcore_analyzer/pipeline.py).

``run`` keeps the reference's exact signature and behaviour (pipeline.py:23-216):
load -> strip silence -> source trim -> windows -> energy gate -> pitch (chroma
xcorr) -> source tempo -> nc tempo prior -> nc tempo -> consensus -> IBI ratio,
with the same log lines and the same exceptions (RuntimeError when every
window is gated out, ValueError when fewer than 3 valid tempo windows).  All
analysis arithmetic runs on the MI355X through ``libncgpu``; ``run_batch``
analyses many pairs in one device batch (the reference has no batch API, its
``run`` is a batch of one); ``analyze`` is an alias of ``run``.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple, Union

import numpy as np

from .consensus import AnalysisResult
from .io import ENERGY_GATE_DB, HOP_SEC, SILENCE_STRIP_DB, WINDOW_SEC, load_audio

PathOrArray = Union[str, np.ndarray]


def _params(window_sec, hop_sec, energy_gate_db, silence_strip_db, src_trim_sec, auto_align, compute_pitch,
            compute_ibi=True):
    from .engine import Params
    return Params(window_sec=window_sec, hop_sec=hop_sec, energy_gate_db=energy_gate_db,
                  silence_strip_db=silence_strip_db, src_trim_sec=src_trim_sec, auto_align=auto_align,
                  compute_pitch=compute_pitch, compute_ibi=compute_ibi)


def _load(x: PathOrArray, log, what: str, sr: int = 22050):
    """A file decoded as load_audio does (a mono 16-bit WAV kept as its stored samples,
    io.Pcm16, and widened on the device at upload: half the PCIe bytes), or an array."""
    log(f"Loading {what} audio…")
    if isinstance(x, np.ndarray):
        y = np.ascontiguousarray(x, dtype=np.float32)
    else:
        y, sr = load_audio(x, sr=sr, keep_pcm16=True)
    log(f"  {len(y) / sr:.1f} s  ({len(y):,} samples @ {sr} Hz)")
    return y


def run(nightcore_path: str, source_path: str, *, window_sec: float = WINDOW_SEC, hop_sec: float = HOP_SEC,
        energy_gate_db: float = ENERGY_GATE_DB, silence_strip_db: Optional[float] = SILENCE_STRIP_DB,
        src_trim_sec: float = 0.0, auto_align: bool = False, compute_pitch: bool = True,
        log: Optional[Callable[[str], None]] = print) -> AnalysisResult:
    """Analyse the tempo and pitch relationship between a nightcore track and its source."""
    def _log(msg: str) -> None:
        if log is not None:
            log(msg)

    nc = _load(nightcore_path, _log, "nightcore")
    src = _load(source_path, _log, "source")
    from .engine import get_engine
    p = _params(window_sec, hop_sec, energy_gate_db, silence_strip_db, src_trim_sec, auto_align, compute_pitch)
    if compute_pitch:
        p.melodia = _melodia_hook([(nc, src)])
    # log lines stream out as the device stages complete (pipeline.py:77-215 logs as it goes;
    # the GUI worker forwards each line live, gui/worker.py:46-53)
    outcome, = get_engine().analyze([(nc, src)], p, log=(lambda i, line: _log(line)) if log is not None else None)
    if outcome.error is not None:
        raise outcome.error
    return outcome.result


analyze = run


def _melodia_hook(pairs):
    """Params.melodia for pairs of host arrays (nc, src) when MELODIA runs (essentia installed,
    or the opt-in device restatement asked for with NC_MELODIA=device; None otherwise, the
    default in this image): MELODIA on the pair's trimmed signals, then
    estimate_pitch_combined's acceptance rule (pitch.py:246-291)."""
    from . import pitch
    if pitch.melodia_backend() is None:
        return None

    def hook(b, chroma_st, log, span):         # b: pair index in `pairs`; span: trimmed (src, nc)
        from .io import as_f32
        (so, sl), (no, nl) = span
        nc, src = (as_f32(a) for a in pairs[b])
        mel = pitch.estimate_pitch_melodia(src[so:so + sl], nc[no:no + nl], 22050, log=log)
        return pitch.melodia_choice(mel, chroma_st, log)
    return hook


def run_batch(pairs: Sequence[Tuple[PathOrArray, PathOrArray]], *, window_sec: float = WINDOW_SEC,
              hop_sec: float = HOP_SEC, energy_gate_db: float = ENERGY_GATE_DB,
              silence_strip_db: Optional[float] = SILENCE_STRIP_DB, src_trim_sec: float = 0.0,
              auto_align: bool = False, compute_pitch: bool = True, compute_ibi: bool = True,
              log: Optional[Callable[[str], None]] = None) -> List[Union[AnalysisResult, BaseException]]:
    """Analyse many (nightcore, source) pairs in one GPU batch.  Returns, per
    pair, the AnalysisResult or the exception ``run`` would have raised."""
    quiet = (lambda m: None)
    arrays = [(_load(n, quiet, "nightcore"), _load(s, quiet, "source")) for n, s in pairs]
    from .engine import get_engine
    p = _params(window_sec, hop_sec, energy_gate_db, silence_strip_db, src_trim_sec, auto_align, compute_pitch,
                compute_ibi)
    if compute_pitch:
        p.melodia = _melodia_hook(arrays)
    outs = get_engine().analyze(arrays, p,
                                log=(lambda i, line: log(f"[pair {i}] {line}")) if log is not None else None)
    return [o.error if o.error is not None else o.result for o in outs]
