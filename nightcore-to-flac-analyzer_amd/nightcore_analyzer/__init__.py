"""nightcore_analyzer — MI355X-native drop-in for Tealdragon204/nightcore-to-flac-analyzer.

Same public surface as the reference package (``__init__.py:20-26``):
``run`` (= ``pipeline.run``), ``AnalysisResult``, ``export``, ``session``,
``__version__``; plus ``analyze`` (alias of ``run``) and ``run_batch``.
All analysis arithmetic runs in hand-written HIP kernels for gfx950
(``_lib/libncgpu.so``, C ABI in ``include/ncgpu.h``); there is no CPU path.
"""
from .pipeline import analyze, run, run_batch
from .consensus import AnalysisResult
from . import export
from . import session

__version__ = "0.3.0"
__all__ = ["run", "analyze", "run_batch", "AnalysisResult", "export", "session"]
