"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the MI355X engine.

Nothing in the product package (``nightcore-to-flac-analyzer_amd/``) may import,
call, link or execute anything under ``oracle/``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and
only as the checker / the timed CPU baseline.

Contents
--------
``ncref``    numpy/scipy restatement of the third-party librosa primitives the
             reference calls on its hot path (librosa is NOT installed here and
             cannot be; semantics restated for librosa 0.11.0 / 0.10.2+, see
             DESIGN.md §Oracle).  Parity vs. real librosa is UNPINNED; it is
             pinned by known-answer tests from first principles instead.
``refglue``  CPU restatement of the reference's own glue (io / tempo / pitch /
             consensus / pipeline / xcorr) on top of ``ncref``.  Pinned against
             golden fixtures produced by running the reference's own modules in
             this container (``tests/golden/make_golden.py``).
"""
