"""GPU parity of the engine's batched, multi-group path: the one bench.py times
(BASELINE config 3: 64 three-minute pairs per GPU).

``Engine.analyze`` splits a batch of more than 16 pairs into pair groups (16/16/16/16
for 64), runs the silence trim in two launches (the first group's files, then the
rest on the tail stream), keeps up to GROUPS_IN_FLIGHT groups queued and recycles
the piptrack peak lists through a ring of GROUPS_IN_FLIGHT + 1 workspaces
(engine.py ``_analyze`` / ``_launch_group``).  None of that runs for B <= 16, so
these tests check, on batches that take it:

* every pair of the config-3 batch equals its own B = 1 run (results, report
  text, logs, chunk lags, tempo margins), and all 64 pairs equal the CPU oracle
  (oracle/refglue.run_arrays: the port of pipeline.py:23-216), run in a process
  pool that starts with the module so it overlaps the GPU tests;
* every PIPELINE_CASES golden (the reference's own pipeline.run outputs) inside a
  17-pair batch, with the default schedule (one group), group_pairs=9 (9/8) and group_pairs=2 (9 groups, more
  than the peak ring's max(GROUPS_IN_FLIGHT, MAX_GROUPS_IN_FLIGHT) + 1 = 6 slots, the
  ring reset before the call so it wraps within it), equals the fixture field for
  field, including str(result), the logs and the CLI JSON.
"""
import dataclasses
import math
import multiprocessing as mp
import os

import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E
from nightcore_analyzer import export, synth
from nightcore_analyzer.cli import output_dict

from golden.cases import PIPELINE_CASES, make_case

pytestmark = pytest.mark.gpu

N_PAIRS = 64          # BASELINE config 3
N_LOAD_LINES = 4      # pipeline.run's "Loading ..." lines come from the caller (pipeline._load)


def _gen(seed):
    return synth.make_pair(180.0, seed)


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return E.get_engine(0)


def _oracle(seed):
    from oracle import refglue
    nc, src = _gen(seed)
    return refglue.run_arrays(nc, src, compute_ibi=False)


def oracle_pool(seeds, reserve: int = 2):
    """(pool, AsyncResult) of refglue.run_arrays(compute_ibi=False) over the synthetic
    3-min pairs of `seeds`: one single-threaded process per host core of this process
    (os.sched_getaffinity: the box's CPU share), `reserve` cores left to the test process.
    spawn: the children never touch the GPU and start from a clean interpreter."""
    n = max(1, min(len(seeds), len(os.sched_getaffinity(0)) - reserve))
    keys = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")
    saved = {k: os.environ.get(k) for k in keys}
    os.environ.update({k: "1" for k in keys})          # inherited by the children at spawn
    try:
        pool = mp.get_context("spawn").Pool(n)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return pool, pool.map_async(_oracle, list(seeds), chunksize=1)


def check_against_oracle(o: E.PairOutcome, pair, ref: dict, tag="", ibi: bool = False):
    """One outcome against refglue.run_arrays of the same pair: tempo lists, chunk lags, nc
    prior, ratios, CIs, classification, counts, exact duration ratio; with ``ibi`` (outcomes of
    run()'s defaults) also the hop-64 IBI ratio and its CI."""
    assert o.error is None, (tag, o.error)
    r, d = o.result, o.detail
    assert r.src_tempos_raw == ref["src_tempos"] and r.nc_tempos_raw == ref["nc_tempos"], tag
    assert d["chunk_lags"] == ref["chunk_lags"], tag
    assert d["nc_start_bpm"] == ref["nc_start_bpm"], tag
    for k in ("tempo_ratio", "pitch_ratio", "classification", "n_source_tempo_windows", "n_nc_tempo_windows",
              "nc_median_bpm", "src_median_bpm"):
        assert getattr(r, k) == ref[k], (tag, k)
    assert tuple(r.tempo_ci) == tuple(ref["tempo_ci"]) and tuple(r.pitch_ci) == tuple(ref["pitch_ci"]), tag
    nc, src = pair
    assert r.src_duration / r.nc_duration == len(src) / len(nc)          # exact sample-count ratio
    if ibi:
        assert r.ibi_ratio == ref["ibi_ratio"], (tag, "ibi_ratio", r.ibi_ratio, ref["ibi_ratio"])
        assert (None if r.ibi_ci is None else tuple(r.ibi_ci)) == \
            (None if ref["ibi_ci"] is None else tuple(ref["ibi_ci"])), (tag, "ibi_ci")


@pytest.fixture(scope="module")
def oracle_results():
    """The oracle on all 64 config-3 pairs, started with the module's first test."""
    pool, res = oracle_pool([1000 + i for i in range(N_PAIRS)])
    yield res
    pool.terminate()
    pool.join()


@pytest.fixture(scope="module")
def bench_pairs(oracle_results):
    # spawn: the children never touch the GPU and start from a clean interpreter
    with mp.get_context("spawn").Pool(8) as pool:
        return pool.map(_gen, [1000 + i for i in range(N_PAIRS)])


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if isinstance(x, float) and not math.isfinite(x):
        return repr(x)
    if isinstance(x, np.ndarray):
        return _norm(x.tolist())
    return x


def _key(o: E.PairOutcome):
    """Everything a caller can observe of one pair's outcome."""
    d = {k: _norm(v) for k, v in o.detail.items()}
    if o.error is not None:
        return ("error", type(o.error).__name__, str(o.error), o.logs, d)
    return ("ok", _norm(dataclasses.asdict(o.result)), str(o.result), o.logs, d)


def test_group_schedule_is_multi_group():
    assert [b - a for a, b in E._group_bounds(N_PAIRS, None)] == [32, 32]
    ring = max(E.Engine.GROUPS_IN_FLIGHT, E.Engine.MAX_GROUPS_IN_FLIGHT) + 1
    assert len(E._group_bounds(17, 2)) == 9 > ring + 1


def test_config3_batch_equals_single_pair_runs(eng, bench_pairs):
    p = E.Params(compute_ibi=False)                       # the bench's step
    outs = eng.analyze(bench_pairs, p)
    assert len(outs) == N_PAIRS
    for i, (pair, o) in enumerate(zip(bench_pairs, outs)):
        assert o.error is None, (i, o.error)
        single, = eng.analyze([pair], p)
        assert _key(o) == _key(single), f"pair {i} differs from its B=1 run"
    # the same batch again (workspaces, peak ring and pinned buffers reused): identical
    again = eng.analyze(bench_pairs, p)
    assert [_key(o) for o in again] == [_key(o) for o in outs]


def _kw_classes():
    out = {}
    for name, _, _, _, kw, _ in PIPELINE_CASES:
        out.setdefault(tuple(sorted(kw.items())), []).append(name)
    return sorted(out.items(), key=lambda kv: kv[1][0])


@pytest.mark.parametrize("group_pairs", [None, 2, 9])
@pytest.mark.parametrize("kw_names", _kw_classes(), ids=lambda kv: "+".join(kv[1]))
def test_goldens_inside_multi_group_batch(eng, bench_pairs, golden_pipeline, kw_names, group_pairs):
    kwkey, names = kw_names
    kw = dict(kwkey)
    p = E.Params(**kw)                                     # run()'s defaults + this case's kwargs
    cases = [make_case(synth, n)[:2] for n in names]
    pad = bench_pairs[:17 - len(cases)]
    # goldens first, in the middle and last: each lands in a different group
    batch = list(pad)
    slots = [0, len(batch) // 2, len(batch)][:len(cases)]
    for s, c in sorted(zip(slots, cases), key=lambda t: -t[0]):
        batch.insert(s, c)
    pos = {}
    for n, c in zip(names, cases):
        pos[n] = next(j for j, b in enumerate(batch) if b is c)
    assert len(batch) >= 17
    eng._peak_ring = -1                 # the ring's slot 0 first: 9 groups wrap it within this call
    outs = eng.analyze(batch, p, group_pairs=group_pairs)
    for n in names:
        g = golden_pipeline[n]
        o = outs[pos[n]]
        assert o.logs == g["log"][N_LOAD_LINES:], n
        if "error" in g:
            assert o.error is not None and type(o.error).__name__ == g["error"]["type"], n
            assert str(o.error) == g["error"]["message"], n
            continue
        assert o.error is None, (n, o.error)
        r, exp = o.result, g["result"]
        got = _norm({k: getattr(r, k) for k in exp})
        for k in exp:
            assert got[k] == exp[k], (n, k)
        assert str(r) == g["str"], n
        assert _norm(export.to_dict(r)) == g["export_dict"], n
        if "cli_json" in g:
            assert _norm(output_dict(r)) == g["cli_json"], n
    # the padding pairs equal their own B = 1 runs under the same parameters
    for j, pair in enumerate(batch):
        if any(pair is c for c in cases):
            continue
        if j % 4:                                          # a sample keeps the test short
            continue
        single, = eng.analyze([pair], p)
        assert _key(outs[j]) == _key(single), j


def test_streamed_logs_equal_outcome_logs(eng, bench_pairs, golden_pipeline):
    """Engine.analyze(log=...) emits every pair's lines stage by stage while the groups run
    (run() / run_batch forward them live, as the reference logs while it works): per pair,
    the streamed lines are exactly the outcome's logs, the goldens' lines included, and
    the results equal the unstreamed run."""
    names = ["chords80", "sweep30", "sweep30_nc_tail_quiet"]
    batch = [make_case(synth, n)[:2] for n in names] + list(bench_pairs[:15])
    got = {}
    outs = eng.analyze(batch, E.Params(), group_pairs=4, log=lambda i, line: got.setdefault(i, []).append(line))
    ref = eng.analyze(batch, E.Params(), group_pairs=4)
    assert sorted(got) == list(range(len(batch)))
    for i, (o, r) in enumerate(zip(outs, ref)):
        assert got[i] == o.logs == r.logs, i
        assert _key(o) == _key(r), i
    for i, n in enumerate(names):
        assert got[i] == golden_pipeline[n]["log"][N_LOAD_LINES:], n


def test_pipelined_batches_equal_separate_calls(eng, bench_pairs):
    """Engine.analyze_batches (bench.py's timed loop): batch k + 1's trims and first groups
    are queued while batch k's last groups run (trims on their own stream).  Every batch's
    outcomes equal its own analyze call, for multi-group batches (split trim), a single-group
    batch and a repeated batch."""
    p = E.Params(compute_ibi=False)
    flat = lambda prs: [a for nc, src in prs for a in (nc, src)]
    a = eng.upload_signals(flat(bench_pairs[:40]))      # two groups of the default schedule (20/20)
    b = eng.upload_signals(flat(bench_pairs[40:45]))
    c = eng.upload_signals(flat(bench_pairs[45:64]))
    batches = [a, b, c, a]
    got = eng.analyze_batches(batches, p)
    assert len(got) == len(batches)
    for sig, outs in zip(batches, got):
        ref = eng.analyze(signals=sig, params=p)
        assert [_key(o) for o in outs] == [_key(o) for o in ref]
    # with a small group size: many groups per batch, more than the peak ring's slots
    got3 = eng.analyze_batches([a, c], p, group_pairs=3)
    assert [_key(o) for o in got3[0]] == [_key(o) for o in eng.analyze(signals=a, params=p)]
    assert [_key(o) for o in got3[1]] == [_key(o) for o in eng.analyze(signals=c, params=p)]


@pytest.mark.timeout(600)
def test_config3_batch_matches_oracle(eng, bench_pairs, oracle_results):
    """every one of the 64 config-3 pairs against the CPU oracle, not 2
    (last in the module: the pool has been running beside the tests above)."""
    outs = eng.analyze(bench_pairs, E.Params(compute_ibi=False))
    refs = oracle_results.get(timeout=600)
    assert len(refs) == len(outs) == N_PAIRS
    for i, (o, pair, ref) in enumerate(zip(outs, bench_pairs, refs)):
        check_against_oracle(o, pair, ref, tag=f"pair {i}")
        assert o.result.src_duration / o.result.nc_duration == 1.25
