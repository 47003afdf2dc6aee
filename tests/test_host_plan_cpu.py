"""Host planning helpers of the pipelined engine, on the CPU: the vectorised shared-tuning
chunk map equals the per-chunk rule it replaced, and device spans address the same bytes as
the torch views they replace."""
import numpy as np
import pytest
import torch

from nightcore_analyzer import engine as E


def _loop_map(pl, tp):
    """The per-chunk rule (engine round 3): chunk i of a pair starts at i * CHUNK in its file;
    it shares its leading tuning frames with the window of that file starting there."""
    win_chunk = np.full(max(1, pl.n_win), -1, np.int32)
    tf_skip = np.zeros(max(1, pl.n_chunks), np.int32)
    cn = int(E.CHUNK_SEC * E.SR)
    for b, (c0, c1) in enumerate(pl.pair_chunks):
        for f, side in ((2 * b + 1, 0), (2 * b, 1)):
            st_f = pl.starts[f]
            for i in range(c1 - c0):
                c = 2 * (c0 + i) + side
                if pl.chunk_len[c] != cn or (i * cn) % pl.hop_n:
                    continue
                k = i * cn // pl.hop_n
                if k < len(st_f) and st_f[k] == i * cn:
                    win_chunk[pl.w0[f] + k] = c
                    tf_skip[c] = tp
    return win_chunk, tf_skip


@pytest.mark.parametrize("seed", range(12))
def test_shared_tuning_map_equals_the_per_chunk_rule(seed):
    rng = np.random.default_rng(seed)
    B = int(rng.integers(1, 9))
    secs = rng.choice([3.0, 9.0, 19.9, 20.0, 41.0, 65.0, 180.0], size=2 * B)
    length = (secs * E.SR).astype(np.int64) + rng.integers(0, 3000, size=2 * B)
    off = np.concatenate([[0], np.cumsum(length)[:-1]]).astype(np.int64)
    start = rng.integers(0, 2000, size=2 * B) * (rng.random(2 * B) < 0.5)
    end = length - rng.integers(0, 2000, size=2 * B) * (rng.random(2 * B) < 0.5)
    window, hop = [(10.0, 5.0), (10.0, 2.5), (8.0, 3.0), (20.0, 10.0), (10.0, 7.0)][seed % 5]
    p = E.Params(window_sec=window, hop_sec=hop, compute_ibi=False)
    pl = E.plan_batch(off, length, start.astype(np.int64), end.astype(np.int64), p)
    tp = 17
    want_w, want_t = _loop_map(pl, tp)
    got_w = np.full(max(1, pl.n_win), -1, np.int32)
    got_t = np.zeros(max(1, pl.n_chunks), np.int32)
    E.shared_tuning_map(pl, tp, got_w, got_t)
    np.testing.assert_array_equal(got_w, want_w)
    np.testing.assert_array_equal(got_t, want_t)
    if seed == 0:
        assert (want_t > 0).any()          # the rule fires on these plans


def test_device_spans_address_the_torch_views():
    up = E._Upload()
    up.add("a", [1, 2, 3], np.int64)
    up.add("b", [1.5], np.float64)
    up.add("c", [], np.int32)
    ar = E._Arena()
    ar.add("x", 5, np.float64)
    ar.add("y", 3, np.int32)
    o = ar.commit(torch.device("cpu"), spans=True)
    assert o["y"].data_ptr() - o["x"].data_ptr() == 48 and o["x"].numel() == 5
    s = o["x"][2:]
    assert s.data_ptr() == o["x"].data_ptr() + 16 and len(s) == 3 and len(o["x"][:0]) == 0
    o["x"][1:3].fill_(7.0)
    assert E._tensor(o["x"]).tolist() == [0.0, 7.0, 7.0, 0.0, 0.0]
    with pytest.raises(ValueError):
        o["x"][::2]
    views = E._Arena()
    views.parts = list(ar.parts)
    v = views.commit(torch.device("cpu"))
    for name in ("x", "y"):
        assert o[name].numel() == v[name].numel() and o[name].dtype == v[name].dtype
