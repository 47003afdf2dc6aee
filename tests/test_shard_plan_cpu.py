"""sharded.shard_plan is vectorised with numpy; this pins it to the per-pair loop form it
replaced (restated below) on random batches: every field of the plan, and the rank queries."""
import numpy as np
import pytest

from nightcore_analyzer import engine as E
from nightcore_analyzer import sharded as S


def plan_loops(lengths, p, world, split_offset=0.0):
    L = np.asarray(lengths, np.int64)
    B = len(L) // 2
    win_n, hop_n = int(p.window_sec * S.SR), int(p.hop_sec * S.SR)
    cn = int(S.CHUNK_SEC * S.SR)
    slots = np.zeros((B, 3), np.int64)
    for b in range(B):
        ln, ls = int(L[2 * b]), int(L[2 * b + 1])
        slots[b] = (S.n_window_slots(ls, win_n, hop_n), S.n_window_slots(ln, win_n, hop_n),
                    max(1, min(ls // cn, ln // cn)) if p.compute_pitch else 0)
    cost = slots[:, 0] + slots[:, 1] + S.CP_COST * slots[:, 2]
    base = np.concatenate([[0], np.cumsum(cost)]).astype(np.int64)
    T = int(base[-1])
    bounds = np.array([T * r // world for r in range(world + 1)], np.int64)
    if split_offset and B:
        shift = int(round(split_offset * T / B))
        bounds[1:world] = np.clip(bounds[1:world] + shift, 0, T)
    bounds = np.maximum.accumulate(bounds)
    bounds[world] = np.iinfo(np.int64).max // 4
    rng = np.zeros((B, 3, world, 2), np.int64)
    for b in range(B):
        u0 = (base[b], base[b] + slots[b, 0], base[b] + slots[b, 0] + slots[b, 1])
        for s, stride in ((0, 1), (1, 1), (2, S.CP_COST)):
            n = int(slots[b, s])
            for r in range(world):
                lo = -(-(int(bounds[r]) - int(u0[s])) // stride)
                hi = -(-(int(bounds[r + 1]) - int(u0[s])) // stride)
                rng[b, s, r] = (min(n, max(0, lo)), min(n, max(0, hi)))
    owner = np.array([int(min(world - 1, max(0, np.searchsorted(bounds, min(int(base[b]), max(T - 1, 0)),
                                                                 side="right") - 1))) for b in range(B)], np.int64)
    split = np.zeros(B, bool)
    for b in range(B):
        split[b] = any(rng[b, s, r, 1] > rng[b, s, r, 0] for s in range(3) for r in range(world) if r != owner[b])
    wrow = np.full(B, -1, np.int64)
    crow = np.full(B, -1, np.int64)
    nw = nc = 0
    for b in np.flatnonzero(split):
        wrow[b], crow[b] = nw, nc
        nw += int(slots[b, 0] + slots[b, 1])
        nc += int(slots[b, 2])
    return slots, rng, owner, split, wrow, crow, nw, nc


@pytest.mark.parametrize("seed", range(6))
def test_vectorised_plan_equals_loops(seed):
    rng = np.random.default_rng(seed)
    for B in (1, 3, 17, 64):
        lengths = []
        for _ in range(B):
            src = int(rng.integers(0, 2_000_000)) if rng.random() < 0.2 else int(rng.integers(200_000, 8_000_000))
            lengths += [int(src * rng.uniform(0.5, 1.0)), src]
        for world in (1, 2, 3, 8):
            for off in (0.0, 0.5, 0.3):
                for pitch in (True, False):
                    p = E.Params(compute_pitch=pitch)
                    sp = S.shard_plan(lengths, p, world, off)
                    ref = plan_loops(lengths, p, world, off)
                    for got, want in zip((sp.slots, sp.rng, sp.owner, sp.split, sp.wrow, sp.crow, sp.n_wrows,
                                          sp.n_crows), ref):
                        assert np.array_equal(np.asarray(got), np.asarray(want)), (B, world, off, pitch)
                    for r in range(world):
                        present = [b for b in range(B) if sp.on_rank(b, r)]
                        assert sp.touched(r) == sorted(set(present) | set(np.flatnonzero(sp.owner == r).tolist()))
                        assert sp.owned(r) == np.flatnonzero(sp.owner == r).tolist()
                        assert sp.needed(r, True) == sorted(set(sp.touched(r)) | set(np.flatnonzero(sp.split).tolist()))
                        assert sp.needed(r, False) == sp.touched(r)
