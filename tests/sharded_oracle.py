"""The stage interface of nightcore_analyzer.sharded (DeviceStages on a GPU) restated
over the CPU oracle, so the window-sharded orchestration — record exchange, energy
gate, nc prior, consensus placement, result gather — runs in multi-process gloo tests
without a GPU.  Test infrastructure only (imports oracle/)."""
from __future__ import annotations

import numpy as np

from oracle import ncref, refglue


class OracleStages:
    def __init__(self, pairs, fail_in=None):
        flat = []
        for nc, src in pairs:
            flat += [np.asarray(nc, np.float32), np.asarray(src, np.float32)]
        self.length = np.array([len(a) for a in flat], np.int64)
        self.off = np.concatenate([[0], np.cumsum(self.length)[:-1]]).astype(np.int64)
        self.buf = np.concatenate(flat) if flat else np.zeros(0, np.float32)
        self._wins = []
        self.fail_in = fail_in            # stage name that raises (error-propagation test)

    def restrict(self, files):
        """The same stages over a subset of the files (the pairs a rank touches)."""
        o = OracleStages.__new__(OracleStages)
        f = np.asarray(files, np.int64)
        o.buf, o.off, o.length, o._wins, o.fail_in = self.buf, self.off[f], self.length[f], [], self.fail_in
        return o

    def _check(self, name):
        if self.fail_in == name:
            raise RuntimeError(f"injected failure in {name}")

    def trim(self, p):
        se = [ncref.trim(self.buf[o:o + n], p.silence_strip_db)[1] for o, n in zip(self.off, self.length)]
        return np.array([s for s, _ in se], np.int64), np.array([e for _, e in se], np.int64)

    def align(self, start, end):
        out = []
        for b in range(len(self.off) // 2):
            fn, fs = 2 * b, 2 * b + 1
            src = self.buf[self.off[fs] + start[fs]:self.off[fs] + end[fs]]
            nc = self.buf[self.off[fn] + start[fn]:self.off[fn] + end[fn]]
            out.append(refglue.find_content_offset(src, nc))
        return out

    def windows(self, win_abs, win_n):
        self._check("windows")
        self._wins = [self.buf[a:a + win_n] for a in win_abs]
        return np.array([refglue.rms_db(w) for w in self._wins], np.float64)

    def tempo(self, sel, start_bpm):
        self._check("tempo")
        out = np.zeros((len(sel), 4))
        for k, (i, sb) in enumerate(zip(sel, start_bpm)):
            t = refglue.estimate_tempo(self._wins[i], 22050, float(sb))
            out[k] = (t, 4, 0, np.nan) if t is not None else (0.0, 0, 0, np.nan)
        return out

    def chunks(self, chunk_off, chunk_len):
        self._check("chunks")
        out = np.zeros((len(chunk_off) // 2, 30))
        for k in range(len(chunk_off) // 2):
            a = self.buf[chunk_off[2 * k]:chunk_off[2 * k] + chunk_len[2 * k]]
            b = self.buf[chunk_off[2 * k + 1]:chunk_off[2 * k + 1] + chunk_len[2 * k + 1]]
            ca, cb = refglue.mean_chroma(a), refglue.mean_chroma(b)
            out[k, 0] = refglue.cyclic_xcorr_peak(ca, cb)
            ta, tb = ncref.estimate_tuning_detail(a), ncref.estimate_tuning_detail(b)
            out[k, 1:3] = ta[0], tb[0]
            out[k, 28:30] = ta[2], tb[2]
            out[k, 3:15], out[k, 15:27] = ca, cb
            xc = np.sort([float(np.dot(ca, np.roll(cb, -j))) for j in range(12)])
            out[k, 27] = (xc[-1] - xc[-2]) / abs(xc[-1]) if xc[-1] else 0.0
        return out

    def bootstrap(self, jobs, seed):
        """numpy default_rng(seed) per job: ratio of medians (draw order A then B), or the
        median of A alone; 'linear' 2.5 / 97.5 percentiles (consensus.py:243-312, pitch.py:143-150)."""
        res = []
        for A, B in jobs:
            rng = np.random.default_rng(seed)
            A = np.asarray(A, np.float64)
            boot = np.empty(2000)
            if B is None:
                point = float(np.median(A))
                for i in range(2000):
                    boot[i] = np.median(rng.choice(A, size=len(A), replace=True))
            else:
                B = np.asarray(B, np.float64)
                point = float(np.median(A) / np.median(B))
                for i in range(2000):
                    a = rng.choice(A, size=len(A), replace=True)
                    b = rng.choice(B, size=len(B), replace=True)
                    boot[i] = np.median(a) / np.median(b)
            res.append((point, (float(np.percentile(boot, 2.5)), float(np.percentile(boot, 97.5)))))
        return res

    # ---- the split hop-64 pass (sharded._sharded_ibi): the same onset and tempogram sums
    def ibi_mel(self, f_off, f_len, t0, t1):
        self._check("ibi")
        self._ibi_S, self._ibi_r = [], []
        mx = []
        for o, n, a, b in zip(f_off, f_len, t0, t1):
            S = ncref.mel_db(self.buf[o:o + n], 22050, 2048, 64)
            T = S.shape[1]
            # the rows its onsets read; the share ending the file also takes the last rows,
            # which feed only the maximum (power_to_db's top_db reference over every frame)
            r0, r1 = max(0, a - 17), (T if b >= T and b > a else min(T, b - 17 + 1))
            self._ibi_S.append(S)
            self._ibi_r.append((a, b))
            mx.append(float(S[:, r0:r1].max()) if r1 > r0 else -np.inf)
        return np.array(mx)

    def ibi_onset(self, gmax):
        out = []
        for S, (a, b), g in zip(self._ibi_S, self._ibi_r, gmax):
            Sc = np.maximum(S, np.float32(g) - np.float32(80.0))
            d = np.maximum(np.float32(0.0), Sc[:, 1:] - Sc[:, :-1])
            od = np.concatenate([np.zeros(17, np.float32), np.mean(d, axis=0, dtype=np.float32)])[:S.shape[1]]
            out.append(od[a:b])
        return np.concatenate(out) if out else np.zeros(0, np.float32)

    def ibi_tiles(self, onsets, b0, b1):
        rows = []
        for on, a, b in zip(onsets, b0, b1):
            for k in range(a, b):
                rows.append(ncref.tempogram_sum(on, 2756, k * 2048, min(len(on), (k + 1) * 2048)))
        return np.array(rows).reshape(-1, 2756)

    def ibi_reduce(self, tiles, T):
        out = []
        for rows, t in zip(tiles, T):
            acc = np.zeros(2756)
            for row in rows:
                acc = acc + row
            out.append(acc / t)
        return np.array(out)

    def ibi_beats(self, onsets, tgs, start_bpm):
        ibis, nibi = [], []
        for on, tg, sb in zip(onsets, tgs, start_bpm):
            _, beats = ncref.beat_track(on, 22050, 64, float(sb), tg_mean=tg)
            v = None
            if len(beats) >= 5:
                t = ncref.frames_to_time(beats, 22050, 64)
                d = np.diff(t)
                d = d[d > 0.05]
                v = d if len(d) >= 4 else None
            ibis.append(v)
            nibi.append(0 if v is None else len(v))
        z = np.zeros(len(onsets), np.int64)
        return ibis, np.array(nibi, np.int64), z, z

    def ibi(self, f_off, f_len, start_bpm):
        ibis, nibi = [], []
        for o, n, sb in zip(f_off, f_len, start_bpm):
            v = refglue.estimate_ibis_global(self.buf[o:o + n], 22050, start_bpm=float(sb))
            ibis.append(v if v is not None and len(v) >= 4 else None)
            nibi.append(0 if v is None else len(v))
        z = np.zeros(len(f_off), np.int64)
        return ibis, np.array(nibi, np.int64), z, z


class FakeStages:
    """Stage outputs of the right shapes with no DSP at all, for the fail-together tests: the
    orchestration's collectives are what is under test, so every stage is cheap.  ``fail_in``
    names the stage that raises on its ``fail_call``-th call (1-based); "pipeline" makes the
    interior pipeline generator raise after its first group."""

    N = 2756                                     # hop-64 tempogram lags (8 s)

    def __init__(self, lengths, fail_in=None, fail_call=1):
        self.length = np.asarray(lengths, np.int64)
        self.off = np.concatenate([[0], np.cumsum(self.length)[:-1]]).astype(np.int64)
        self.fail_in, self._left = fail_in, fail_call
        self._n = 0

    def restrict(self, files):
        f = np.asarray(files, np.int64)
        o = FakeStages.__new__(FakeStages)
        o.length, o.off, o.fail_in, o._left, o._n = self.length[f], self.off[f], self.fail_in, self._left, 0
        o._root = getattr(self, "_root", self)
        return o

    def _check(self, name):
        root = getattr(self, "_root", self)
        if root.fail_in == name:
            root._left -= 1
            if root._left == 0:
                raise RuntimeError(f"injected failure in {name}")

    def pipeline(self, files, p, steps=1, on_group=None):
        n = len(files) // 2
        fail = self.fail_in == "pipeline"

        def gen():
            from nightcore_analyzer.engine import PairOutcome
            res = [[PairOutcome() for _ in range(n)] for _ in range(steps)]
            for k in range(2 * steps):
                yield
                if fail:
                    raise RuntimeError("injected failure in pipeline")
                if on_group is not None and k % 2:        # one group per step, as it is assembled
                    on_group(k // 2, 0, res[k // 2])
            return res
        return gen()

    def trim(self, p):
        self._check("trim")
        return np.zeros(len(self.length), np.int64), self.length.copy()

    def windows(self, win_abs, win_n):
        self._check("windows")
        self._n = len(win_abs)
        return np.zeros(len(win_abs))

    def tempo(self, sel, start_bpm):
        self._check("tempo")
        out = np.zeros((len(sel), 4))
        out[:, 0], out[:, 1] = 120.0, 8
        return out

    def chunks(self, chunk_off, chunk_len):
        self._check("chunks")
        return np.zeros((len(chunk_off) // 2, 30))

    def bootstrap(self, jobs, seed):
        self._check("bootstrap")
        return [(1.0, (1.0, 1.0)) for _ in jobs]

    def ibi_mel(self, f_off, f_len, t0, t1):
        self._check("ibi_mel")
        self._t = (np.asarray(t0), np.asarray(t1))
        return np.zeros(len(f_off))

    def ibi_onset(self, gmax):
        self._check("ibi_onset")
        t0, t1 = self._t
        return np.zeros(int(np.maximum(0, t1 - t0).sum()), np.float32)

    def ibi_tiles(self, onsets, b0, b1):
        self._check("ibi_tiles")
        return np.zeros((int(np.maximum(0, np.asarray(b1) - np.asarray(b0)).sum()), self.N))

    def ibi_reduce(self, tiles, T):
        self._check("ibi_reduce")
        return np.zeros((len(tiles), self.N))

    def ibi_beats(self, onsets, tgs, start_bpm):
        self._check("ibi_beats")
        z = np.zeros(len(onsets), np.int64)
        return [np.full(8, 0.5)] * len(onsets), z + 8, z + 9, z

    def ibi(self, f_off, f_len, start_bpm):
        self._check("ibi")
        z = np.zeros(len(f_off), np.int64)
        return [np.full(8, 0.5)] * len(f_off), z + 8, z + 9, z
