#!/usr/bin/env python3
"""Times libncgpu.so variants on spectral.analyze (nc_spectral_stats over 128 resident 3-min
22.05 kHz files, the bench's spectral workload, plus VS_ODD=1 for files at odd offsets), in
rotation as tools/var_bench.py does, with the library's per-kernel HIP-event timers; prints
each variant's per-kernel minimum and an exact checksum of its outputs.
    python3 tools/spec_var.py tools/var/<name>/libncgpu.so [...]"""
import ctypes as C
import hashlib
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))
from nightcore_analyzer import synth  # noqa: E402

TAGS = (b"spectral_frames", b"spectral_bins")
ROUNDS, ITERS = 6, 3
BANDS = ((20, 80), (80, 250), (250, 2000), (2000, 6000), (6000, 20000))


def inputs():
    dev = torch.device("cuda")
    n, sr = 128, 22050
    src = synth.make_source(180.0, 1000).astype(np.float32)
    odd = os.environ.get("VS_ODD") == "1"
    lens = np.array([len(src) - 977 * (i % 7) for i in range(n)], np.int64)
    off = np.zeros(n, np.int64)
    pos = 0
    for i in range(n):
        pos += (i & 1) if odd else 0
        off[i] = pos
        pos += int(lens[i])
    sig = np.zeros(pos, np.float32)
    for i in range(n):
        sig[off[i]:off[i] + lens[i]] = np.roll(src, 5000 * i)[:lens[i]]
    T = 1 + lens // 512
    base = np.zeros(n + 1, np.int64)
    base[1:] = np.cumsum(T)
    freqs = np.fft.rfftfreq(2048, 1.0 / sr)
    bands = np.zeros((n, 5, 2), np.int32)
    for b, (lo, hi) in enumerate(BANDS):
        idx = np.flatnonzero((freqs >= lo) & (freqs < hi))
        bands[:, b] = (idx[0], idx[-1] + 1)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return dict(n=n, sig=t(sig), off=t(off), len=t(lens), base=t(base), hz=t(np.full(n, freqs[1])),
                bands=t(bands), tot=int(base[-1]), mx=int(T.max()))


class Variant:
    def __init__(self, path, inp):
        self.name = Path(path).parent.name
        lib = self.lib = C.CDLL(path)
        P, I32, SZ, I64 = C.c_void_p, C.c_int, C.c_size_t, C.c_int64
        lib.nc_create.argtypes = [I32, C.POINTER(P)]
        lib.nc_spectral_workspace_bytes.restype = SZ
        lib.nc_spectral_workspace_bytes.argtypes = [I64, I32, I64]
        lib.nc_spectral_stats.argtypes = [P, P, P, P, P, P, P, I32, I64, I64, C.c_float, P, P, P, P, SZ, P]
        lib.nc_profile_enable.argtypes = [P, I32]
        lib.nc_profile_read.argtypes = [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I32)]
        self.ctx = P()
        assert lib.nc_create(0, C.byref(self.ctx)) == 0
        self.inp = inp
        dev = torch.device("cuda")
        n = inp["n"]
        self.rms = torch.empty(inp["tot"], device=dev)
        self.stats = torch.empty(12 * n, dtype=torch.float64, device=dev)
        self.bins = torch.empty(1025 * n, dtype=torch.float64, device=dev)
        self.wsb = lib.nc_spectral_workspace_bytes(inp["tot"], n, inp["mx"])
        self.ws = torch.empty(self.wsb, dtype=torch.uint8, device=dev)
        self.best = {}

    def run(self):
        i, st = self.inp, torch.cuda.current_stream().cuda_stream
        assert self.lib.nc_spectral_stats(self.ctx, i["sig"].data_ptr(), i["off"].data_ptr(), i["len"].data_ptr(),
                                          i["base"].data_ptr(), i["hz"].data_ptr(), i["bands"].data_ptr(), i["n"],
                                          i["tot"], i["mx"], 0.85, self.rms.data_ptr(), self.stats.data_ptr(),
                                          self.bins.data_ptr(), self.ws.data_ptr(), self.wsb, st) == 0

    def timed(self):
        torch.cuda.synchronize()
        self.lib.nc_profile_enable(self.ctx, 1)
        for _ in range(ITERS):
            self.run()
        torch.cuda.synchronize()
        for tag in TAGS:
            ms, k = C.c_double(), C.c_int()
            self.lib.nc_profile_read(self.ctx, tag, C.byref(ms), C.byref(k))
            us = ms.value / ITERS * 1e3
            self.best[tag.decode()] = round(min(self.best.get(tag.decode(), 1e30), us), 1)
        self.lib.nc_profile_enable(self.ctx, 0)

    def report(self):
        h = hashlib.sha1()
        for x in (self.rms, self.stats, self.bins):
            h.update(x.cpu().numpy().tobytes())
        print(f"{self.name:10s} min us/run {self.best}  sha1 {h.hexdigest()[:16]}", flush=True)


if __name__ == "__main__":
    inp = inputs()
    vs = [Variant(p, inp) for p in sys.argv[1:]]
    for v in vs:
        for _ in range(2):
            v.run()
    for _ in range(ROUNDS):
        for v in vs:
            v.timed()
    for v in vs:
        v.report()
