#!/usr/bin/env python3
"""Times libncgpu.so variants (tools/var/<name>/libncgpu.so) on the chroma path
(nc_chroma_mean over 224 synthetic 20 s chunks) and the window path (nc_window_stage
over 560 synthetic 10 s windows) with the library's own per-kernel HIP-event timers.
The variants are loaded side by side and timed in rotation (A B C A B C ...), so clock
drift over the run hits them alike; each prints its per-kernel minimum over the rounds
and a checksum of its outputs so variants can be compared for equality.
    python3 tools/var_bench.py tools/var/<name>/libncgpu.so [...]"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))
from nightcore_analyzer import synth  # noqa: E402

TAGS = (b"stft_mel", b"window_tg", b"decimate", b"tuning_peaks", b"tuning_select", b"cqt_low", b"cqt_high")
ROUNDS, ITERS = 6, 3


class Variant:
    def __init__(self, path, inp):
        self.name = Path(path).parent.name
        lib = self.lib = C.CDLL(path)
        P, I32, SZ, I64 = C.c_void_p, C.c_int, C.c_size_t, C.c_int64
        lib.nc_create.argtypes = [I32, C.POINTER(P)]
        lib.nc_window_stage_workspace_bytes.restype = SZ
        lib.nc_window_stage_workspace_bytes.argtypes = [P, I32, I32, I32]
        lib.nc_window_stage.argtypes = [P, P, P, P, I32, I32, I32, P, P, P, P, SZ, P]
        lib.nc_chroma_workspace_bytes.restype = SZ
        lib.nc_chroma_workspace_bytes.argtypes = [P, I32, I64]
        lib.nc_chroma_mean.argtypes = [P, P, P, P, I32, I64, I64, P, P, P, P, P, SZ, P]
        lib.nc_profile_enable.argtypes = [P, I32]
        lib.nc_profile_read.argtypes = [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I32)]
        self.ctx = P()
        assert lib.nc_create(0, C.byref(self.ctx)) == 0
        self.inp = inp
        dev = torch.device("cuda")
        n, T, acw, cn = inp["n"], inp["T"], inp["acw"], inp["cn"]
        self.onset = torch.empty(n * T, device=dev)
        self.tg = torch.empty(n * acw, dtype=torch.float64, device=dev)
        self.en = torch.empty(n, dtype=torch.float64, device=dev)
        self.wsb = lib.nc_window_stage_workspace_bytes(self.ctx, n, inp["L"], 512)
        self.ws = torch.empty(self.wsb, dtype=torch.uint8, device=dev)
        self.chroma = torch.empty(cn * 12, device=dev)
        self.tun = torch.empty(cn, device=dev)
        self.cwsb = lib.nc_chroma_workspace_bytes(self.ctx, cn, cn * inp["CL"])
        self.cws = torch.empty(self.cwsb, dtype=torch.uint8, device=dev)
        self.best = {}
        # VB_TUNING=1: the window STFT also runs the shared tuning frames' piptrack, as in the
        # engine (nc_window_stage_tuning), for every fourth window (a 20 s chunk start)
        self.tuning = os.environ.get("VB_TUNING") == "1"
        if self.tuning:
            lib.nc_window_stage_tuning.argtypes = [P, P, P, P, I32, I32, I32, P, P, P, P, P, I32, P, P, P, P, P,
                                                   SZ, P]
            nch = (n + 3) // 4
            wc = np.full(n, -1, np.int32)
            wc[::4] = np.arange(nch, dtype=np.int32)
            self.win_chunk = torch.from_numpy(wc).to(dev)
            self.tf_base = torch.arange(nch + 1, dtype=torch.int64, device=dev) * (1 + inp["CL"] // 512)
            slots = int(self.tf_base[-1]) * 192
            self.pp = torch.empty(slots, device=dev)
            self.pm = torch.empty(slots, device=dev)
            self.npk = torch.zeros(nch, dtype=torch.int32, device=dev)
            self.tp = (inp["L"] - 1024) // 512 + 1

    def run(self):
        i, lib, st = self.inp, self.lib, torch.cuda.current_stream().cuda_stream
        if self.tuning:
            self.npk.zero_()
            assert lib.nc_window_stage_tuning(self.ctx, i["sig"].data_ptr(), i["off"].data_ptr(), None, i["n"], i["L"],
                                              512, self.onset.data_ptr(), self.tg.data_ptr(), self.en.data_ptr(),
                                              self.win_chunk.data_ptr(), self.tf_base.data_ptr(), self.tp,
                                              self.pp.data_ptr(), self.pm.data_ptr(), self.npk.data_ptr(), None,
                                              self.ws.data_ptr(), self.wsb, st) == 0
        else:
            assert lib.nc_window_stage(self.ctx, i["sig"].data_ptr(), i["off"].data_ptr(), None, i["n"], i["L"], 512,
                                       self.onset.data_ptr(), self.tg.data_ptr(), self.en.data_ptr(),
                                       self.ws.data_ptr(), self.wsb, st) == 0
        assert lib.nc_chroma_mean(self.ctx, i["csig"].data_ptr(), i["coff"].data_ptr(), i["clen"].data_ptr(),
                                  i["cn"], i["cn"] * i["CL"], i["CL"], self.chroma.data_ptr(), self.tun.data_ptr(),
                                  None, None, self.cws.data_ptr(), self.cwsb, st) == 0

    def timed(self):
        lib = self.lib
        torch.cuda.synchronize()
        lib.nc_profile_enable(self.ctx, 1)
        for _ in range(ITERS):
            self.run()
        torch.cuda.synchronize()
        for tag in TAGS:
            ms, k = C.c_double(), C.c_int()
            lib.nc_profile_read(self.ctx, tag, C.byref(ms), C.byref(k))
            us = ms.value / ITERS * 1e3
            self.best[tag.decode()] = round(min(self.best.get(tag.decode(), 1e30), us), 1)
        lib.nc_profile_enable(self.ctx, 0)

    def report(self):
        cks = (float(self.onset.double().sum()), float(self.tg.sum()), float(self.chroma.double().sum()))
        if self.tuning:
            print(f"  tuning peaks {int(self.npk.sum())}", flush=True)
        print(f"{self.name:18s} min us/run {self.best}  checksum onset {cks[0]:.6f} tg {cks[1]:.9f} "
              f"chroma {cks[2]:.7f}", flush=True)
        if hasattr(self.lib, "nc_dbg_stamps"):  # a phase-stamped diagnostic build
            buf = (C.c_ulonglong * 16)()
            self.lib.nc_dbg_stamps(buf, 0)
            n = max(1, buf[7])
            print(f"  stamped kernel, cycles per item over {n} items, by phase: " +
                  ", ".join(f"{buf[i] / n:.0f}" for i in range(7)), flush=True)


def inputs(src):
    dev = torch.device("cuda")
    n, L, T, acw = 560, 220500, 431, 344
    wins = np.stack([src[(i % 35) * 110250:(i % 35) * 110250 + L] for i in range(n)]).astype(np.float32)
    cn, CL = 224, 441000
    chunks = np.stack([src[(i % 9) * CL:(i % 9) * CL + CL] for i in range(cn)]).astype(np.float32)
    return dict(n=n, L=L, T=T, acw=acw, cn=cn, CL=CL,
                # VB_WINSHIFT=k: every window k samples later in the buffer (a trimmed file's windows
                # start at any sample; odd starts miss stft_mel's float2 fast path)
                sig=torch.from_numpy(np.concatenate([np.zeros(int(os.environ.get("VB_WINSHIFT", "0")), np.float32),
                                                     wins.reshape(-1)])).to(dev),
                off=torch.arange(n, dtype=torch.int64, device=dev) * L + int(os.environ.get("VB_WINSHIFT", "0")),
                # VB_CHUNKSHIFT=k: every chunk k samples past a 16-byte boundary (a trimmed file's
                # chunks start anywhere; the low-octave CQT's DMA path needs 16-byte alignment)
                csig=torch.from_numpy(np.concatenate([np.zeros(int(os.environ.get("VB_CHUNKSHIFT", "0")), np.float32),
                                                      chunks.reshape(-1)])).to(dev),
                # VB_SAMECHUNK=1: every chunk at offset 0 (their level-0 reads become L2 / MALL hits;
                # a probe of the low-octave CQT's exposed block latency)
                coff=torch.arange(cn, dtype=torch.int64, device=dev) * CL * (os.environ.get("VB_SAMECHUNK") != "1")
                + int(os.environ.get("VB_CHUNKSHIFT", "0")),
                clen=torch.full((cn,), CL, dtype=torch.int64, device=dev))


if __name__ == "__main__":
    inp = inputs(synth.make_source(180.0, 1000))
    vs = [Variant(p, inp) for p in sys.argv[1:]]
    for v in vs:
        for _ in range(2):
            v.run()
    for _ in range(ROUNDS):
        for v in vs:
            v.timed()
    for v in vs:
        v.report()
