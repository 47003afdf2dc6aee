#!/usr/bin/env python3
"""Times one libncgpu.so variant (tools/var/<name>/libncgpu.so) on the chroma path
(nc_chroma_mean over 224 synthetic 20 s chunks) and the window path (nc_window_stage
over 560 synthetic 10 s windows) with the library's own per-kernel HIP-event timers,
and prints a checksum of the outputs so variants can be compared for equality.
    python3 tools/var_bench.py tools/var/<name>/libncgpu.so [...]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))
from nightcore_analyzer import synth  # noqa: E402

TAGS = (b"stft_mel", b"window_tg", b"decimate", b"tuning_peaks", b"tuning_select", b"cqt_low", b"cqt_high")


def bench(path, src):
    lib = C.CDLL(path)
    P, I32, SZ, I64 = C.c_void_p, C.c_int, C.c_size_t, C.c_int64
    lib.nc_create.argtypes = [I32, C.POINTER(P)]
    lib.nc_destroy.argtypes = [P]
    lib.nc_window_stage_workspace_bytes.restype = SZ
    lib.nc_window_stage_workspace_bytes.argtypes = [P, I32, I32, I32]
    lib.nc_window_stage.argtypes = [P, P, P, P, I32, I32, I32, P, P, P, P, SZ, P]
    lib.nc_chroma_workspace_bytes.restype = SZ
    lib.nc_chroma_workspace_bytes.argtypes = [P, I32, I64]
    lib.nc_chroma_mean.argtypes = [P, P, P, P, I32, I64, I64, P, P, P, P, P, SZ, P]
    lib.nc_profile_enable.argtypes = [P, I32]
    lib.nc_profile_read.argtypes = [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I32)]
    ctx = P()
    assert lib.nc_create(0, C.byref(ctx)) == 0
    dev = torch.device("cuda")
    st = torch.cuda.current_stream().cuda_stream
    # window path
    n, L, T, acw = 560, 220500, 431, 344
    wins = np.stack([src[(i % 35) * 110250:(i % 35) * 110250 + L] for i in range(n)]).astype(np.float32)
    sig = torch.from_numpy(wins.reshape(-1)).to(dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    onset = torch.empty(n * T, device=dev)
    tg = torch.empty(n * acw, dtype=torch.float64, device=dev)
    en = torch.empty(n, dtype=torch.float64, device=dev)
    wsb = lib.nc_window_stage_workspace_bytes(ctx, n, L, 512)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    # chroma path
    cn, CL = 224, 441000
    chunks = np.stack([src[(i % 9) * CL:(i % 9) * CL + CL] for i in range(cn)]).astype(np.float32)
    csig = torch.from_numpy(chunks.reshape(-1)).to(dev)
    coff = torch.arange(cn, dtype=torch.int64, device=dev) * CL
    clen = torch.full((cn,), CL, dtype=torch.int64, device=dev)
    chroma = torch.empty(cn * 12, device=dev)
    tun = torch.empty(cn, device=dev)
    cwsb = lib.nc_chroma_workspace_bytes(ctx, cn, cn * CL)
    cws = torch.empty(cwsb, dtype=torch.uint8, device=dev)

    def run():
        assert lib.nc_window_stage(ctx, sig.data_ptr(), off.data_ptr(), None, n, L, 512, onset.data_ptr(),
                                   tg.data_ptr(), en.data_ptr(), ws.data_ptr(), wsb, st) == 0
        assert lib.nc_chroma_mean(ctx, csig.data_ptr(), coff.data_ptr(), clen.data_ptr(), cn, cn * CL, CL,
                                  chroma.data_ptr(), tun.data_ptr(), None, None, cws.data_ptr(), cwsb, st) == 0
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    lib.nc_profile_enable(ctx, 1)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    out = {}
    for tag in TAGS:
        ms, k = C.c_double(), I32()
        lib.nc_profile_read(ctx, tag, C.byref(ms), C.byref(k))
        out[tag.decode()] = round(ms.value / 5 * 1e3, 1)
    lib.nc_profile_enable(ctx, 0)
    cks = (float(onset.double().sum()), float(tg.sum()), float(chroma.double().sum()))
    print(f"{Path(path).parent.name:18s} us/run {out}  checksum onset {cks[0]:.6f} tg {cks[1]:.9f} "
          f"chroma {cks[2]:.7f}", flush=True)


if __name__ == "__main__":
    src = synth.make_source(180.0, 1000)
    for p in sys.argv[1:]:
        bench(p, src)
