#!/usr/bin/env python3
"""Times nc_window_stage (stft_mel + window_tg) of libncgpu.so variants on N synthetic
10 s windows (default 3968, the bench step's count) with the library's own per-kernel
HIP-event timers.
    python3 tools/wtg_bench.py N tools/var/<name>/libncgpu.so ..."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))
from nightcore_analyzer import synth  # noqa: E402


def main(path, n):
    lib = C.CDLL(path)
    P, I32, SZ = C.c_void_p, C.c_int, C.c_size_t
    lib.nc_create.argtypes = [I32, C.POINTER(P)]
    lib.nc_window_stage_workspace_bytes.restype = SZ
    lib.nc_window_stage_workspace_bytes.argtypes = [P, I32, I32, I32]
    lib.nc_window_stage.argtypes = [P, P, P, P, I32, I32, I32, P, P, P, P, SZ, P]
    lib.nc_profile_enable.argtypes = [P, I32]
    lib.nc_profile_read.argtypes = [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I32)]
    ctx = P()
    assert lib.nc_create(0, C.byref(ctx)) == 0
    src = synth.make_source(180.0, 1000)
    L, T, acw = 220500, 431, 344
    wins = np.stack([src[(i % 35) * 110250:(i % 35) * 110250 + L] for i in range(n)]).astype(np.float32)
    dev = torch.device("cuda")
    sig = torch.from_numpy(wins.reshape(-1)).to(dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    onset = torch.empty(n * T, device=dev)
    tg = torch.empty(n * acw, dtype=torch.float64, device=dev)
    en = torch.empty(n, dtype=torch.float64, device=dev)
    wsb = lib.nc_window_stage_workspace_bytes(ctx, n, L, 512)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def run():
        assert lib.nc_window_stage(ctx, sig.data_ptr(), off.data_ptr(), None, n, L, 512, onset.data_ptr(),
                                   tg.data_ptr(), en.data_ptr(), ws.data_ptr(), wsb, st) == 0
    for _ in range(2):
        run()
    torch.cuda.synchronize()
    lib.nc_profile_enable(ctx, 1)
    for _ in range(5):
        run()
    out = {}
    for tag in (b"stft_mel", b"window_tg"):
        ms, k = C.c_double(), I32()
        lib.nc_profile_read(ctx, tag, C.byref(ms), C.byref(k))
        out[tag.decode()] = round(ms.value / max(1, k.value) * 1e3, 1)
    print(Path(path).parent.name, n, "us per launch:", out, "tg[0][:3]", tg[:3].cpu().numpy(), flush=True)


if __name__ == "__main__":
    for p in sys.argv[2:]:
        main(p, int(sys.argv[1]))
