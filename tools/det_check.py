#!/usr/bin/env python3
"""Run-to-run determinism of nc_chroma_mean: the same 224 chunks R times in one process (fresh
workspace contents between runs), per-chunk max difference between runs, and against a
reference library if given.
    python3 tools/det_check.py LIB [REFLIB]"""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))
from nightcore_analyzer import synth  # noqa: E402


def runs(path, csig, coff, clen, cn, CL, R=6):
    lib = C.CDLL(path)
    P, I32, SZ, I64 = C.c_void_p, C.c_int, C.c_size_t, C.c_int64
    lib.nc_create.argtypes = [I32, C.POINTER(P)]
    lib.nc_chroma_workspace_bytes.restype = SZ
    lib.nc_chroma_workspace_bytes.argtypes = [P, I32, I64]
    lib.nc_chroma_mean.argtypes = [P, P, P, P, I32, I64, I64, P, P, P, P, P, SZ, P]
    ctx = P()
    assert lib.nc_create(0, C.byref(ctx)) == 0
    st = torch.cuda.current_stream().cuda_stream
    cwsb = lib.nc_chroma_workspace_bytes(ctx, cn, cn * CL)
    outs = []
    for r in range(R):
        cws = torch.full((cwsb,), 0x7f if r % 2 else 0x11, dtype=torch.uint8, device="cuda")
        chroma = torch.full((cn * 12,), float("nan"), device="cuda")
        tun = torch.empty(cn, device="cuda")
        assert lib.nc_chroma_mean(ctx, csig.data_ptr(), coff.data_ptr(), clen.data_ptr(), cn, cn * CL, CL,
                                  chroma.data_ptr(), tun.data_ptr(), None, None, cws.data_ptr(), cwsb, st) == 0
        torch.cuda.synchronize()
        outs.append(chroma.cpu().numpy().reshape(cn, 12).copy())
    return outs


def main():
    src = synth.make_source(180.0, 1000)
    cn, CL = 224, 441000
    dev = torch.device("cuda")
    chunks = np.stack([src[(i % 9) * CL:(i % 9) * CL + CL] for i in range(cn)]).astype(np.float32)
    csig = torch.from_numpy(chunks.reshape(-1)).to(dev)
    coff = torch.arange(cn, dtype=torch.int64, device=dev) * CL
    clen = torch.full((cn,), CL, dtype=torch.int64, device=dev)
    res = {p: runs(p, csig, coff, clen, cn, CL) for p in sys.argv[1:]}
    for p, outs in res.items():
        d = [np.abs(o - outs[0]).max(axis=1) for o in outs[1:]]
        bad = sorted({int(i) for x in d for i in np.nonzero(x)[0]})
        print(Path(p).parent.name, "run-to-run max", max(float(x.max()) for x in d), "chunks differing", bad[:20],
              "nan", int(sum(np.isnan(o).sum() for o in outs)), flush=True)
    if len(res) == 2:
        a, b = list(res.values())
        d = np.abs(a[0] - b[0]).max(axis=1)
        print("vs ref: max", float(d.max()), "worst chunks", np.argsort(d)[-5:].tolist(), d[np.argsort(d)[-5:]].tolist())


if __name__ == "__main__":
    main()
