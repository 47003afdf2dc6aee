"""Resource checks of the built gfx950 code objects: the kernels whose loads are
issued by inline asm and retired by counted waits (the CQT kernels: c2_ld16 / cm_dma16 outputs
tied to the registers only at their s_waitcnt) must not spill — a spill or copy of a staged
register before its wait would read a load that has not landed.  Reads each kernel's
.private_segment_fixed_size (scratch bytes per lane) and VGPR count from the code-object notes of
the in-tree libncgpu.so (llvm-objdump --offloading, llvm-readelf --notes).  Host only."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
LIB = REPO / "nightcore-to-flac-analyzer_amd" / "nightcore_analyzer" / "_lib" / "libncgpu.so"
LLVM = Path("/opt/rocm/lib/llvm/bin")
NO_SCRATCH = ("cqt_mfma_low_kernel", "cqt_mfma_kernel", "stft_mel_kernel", "tuning_peaks_kernel", "decimate3_kernel")


def _kernels(tmp_path):
    if not LIB.exists() or not (LLVM / "llvm-objdump").exists():
        pytest.skip("needs the built library and the ROCm LLVM tools")
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(lib)], cwd=tmp_path, check=True,
                   capture_output=True)
    out = {}
    for co in tmp_path.glob("lib.so.*gfx950"):
        notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], capture_output=True,
                               text=True).stdout
        for block in re.split(r"\n  - (?=\.)", notes)[1:]:
            name = re.search(r"\.name:\s+(\S+)", block)
            scratch = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
            vgpr = re.search(r"\.vgpr_count:\s+(\d+)", block)
            if name and scratch and vgpr:
                out[name.group(1)] = (int(scratch.group(1)), int(vgpr.group(1)))
    return out


def test_staged_load_kernels_do_not_spill(tmp_path):
    k = _kernels(tmp_path)
    seen = {n: v for n, v in k.items() if any(t in n for t in NO_SCRATCH)}
    assert {t for t in NO_SCRATCH if any(t in n for n in seen)} == set(NO_SCRATCH), sorted(k)
    bad = {n: v for n, v in seen.items() if v[0] != 0}
    assert not bad, bad
    # the CQT octave 0-2 kernel's occupancy budget (two waves per SIMD: <= 256 registers)
    low = [v for n, v in seen.items() if "cqt_mfma_low_kernel" in n]
    assert low and all(v[1] <= 256 for v in low), low
