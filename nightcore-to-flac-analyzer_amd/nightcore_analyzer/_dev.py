"""Device-memory plumbing: torch-ROCm tensors as the allocator, raw pointers for the C ABI."""
from __future__ import annotations

import numpy as np
import torch


def device(idx: int = 0) -> torch.device:
    return torch.device("cuda", idx)


def stream_handle(dev: torch.device | None = None) -> int:
    """hipStream_t of torch's current stream (the engine launches everything on it)."""
    return torch.cuda.current_stream(dev).cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def to_dev(a, dev: torch.device, dtype=None) -> torch.Tensor:
    arr = np.ascontiguousarray(a if dtype is None else np.asarray(a, dtype=dtype))
    return torch.from_numpy(arr).to(dev, non_blocking=False)


def empty(n, dtype, dev: torch.device) -> torch.Tensor:
    return torch.empty(int(max(1, n)), dtype=dtype, device=dev)


def workspace(nbytes: int, dev: torch.device) -> torch.Tensor:
    return torch.empty(int(max(256, nbytes)), dtype=torch.uint8, device=dev)
