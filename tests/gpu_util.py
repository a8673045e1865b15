# SPDX-License-Identifier: BSD-2-Clause
"""Helpers that run the gfx950 library on HBM-resident torch buffers."""
from __future__ import annotations

import numpy as np

from onload_amd import _abi


def to_dev(arr: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8)).to("cuda")


def run_dev(stack, buf: np.ndarray, desc: np.ndarray, frames_bytes: int | None = None):
    """Device-resident transform; returns (results, counters) on the host."""
    import torch
    n = len(desc)
    fr = to_dev(buf)
    de = to_dev(desc)
    out = torch.full((max(n, 1) * 32,), 0xAB, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(_abi.R_COUNT, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    stack.handle_rx_batch_dev(fr.data_ptr(), fr.numel() if frames_bytes is None else frames_bytes,
                              de.data_ptr(), n, out.data_ptr(), ctr.data_ptr(), stream)
    torch.cuda.synchronize()
    res = out.cpu().numpy()[: n * 32].view(_abi.RESULT_DTYPE)
    return res, ctr.cpu().numpy().astype(np.uint32)


def diff_report(a: np.ndarray, b: np.ndarray, desc=None, limit: int = 5) -> str:
    A = a.view(np.uint8).reshape(-1, 32)
    B = b.view(np.uint8).reshape(-1, 32)
    bad = np.nonzero((A != B).any(1))[0]
    lines = [f"{len(bad)} of {len(a)} records differ"]
    for i in bad[:limit]:
        lines.append(f"  [{i}] gpu={a[i]} oracle={b[i]}"
                     + (f" len={desc[i]['len']} off={desc[i]['frame_off']}" if desc is not None else ""))
    return "\n".join(lines)
