# SPDX-License-Identifier: BSD-2-Clause
"""onload_amd: Onload's software receive transform (checksum verify, header
parse, 4-tuple socket demux) as hand-written gfx950 HIP kernels behind a C ABI
(include/oo_gpu_rx.h).  See DESIGN.md."""
from ._abi import (DESC_DTYPE, RESULT_DTYPE, REASON_NAMES, R_DROP_BASE,  # noqa: F401
                   load_library)
from .rx import GpuRxStack, handled, htons  # noqa: F401

__all__ = ["GpuRxStack", "handled", "htons", "load_library", "DESC_DTYPE", "RESULT_DTYPE",
           "REASON_NAMES", "R_DROP_BASE"]
