# SPDX-License-Identifier: BSD-2-Clause
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

_LIBS = ["onload_amd/liboo_gpu_rx.so", "onload_amd/liboo_pktgen.so", "oracle/liboorx_oracle.so"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    # The compiled reference (oracle/_ref: fixture generators and this
    # container's live checks) never travels to the GPU box (SURVEY.md
    # §8(c), .gpurunignore): a session where it exists without the reference
    # tree it was built from is one whose snapshot carried it.
    ref_build = os.path.join(ROOT, "oracle", "_ref")
    if os.path.exists(ref_build) and not os.path.isdir("/root/reference"):
        raise pytest.UsageError(
            "oracle/_ref is present but /root/reference is not: the compiled reference "
            "travelled with the snapshot (.gpurunignore must list ./oracle/_ref)")
    if any(not os.path.exists(os.path.join(ROOT, p)) for p in _LIBS):
        subprocess.run(["make", "-C", ROOT, "-j4"], check=True)
