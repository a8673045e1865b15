# SPDX-License-Identifier: BSD-2-Clause
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

_LIBS = ["onload_amd/liboo_gpu_rx.so", "onload_amd/liboo_pktgen.so", "oracle/liboorx_oracle.so"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    if any(not os.path.exists(os.path.join(ROOT, p)) for p in _LIBS):
        subprocess.run(["make", "-C", ROOT, "-j4"], check=True)
