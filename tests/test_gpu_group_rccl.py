# SPDX-License-Identifier: BSD-2-Clause
"""The across-processes group (oo_gpu_rx_group_join) run for real on one
GPU: a group of one rank whose every collective goes through librccl -- the
op broadcast in chunks (config 5's world is 11,936 queued changes: more than
one chunk), the table-image broadcast, the records gathered by a send/receive
pair to itself, the counters summed by an all-reduce -- bit-exact with the
oracle.  The same calls a rank of an 8-GPU job makes (bench.py --gpus N);
only the peers are missing.

Each case runs in a child process of its own (rccl_one_rank.py), as a rank
of a real job does: librccl, its communicator and its threads never share a
process with the rest of the suite (the faults)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("case", ["every_leg", "bad_count"])
def test_one_rank_group(case):
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_one_rank.py"), case],
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith(f"ok {case}"), \
        f"rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert "Memory Fault" not in r.stderr, r.stderr[-4000:]
