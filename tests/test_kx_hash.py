# SPDX-License-Identifier: BSD-2-Clause
"""The key index's hash (oo_rx_device.h kx_hash), compiled for the host with
g++, against the Python restatement tests/test_gpu_key_index.py builds its
colliding keys with: if they drifted apart, those keys would stop sharing a
bucket and the GPU test would lose what it covers."""
import os
import subprocess

import numpy as np

from test_gpu_key_index import kx_hash

HERE = os.path.dirname(os.path.abspath(__file__))


def test_kx_hash_matches_the_device_header(tmp_path):
    exe = tmp_path / "kx_hash_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe),
                    os.path.join(HERE, "c", "kx_hash_check.cpp")], check=True)
    rng = np.random.default_rng(11)
    keys = rng.integers(0, 1 << 32, size=(200, 10), dtype=np.uint64).astype(np.uint32)
    keys[:50, 1:4] = 0  # IPv4 keys: la[1..3] = ra[1..3] = pw = 0
    keys[:50, 5:8] = 0
    keys[:50, 9] = 0
    inp = "\n".join(" ".join(str(int(v)) for v in k) for k in keys) + "\n"
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout
    want = kx_hash([keys[:, i] for i in range(10)])
    got = np.array([int(x) for x in out.split()], dtype=np.uint32)
    np.testing.assert_array_equal(got, want)
