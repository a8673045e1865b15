# SPDX-License-Identifier: BSD-2-Clause
"""oo_gpu_rx_set_tuning's argument checks, oo_gpu_rx_last_path and
oo_gpu_rx_table_gen on a host-only context (no GPU): the launch settings are
validated before any launch, the path report starts at "none", and every
table or socket change moves the generation the poll shim watches."""
import pytest

from onload_amd import _abi
from onload_amd.rx import GpuRxStack


def _tuning(**kw):
    t = _abi.Tuning()
    t.gshift = -1
    for k, v in kw.items():
        setattr(t, k, v)
    return t


def test_tuning_validated():
    g = GpuRxStack(device=-1, max_socks=16, ip6_log2=4)
    g.set_tuning(None)
    for path in (0, 1, 2, 3, 4):
        g.set_tuning(_tuning(path=path))
    for engine in (0, 1, 2):
        g.set_tuning(_tuning(path=3, body_engine=engine))
    for walks in (0, 1):
        g.set_tuning(_tuning(walks=walks))
    for bad in (dict(path=5), dict(grid_pct=101), dict(body_engine=3), dict(walks=2)):
        with pytest.raises(OSError):
            g.set_tuning(_tuning(**bad))
    g.close()


def test_last_path_and_table_gen():
    g = GpuRxStack(device=-1, max_socks=16, ip6_log2=4)
    assert g.last_path() == 0  # no batch yet
    gen = g.table_gen()
    assert g.filter_insert(1, 4, "10.0.0.1", 80, None, 0, 17) == 0
    assert g.table_gen() == gen + 1
    assert g.filter_remove(1, 4, "10.0.0.1", 80, None, 0, 17) == 0
    assert g.table_gen() == gen + 2
    # a socket-field change counts too
    assert g.sock_set(1, _abi.Sock()) == 0
    assert g.table_gen() == gen + 3
    # an insert that fails (an id past max_socks) changes nothing
    assert g.filter_insert(99, 4, "10.0.0.1", 81, None, 0, 17) != 0
    assert g.table_gen() == gen + 3
    g.close()
