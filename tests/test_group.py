# SPDX-License-Identifier: BSD-2-Clause
"""The multi-GPU group of the C ABI (include/oo_gpu_rx.h "Multi-GPU group",
onload_amd/group.py) without a GPU: members that are host-only contexts
(device < 0) keep byte-identical replicas of the tables through a whole
insert / remove / socket-churn script applied through the group (return
codes included, equal to one stack running the script alone), and the
byte-balanced split covers a batch exactly with shares of equal bytes."""
import numpy as np
import pytest

import table_scripts as ts
from onload_amd import pktgen
from onload_amd.group import GpuRxGroup
from onload_amd.rx import GpuRxStack


def test_host_only_members_stay_identical():
    cfg, socks, ops = ts.build("mixed")
    ops = [o for o in ops if o[0] in "AR"]
    g = GpuRxGroup(devices=[-1, -1, -1], max_socks=1024, ip4_log2=cfg["log4"],
                   ip6_log2=cfg["log6"], intf_hwport=cfg["hwports"])
    one = GpuRxStack(device=-1, max_socks=1024, ip4_log2=cfg["log4"], ip6_log2=cfg["log6"],
                     intf_hwport=cfg["hwports"])
    got, want = [], []
    for at in range(0, len(ops), 500):  # op batches with socket churn between
        got += ts.replay(g, socks if at == 0 else [], ops[at:at + 500])
        want += ts.replay(one, socks if at == 0 else [], ops[at:at + 500])
        s = socks[(at // 500) % len(socks)]
        s.hwports ^= 1
        got.append(g.sock_set(s.id, ts.sock_struct(s)))
        want.append(one.sock_set(s.id, ts.sock_struct(s)))
    assert len(got) >= 5800  # the ~6000-op mixed script (inserts, removes, socket churn)
    assert got == want
    assert any(rc != 0 for rc in want)  # -ENOBUFS / removes of absent filters
    ref = one.image_host().tobytes()
    for m in g.members:
        assert m.image_host().tobytes() == ref
    g.close()
    one.close()


@pytest.mark.parametrize("config,n,parts", [(2, 4096, 3), (4, 20000, 8), (5, 30001, 7),
                                            (3, 5, 8)])
def test_split_is_exact_and_byte_balanced(config, n, parts):
    g = GpuRxGroup(devices=[-1])
    _, desc = pktgen.generate(config, n)
    sh = g.split(desc, parts)
    assert sh[0][0] == 0 and sum(c for _, c in sh) == n
    assert all(sh[k][0] + sh[k][1] == sh[k + 1][0] for k in range(parts - 1))
    cost = desc["len"].astype(np.int64) + 48
    if n >= 100 * parts:
        tot = cost.sum()
        for f, c in sh:
            assert abs(cost[f:f + c].sum() - tot / parts) <= cost.max()
    g.close()


def test_join_rejects_bad_arguments():
    with pytest.raises(OSError):
        GpuRxGroup.join(device=-1, rank=0, nranks=2, gid=b"\0" * 128)  # host-only
    with pytest.raises(OSError):
        GpuRxGroup.join(device=0, rank=2, nranks=2, gid=b"\0" * 128)   # rank out of range
