# SPDX-License-Identifier: BSD-2-Clause
"""Table images (oo_gpu_rx_table_export / _import) on host-only contexts:
the image holds exactly the reference's slot state (the oracle's restatement
of netif_table.c / netif_table_ip6.c: states, ids, laddr, lport, route
counts) plus the socket fields each slot names, and an import reproduces the
tables so that later inserts/removes place entries identically."""
import errno

import numpy as np
import pytest

from onload_amd import _abi
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack
from test_abi_tables import _random_ops

ST_MASK, ST_EMPTY = 0xC0000000, 0x80000000


def _socks(n):
    socks = []
    for i in range(n):
        s = _abi.Sock()
        s.protocol = 6 if i % 2 else 17
        s.rport_be16 = i
        s.lport_be16 = (i * 7) & 0xFFFF
        s.raddr_be32 = i * 0x01010101
        s.flags = _abi.SOCK_CONNECTED if i % 3 == 0 else 0
        s.bind2dev_hwports = i
        for k in range(16):
            s.raddr6[k] = (i + k) & 0xFF
        socks.append(s)
    return socks


def _run_script(stacks, ops):
    for op in ops:
        kind, args = op[0], op[1:]
        rcs = {(st.filter_insert if kind == "ins" else st.filter_remove)(*args) for st in stacks}
        assert len(rcs) == 1, (op, rcs)


def _check_image_against_oracle(img, o, socks, n4, n6):
    p = _abi.parse_image(img)
    assert p["hdr"]["magic"] == 0x42544F4F and int(p["hdr"]["total"]) == len(img)
    for i in range(n4):
        st, rc, lp = o.table_slot(4, i)
        r = p["slot4"][i]
        assert (int(r["id_state"]), int(p["rc4"][i]), int(r["lport"])) == (st, rc, lp), i
        if (st & ST_MASK) != ST_EMPTY:
            s = socks[st & 0x3FFFFFFF]
            assert (int(r["raddr"]), int(r["rport"]), int(r["proto"])) == \
                (s.raddr_be32, s.rport_be16, s.protocol)
        else:
            assert int(r["raddr"]) == 0 and int(r["hwports"]) == 0
    for i in range(n6):
        st, rc, _ = o.table_slot(6, i)
        r = p["slot6"][i]
        assert (int(r["id"]) & 0xFFFFFFFF, int(r["route_count"])) == (st, rc), i
        if int(r["id"]) >= 0:
            s = socks[int(r["id"])]
            assert bytes(r["raddr"].tobytes()) == bytes(s.raddr6) and int(r["lport"]) == s.lport_be16


@pytest.mark.parametrize("af,log2,nops", [(4, 16, 3000), (6, 5, 800)])
def test_image_holds_reference_slot_state(af, log2, nops):
    rng = np.random.default_rng(11 + af)
    n_socks = 256
    kw = dict(max_socks=n_socks, ip4_log2=16, ip6_log2=log2 if af == 6 else 4)
    g = GpuRxStack(device=-1, **kw)
    o = OracleStack(**kw)
    socks = _socks(n_socks)
    for i, s in enumerate(socks):
        assert g.sock_set(i, s) == 0 and o.sock_set(i, s) == 0
    _run_script([g, o], _random_ops(rng, nops, af, n_socks, 40 if af == 6 else 2000))
    img = g.image_host()
    assert len(img) == g.image_bytes()
    _check_image_against_oracle(img, o, socks, 1 << 16, 1 << kw["ip6_log2"])

    # A fresh stack loaded from the image continues exactly like the oracle.
    h = GpuRxStack(device=-1, **kw)
    h.table_import(img.ctypes.data, img.nbytes)
    assert np.array_equal(h.image_host(), img)
    more = _random_ops(rng, nops // 2, af, n_socks, 40 if af == 6 else 2000)
    _run_script([h, o], more)
    _check_image_against_oracle(h.image_host(), o, socks, 1 << 16, 1 << kw["ip6_log2"])


def test_image_size_mismatch_rejected():
    a = GpuRxStack(device=-1, max_socks=64, ip6_log2=4)
    b = GpuRxStack(device=-1, max_socks=64, ip6_log2=5)
    img = a.image_host()
    with pytest.raises(OSError) as e:
        b.table_import(img.ctypes.data, img.nbytes)
    assert e.value.errno == errno.EINVAL
    with pytest.raises(OSError):
        a.table_export(img.ctypes.data, img.nbytes - 1)
