# SPDX-License-Identifier: BSD-2-Clause
"""The oracle reproduces the reference-run outcomes of SURVEY.md §8(c) and the
lookup order pinned by the reference's tcp_rx unit test."""
import numpy as np
import pytest

import cases
from frames import install, pack
from oracle_lib import OracleStack


@pytest.mark.parametrize("case", cases.survey_cases(), ids=lambda c: c[0])
def test_survey_case(case):
    name, frame, intf, want = case
    st = OracleStack()
    install(st, cases.survey_world())
    buf, desc = pack([(frame, intf)])
    r = st.handle_rx_batch(buf, desc)[0]
    for k, v in want.items():
        assert r[k] == v, (name, k, r[k], v)


def test_tcp_lookup_order():
    """(daddr,dport,saddr,sport) -> (daddr,dport,0,0) -> (0,dport,0,0)
    (src/tests/unit/lib/transport/ip/tcp_rx.c:42-66)."""
    st = OracleStack()
    socks, filters = cases.order_world()
    install(st, (socks, filters))
    buf, desc = pack([(cases.order_frame(), 0)])
    for stage, sock in ((1, 1), (2, 2), (3, 3)):
        r = st.handle_rx_batch(buf, desc)[0]
        assert (r["stage"], r["sock"]) == (stage, sock)
        f = filters[stage - 1]
        st.filter_remove(*f)
    r = st.handle_rx_batch(buf, desc)[0]
    assert r["reason"] == 1 and r["sock"] == -1  # NO_MATCH


def test_udp_multicast_counts_all_matches():
    from frames import edge_world, eth, ipv4, udp, MC4, PEER4
    st = OracleStack()
    install(st, edge_world())
    f = eth(ipv4(PEER4, MC4, 17, udp(4, PEER4, MC4, 1, 5000, b"abc")), 0x0800)
    buf, desc = pack([(f, 0)])
    r = st.handle_rx_batch(buf, desc)[0]
    assert r["reason"] == 0 and r["nmatch"] == 2 and r["flags"] & 0x18 == 0x18
    assert r["sock"] in (4, 5)


def test_batch_threads_agree():
    from frames import edge_frames, edge_world
    st = OracleStack()
    install(st, edge_world())
    buf, desc = pack(edge_frames())
    a = st.handle_rx_batch(buf, desc, nthreads=1)
    b = st.handle_rx_batch(buf, desc, nthreads=4)
    assert a.tobytes() == b.tobytes()
    # every reason the corpus is meant to reach is reached
    reasons = set(np.unique(a["reason"]).tolist())
    assert {0, 1, 2, 3, 4, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25} <= reasons, reasons


def test_tcp_timestamp_fast_layout_flag():
    """OO_RX_F_TSO exactly for TCP headers of length 32 whose first options
    word is NOP NOP TIMESTAMP 10 (tcp_rx.c:4537-4543), checksum passed."""
    from frames import L4A, L6A, PEER4, PEER6, TSO_VARIANTS, edge_world, eth, ipv4, ipv6, tcp
    from onload_amd import _abi
    st = OracleStack()
    install(st, edge_world())
    for k, (doff, opts) in enumerate(TSO_VARIANTS):
        for af in (4, 6):
            for csum in ("ok", "bad"):
                if af == 4:
                    f = eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, b"xy" * 9, doff=doff,
                                                    options=opts, csum=csum)), 0x0800)
                else:
                    f = eth(ipv6(PEER6, L6A, 6, tcp(6, PEER6, L6A, 41000, 443, b"xy" * 9,
                                                    doff=doff, options=opts, csum=csum)), 0x86DD)
                buf, desc = pack([(f, 0)])
                r = st.handle_rx_batch(buf, desc)[0]
                want = k == 0 and csum == "ok"
                assert bool(r["flags"] & _abi.F_TSO) == want, (k, af, csum, r)
