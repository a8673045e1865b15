# SPDX-License-Identifier: BSD-2-Clause
"""Outcomes observed by running the REFERENCE's own code (SURVEY.md §8(c),
"Verified results": the unmodified ci_udp_handle_rx / ci_tcp_handle_rx /
ci_netif_filter_for_each_match behind handle_rx_csum_bad), restated as
frames + expected records.  Plus the reference unit test's lookup order
(src/tests/unit/lib/transport/ip/tcp_rx.c:30-70)."""
from __future__ import annotations

import random

from onload_amd import _abi
from frames import eth, ip, ipv4, ipv6, tcp, udp, _sock

LA = ip("10.0.0.1")
PEER = ip("10.1.2.3")
LA6 = ip("fd00::1")
PEER6 = ip("fd00::2")

R = _abi


def survey_world():
    socks = {
        3: _sock(17, 6003),                                             # UDP 10.0.0.1:6003
        5: _sock(6, 5000, PEER, 40000, flags=_abi.SOCK_CONNECTED),      # TCP connected
        6: _sock(6, 80),                                                # laddr:80 listener
        7: _sock(6, 8080),                                              # *:8080 listener
        8: _sock(17, 6004),                                             # UDP6 [fd00::1]:6004
        9: _sock(6, 7443),                                              # TCP6 [::]:7443
    }
    filters = [
        (3, 4, LA, 6003, None, 0, 17),
        (5, 4, LA, 5000, PEER, 40000, 6),
        (6, 4, LA, 80, None, 0, 6),
        (7, 4, b"\0\0\0\0", 8080, None, 0, 6),
        (8, 6, LA6, 6004, None, 0, 17),
        (9, 6, bytes(16), 7443, None, 0, 6),
    ]
    return socks, filters


def survey_cases():
    """[(name, frame, intf_i, {field: expected})]."""
    rnd = random.Random(8)
    pay = lambda n: bytes(rnd.getrandbits(8) for _ in range(n))  # noqa: E731
    c = []

    def u4(n, **kw):
        ucs = kw.pop("ucsum", "ok")
        vlan = kw.pop("vlan", None)
        return eth(ipv4(PEER, LA, 17, udp(4, PEER, LA, 33000, kw.pop("dport", 6003), pay(n),
                                          csum=ucs), **kw), 0x0800, vlan=vlan)

    c.append(("udp 1514 good", u4(1472), 0, dict(reason=R.R_DELIVER, stage=2, sock=3)))
    c.append(("udp bad csum", u4(1472, ucsum="bad"), 0, dict(reason=R.R_UDP_CSUM)))
    c.append(("udp v4 csum 0", u4(1472, ucsum="zero"), 0,
              dict(reason=R.R_DELIVER, stage=2, sock=3)))
    c.append(("udp unbound port", u4(100, dport=6999), 0, dict(reason=R.R_NO_MATCH, sock=-1)))
    c.append(("vlan + odd payload", u4(33, vlan=12), 0,
              dict(reason=R.R_DELIVER, stage=2, sock=3, l4_off=38)))
    c.append(("ihl 8 nop options", u4(40, ihl=8, options=b"\x01" * 12), 0,
              dict(reason=R.R_DELIVER, stage=2, sock=3, l4_off=46)))
    t4 = lambda dst, sp, dp, n, **kw: eth(ipv4(PEER, dst, 6, tcp(4, PEER, dst, sp, dp, pay(n),  # noqa: E731
                                                                 csum=kw.pop("tcs", "ok")),
                                                **kw), 0x0800)
    c.append(("tcp connected", t4(LA, 40000, 5000, 100), 0,
              dict(reason=R.R_DELIVER, stage=1, sock=5)))
    c.append(("tcp laddr:80 listener", t4(LA, 40001, 80, 0), 0,
              dict(reason=R.R_DELIVER, stage=2, sock=6)))
    c.append(("tcp *:8080 listener", t4(ip("10.0.0.9"), 40002, 8080, 0), 0,
              dict(reason=R.R_DELIVER, stage=3, sock=7)))
    c.append(("tcp 9000 B jumbo", t4(LA, 40000, 5000, 8946), 0,
              dict(reason=R.R_DELIVER, stage=1, sock=5)))
    c.append(("tcp bad csum", t4(LA, 40000, 5000, 100, tcs="bad"), 0, dict(reason=R.R_TCP_CSUM)))
    c.append(("tcp MF valid csum", t4(LA, 40000, 5000, 100, frag=0x2000), 0,
              dict(reason=R.R_IP4_FRAG)))
    u6 = lambda n, cs="ok": eth(ipv6(PEER6, LA6, 17, udp(6, PEER6, LA6, 1000, 6004, pay(n),  # noqa: E731
                                                        csum=cs)), 0x86DD)
    c.append(("udp6 good", u6(200), 0, dict(reason=R.R_DELIVER, stage=2, sock=8)))
    c.append(("udp6 bad csum", u6(200, "bad"), 0, dict(reason=R.R_UDP_CSUM)))
    c.append(("udp6 csum 0", u6(200, "zero"), 0, dict(reason=R.R_UDP_CSUM)))
    c.append(("tcp6 syn [::]:7443",
              eth(ipv6(PEER6, LA6, 6, tcp(6, PEER6, LA6, 1000, 7443, b"", flags=0x02)), 0x86DD), 0,
              dict(reason=R.R_DELIVER, stage=3, sock=9)))
    return c


def order_world():
    """One socket per TCP lookup stage for the same packet (tcp_rx.c unit test)."""
    socks = {1: _sock(6, 443, PEER, 50000, flags=_abi.SOCK_CONNECTED), 2: _sock(6, 443),
             3: _sock(6, 443)}
    filters = [(1, 4, LA, 443, PEER, 50000, 6), (2, 4, LA, 443, None, 0, 6),
               (3, 4, b"\0\0\0\0", 443, None, 0, 6)]
    return socks, filters


def order_frame():
    return eth(ipv4(PEER, LA, 6, tcp(4, PEER, LA, 50000, 443, b"x" * 10)), 0x0800)
