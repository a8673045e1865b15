# SPDX-License-Identifier: BSD-2-Clause
"""Frame builder and edge corpus for parity tests.

Builds Ethernet (+802.1Q) / IPv4 (+options) / IPv6 / UDP / TCP (+options)
frames with correct or deliberately broken fields, and a socket world that
exercises every lookup stage, multicast (nmatch > 1), bind-to-device and
IPv6 wildcard/connected sockets.
"""
from __future__ import annotations

import ipaddress
import random
import struct

import numpy as np

from onload_amd import _abi
from onload_amd.rx import htons


def csum16(data: bytes, init: int = 0) -> int:
    """RFC 1071 folded sum (not complemented) of big-endian words."""
    if len(data) & 1:
        data = data + b"\0"
    s = init + sum(struct.unpack(f"!{len(data) // 2}H", data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def ip(a: str) -> bytes:
    return ipaddress.ip_address(a).packed


def eth(payload: bytes, ethertype: int, vlan: int | None = None, qinq: bool = False,
        dst: bytes = b"\x02\0\0\0\0\x01", src: bytes = b"\x02\0\0\0\0\x02") -> bytes:
    h = dst + src
    if qinq:
        h += struct.pack("!HH", 0x88A8, 100)
    if vlan is not None:
        h += struct.pack("!HH", 0x8100, vlan)
    return h + struct.pack("!H", ethertype) + payload


def ipv4(src: bytes, dst: bytes, proto: int, l4: bytes, ihl: int = 5, options: bytes = b"",
         tot_len: int | None = None, frag: int = 0x4000, version: int = 4,
         csum: str | int = "ok") -> bytes:
    opts = options.ljust((ihl - 5) * 4, b"\0")[: max(0, (ihl - 5) * 4)] if ihl > 5 else b""
    tl = (20 + len(opts) + len(l4)) if tot_len is None else tot_len
    h = struct.pack("!BBHHHBBH4s4s", (version << 4) | (ihl & 0xF), 0, tl & 0xFFFF, 0x1234,
                    frag, 64, proto, 0, src, dst) + opts
    if ihl < 5:
        h = h[: ihl * 4] + h[ihl * 4: 20]  # header bytes still present on the wire
    if csum == "ok":
        c = (~csum16(h[: max(ihl, 0) * 4])) & 0xFFFF if ihl >= 5 else 0
        h = h[:10] + struct.pack("!H", c) + h[12:]
    elif isinstance(csum, int):
        h = h[:10] + struct.pack("!H", csum) + h[12:]
    elif csum == "bad":
        c = (~csum16(h[: ihl * 4])) & 0xFFFF
        h = h[:10] + struct.pack("!H", c ^ 0x1111) + h[12:]
    return h + l4


def ipv6(src: bytes, dst: bytes, nh: int, l4: bytes, plen: int | None = None) -> bytes:
    pl = len(l4) if plen is None else plen
    return struct.pack("!IHBB16s16s", 0x60000000, pl & 0xFFFF, nh, 64, src, dst) + l4


def pseudo(af: int, src: bytes, dst: bytes, proto: int, length: int) -> int:
    return csum16(src + dst, 0) + proto + length if af == 4 else csum16(src + dst) + proto + length


def udp(af: int, src: bytes, dst: bytes, sport: int, dport: int, payload: bytes,
        ulen: int | None = None, csum: str | int = "ok") -> bytes:
    L = 8 + len(payload) if ulen is None else ulen
    h = struct.pack("!HHHH", sport, dport, L & 0xFFFF, 0) + payload
    if csum in ("ok", "bad", "ffff"):
        c = (~csum16(h[: max(0, min(L, len(h)))], pseudo(af, src, dst, 17, L))) & 0xFFFF
        if c == 0:
            c = 0xFFFF
        if csum == "bad":
            c ^= 0x0101
        h = h[:6] + struct.pack("!H", c) + h[8:]
    elif isinstance(csum, int):
        h = h[:6] + struct.pack("!H", csum) + h[8:]
    # csum == "zero": leave 0
    return h


def tcp(af: int, src: bytes, dst: bytes, sport: int, dport: int, payload: bytes,
        doff: int = 5, options: bytes = b"", csum: str | int = "ok", flags: int = 0x10,
        paylen_for_pseudo: int | None = None) -> bytes:
    opts = options.ljust(max(0, doff - 5) * 4, b"\x01")[: max(0, doff - 5) * 4]
    h = struct.pack("!HHIIBBHHH", sport, dport, 1000, 2000, (doff & 0xF) << 4, flags, 8192, 0,
                    0) + opts + payload
    if csum in ("ok", "bad", "zero_equiv"):
        L = len(h) if paylen_for_pseudo is None else paylen_for_pseudo
        c = (~csum16(h, pseudo(af, src, dst, 6, L))) & 0xFFFF
        if csum == "bad":
            c ^= 0x0202
        if csum == "zero_equiv":  # 0x0000 <-> 0xffff are the same in 1's complement
            c = 0xFFFF if c == 0 else (0 if c == 0xFFFF else c)
        h = h[:16] + struct.pack("!H", c) + h[18:]
    elif isinstance(csum, int):
        h = h[:16] + struct.pack("!H", csum) + h[18:]
    return h


# ---------------------------------------------------------------------------
# The edge world.

L4A = ip("10.0.0.1")
L6A = ip("fd00::1")
MC4 = ip("239.1.1.1")
PEER4 = ip("192.168.7.9")
PEER6 = ip("fd00:9::7")


def _sock(proto, lport=0, raddr4=b"\0\0\0\0", rport=0, raddr6=bytes(16), flags=0,
          b2d=False, hwports=0, vlan=0):
    s = _abi.Sock()
    s.raddr_be32 = int.from_bytes(raddr4, "little")
    s.rport_be16 = htons(rport)
    s.lport_be16 = htons(lport)
    s.protocol = proto
    s.flags = flags | (_abi.SOCK_BIND2DEV if b2d else 0)
    s.bind2dev_hwports = hwports
    s.bind2dev_vlan = vlan
    for i, b in enumerate(raddr6):
        s.raddr6[i] = b
    return s


def edge_world():
    """(socks dict id->Sock, filters list of (id, af, laddr, lport, raddr|None, rport, proto))."""
    socks, filters = {}, []

    def add(i, sock, af, la, lp, ra, rp, proto):
        socks[i] = sock
        filters.append((i, af, la, lp, ra, rp, proto))

    add(1, _sock(17, 5001), 4, L4A, 5001, None, 0, 17)                       # UDP unconnected
    add(2, _sock(17, 5002, PEER4, 7002, flags=_abi.SOCK_CONNECTED), 4, L4A, 5002, PEER4, 7002, 17)
    add(3, _sock(17, 5003), 4, L4A, 5003, None, 0, 17)
    add(4, _sock(17, 5000), 4, MC4, 5000, None, 0, 17)                       # multicast x2
    add(5, _sock(17, 5000), 4, MC4, 5000, None, 0, 17)
    add(6, _sock(6, 80, PEER4, 40000, flags=_abi.SOCK_CONNECTED), 4, L4A, 80, PEER4, 40000, 6)
    add(7, _sock(6, 80), 4, L4A, 80, None, 0, 6)                             # listener laddr
    add(8, _sock(6, 8080), 4, b"\0\0\0\0", 8080, None, 0, 6)                 # wildcard listener
    add(9, _sock(17, 5009, b2d=True, hwports=1 << 3, vlan=7), 4, L4A, 5009, None, 0, 17)
    add(10, _sock(17, 6001), 6, L6A, 6001, None, 0, 17)                      # UDP6 unconnected
    add(11, _sock(6, 443, raddr6=PEER6, rport=41000, flags=_abi.SOCK_CONNECTED), 6, L6A, 443,
        PEER6, 41000, 6)
    add(12, _sock(6, 7443), 6, bytes(16), 7443, None, 0, 6)                  # TCP6 [::]:7443
    add(13, _sock(6, 443), 6, L6A, 443, None, 0, 6)                          # TCP6 listener
    add(14, _sock(17, 6002, raddr6=PEER6, rport=7777, flags=_abi.SOCK_CONNECTED), 6, L6A, 6002,
        PEER6, 7777, 17)
    # an unconnected UDP socket beside the connected socket 2: a packet from
    # PEER4:7002 matches socket 2 in stage 1 and this one in stage 2 (the
    # future rule then gives up, udp_internal.h:41-52), others only this one
    add(15, _sock(17, 5002), 4, L4A, 5002, None, 0, 17)
    # a connected UDP socket alone on its port: its stage-1 match resolves
    # the future
    add(16, _sock(17, 5004, PEER4, 7004, flags=_abi.SOCK_CONNECTED), 4, L4A, 5004, PEER4, 7004, 17)
    return socks, filters


def install(stack, world):
    socks, filters = world
    for i, s in socks.items():
        assert stack.sock_set(i, s) == 0
    for (i, af, la, lp, ra, rp, proto) in filters:
        assert stack.filter_insert(i, af, la, lp, ra, rp, proto) == 0


# ---------------------------------------------------------------------------
# The edge corpus.

def _u4(sp, dp, pay, **kw):
    return eth(ipv4(kw.pop("src", PEER4), kw.pop("dst", L4A), 17,
                    udp(4, kw.pop("usrc", PEER4), kw.pop("udst", L4A), sp, dp, pay,
                        ulen=kw.pop("ulen", None), csum=kw.pop("ucsum", "ok")), **kw), 0x0800)


_TSO = b"\x01\x01\x08\x0a" + struct.pack("!II", 0x11223344, 0x55667788)
# (doff, options): the fast layout first, then near misses.
TSO_VARIANTS = ((8, _TSO), (9, _TSO + b"\x01" * 4), (7, _TSO[:8]),
                (8, b"\x01\x01\x08\x0b" + _TSO[4:]), (8, b"\x08\x0a" + _TSO[4:] + b"\x01\x01"),
                (8, b"\x01\x01\x05\x0a" + _TSO[4:]))


def edge_frames(seed: int = 1234) -> list[tuple[bytes, int]]:
    """List of (frame, intf_i)."""
    rnd = random.Random(seed)
    out: list[tuple[bytes, int]] = []

    def add(f, intf=0):
        out.append((bytes(f), intf))

    pay = lambda n: bytes(rnd.getrandbits(8) for _ in range(n))  # noqa: E731

    # -- UDP v4 basics: stage 1 (connected), stage 2, no match, multicast x2
    for n in (0, 1, 2, 3, 7, 8, 17, 22, 100, 1472, 1473, 2000, 8972):
        add(_u4(7002, 5002, pay(n)))
        add(_u4(33333, 5001, pay(n)))
        add(_u4(33333, 5999, pay(n)))
        add(_u4(7003, 5002, pay(n)))
        add(_u4(7004, 5004, pay(n)))
    add(_u4(1234, 5000, pay(30), dst=MC4, udst=MC4))
    add(eth(ipv4(PEER4, ip("255.255.255.255"), 17,
                 udp(4, PEER4, ip("255.255.255.255"), 1, 5001, pay(10))), 0x0800))
    # UDP checksum variants
    for c in ("zero", "bad", 0xFFFF, 0x0001):
        add(_u4(33333, 5001, pay(40), ucsum=c))
    # udp_len edge cases: 0, 7, 8, paylen-1, paylen, paylen+1
    for ul in (0, 7, 8, 47, 48, 49, 1000):
        add(_u4(33333, 5001, pay(40), ulen=ul))
        add(_u4(33333, 5001, pay(40), ulen=ul, ucsum="zero"))
    # IP length vs frame: tot_len +-1, tiny, ip_paylen <= 0
    base = udp(4, PEER4, L4A, 1, 5001, pay(40))
    for tl in (0, 1, 19, 20, 21, 27, 28, 47, 48, 49, 68, 69, 70, 65535):
        add(eth(ipv4(PEER4, L4A, 17, base, tot_len=tl), 0x0800))
    # trailing Ethernet padding beyond tot_len (allowed)
    add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(4))), 0x0800) + b"\0" * 12)
    # IHL 0..15 with valid-looking payload
    for ihl in range(16):
        add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(16)), ihl=ihl,
                     options=b"\x01" * 40), 0x0800))
    # version nibble != 4 (not checked by the reference)
    for v in (0, 5, 6, 15):
        add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(16)), version=v), 0x0800))
    # IP header checksum bad / 0xffff equivalence
    add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(16)), csum="bad"), 0x0800))
    # frag bits: reserved, DF, MF, offset, for UDP and TCP
    for fr in (0x0000, 0x4000, 0x8000, 0x2000, 0x0001, 0x1FFF, 0x6000, 0xC000, 0xE000):
        add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(16)), frag=fr), 0x0800))
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(16)), frag=fr), 0x0800))
        add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(16), csum="bad"), frag=fr),
                0x0800))
    # IP options
    opts = [b"\x00", b"\x01\x01\x01\x00", b"\x07\x07\x04" + b"\0" * 4, b"\x44\x04\x05\x00",
            b"\x82\x0b" + b"\0" * 9, b"\x88\x04\x00\x01", b"\x83\x07\x04" + b"\0" * 4,
            b"\x89\x07\x04" + b"\0" * 4, b"\x99\x04\0\0", b"\x07\x00", b"\x07\x03\0\0",
            b"\x07\x04\0\0", b"\x07\x28" + b"\0" * 38, b"\x07\x29", b"\x07\x80\0\0",
            b"\x07\xff\0\0", b"\x01\x07\x08" + b"\0" * 5 + b"\x44\x04\0\0", b"\x01" * 40,
            b"\x07\x08" + b"\0" * 6 + b"\x00\x83"]
    for o in opts:
        for ihl in (6, 7, 8, 15):
            add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(8)), ihl=ihl, options=o),
                    0x0800))
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(8)), ihl=8, options=o),
                0x0800))
    # option walk with MF set: frag wins over options
    add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(8)), ihl=7,
                 options=b"\x83\x07", frag=0x2000), 0x0800))
    # TCP: stages 1/2/3, doff 0..15, checksum variants, odd lengths, short
    for n in (0, 1, 2, 3, 5, 40, 1460, 8960):
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(n))), 0x0800))
        add(eth(ipv4(ip("10.9.9.9"), L4A, 6, tcp(4, ip("10.9.9.9"), L4A, 1234, 80, pay(n),
                                                  flags=0x02)), 0x0800))
        add(eth(ipv4(PEER4, ip("10.0.0.77"), 6, tcp(4, PEER4, ip("10.0.0.77"), 5, 8080, pay(n))),
                0x0800))
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 5, 9999, pay(n))), 0x0800))
    for doff in range(16):
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(24), doff=doff,
                                        options=b"\x02\x04\x05\xb4" + b"\x01" * 40)), 0x0800))
    for c in ("bad", "zero_equiv", 0, 0xFFFF):
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(33), csum=c)), 0x0800))
    for tl in (20 + 19, 20 + 20, 20 + 21):  # ip_paylen around sizeof(tcp hdr)
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, b""), tot_len=tl), 0x0800))
    # VLAN: tagged, QinQ, bind2dev (intf with hwport 3 on vlan 7 matches socket 9)
    add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(31))), 0x0800, vlan=7))
    add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(31))), 0x0800, vlan=0x2ABC))
    add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(31))), 0x0800, vlan=7,
            qinq=True))
    for intf in (0, 1, 2, 5, 31, -1):
        for vl in (None, 7, 8):
            add(eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5009, pay(9))), 0x0800, vlan=vl),
                intf)
    # non-IP ethertypes and short frames
    for et in (0x0806, 0x88CC, 0x0000, 0xFFFF, 0x86DE):
        add(eth(pay(50), et))
    full = _u4(33333, 5001, pay(20))
    for n in range(0, 44):
        add(full[:n])
    vfull = eth(ipv4(PEER4, L4A, 17, udp(4, PEER4, L4A, 1, 5001, pay(20))), 0x0800, vlan=5)
    for n in (16, 17, 18, 37, 38, 41, 42):
        add(vfull[:n])
    # other IP protocols
    for proto in (0, 1, 2, 47, 132, 255):
        add(eth(ipv4(PEER4, L4A, proto, pay(40)), 0x0800))
        add(eth(ipv6(PEER6, L6A, proto, pay(40)), 0x86DD))
    # IPv6: UDP stage 1/2, csum 0 (must verify on v6), TCP stages, payload_len edges
    for n in (0, 1, 9, 100, 1400, 8900):
        add(eth(ipv6(PEER6, L6A, 17, udp(6, PEER6, L6A, 7777, 6002, pay(n))), 0x86DD))
        add(eth(ipv6(PEER6, L6A, 17, udp(6, PEER6, L6A, 1111, 6001, pay(n))), 0x86DD))
        add(eth(ipv6(PEER6, L6A, 6, tcp(6, PEER6, L6A, 41000, 443, pay(n))), 0x86DD))
        add(eth(ipv6(ip("fd00:5::5"), L6A, 6, tcp(6, ip("fd00:5::5"), L6A, 2, 443, pay(n),
                                                   flags=0x02)), 0x86DD))
        add(eth(ipv6(ip("fd00:5::5"), ip("fd00::99"), 6,
                     tcp(6, ip("fd00:5::5"), ip("fd00::99"), 2, 7443, pay(n), flags=0x02)), 0x86DD))
    add(eth(ipv6(PEER6, L6A, 17, udp(6, PEER6, L6A, 1111, 6001, pay(20), csum="zero")), 0x86DD))
    add(eth(ipv6(PEER6, L6A, 17, udp(6, PEER6, L6A, 1111, 6001, pay(20), csum="bad")), 0x86DD))
    add(eth(ipv6(PEER6, L6A, 6, tcp(6, PEER6, L6A, 41000, 443, pay(20), csum="bad")), 0x86DD))
    u6 = udp(6, PEER6, L6A, 1111, 6001, pay(40))
    for pl in (0, 1, 7, 8, 47, 48, 49, 65535):
        add(eth(ipv6(PEER6, L6A, 17, u6, plen=pl), 0x86DD))
    add(eth(ipv6(PEER6, L6A, 17, udp(6, PEER6, L6A, 1111, 6001, pay(40))), 0x86DD, vlan=3))
    # IPv6 multicast destination (mcast flag comes from bytes 16..19 of the L3 header)
    add(eth(ipv6(ip("fd00::e000:1"), ip("ff02::1"), 17,
                 udp(6, ip("fd00::e000:1"), ip("ff02::1"), 1, 6001, pay(8))), 0x86DD))
    # random garbage frames
    for _ in range(200):
        n = rnd.randrange(0, 300)
        b = bytearray(pay(n))
        if n > 14 and rnd.random() < 0.7:
            b[12:14] = rnd.choice([b"\x08\x00", b"\x86\xdd", b"\x81\x00"])
        add(bytes(b))
    # random mutations of valid frames (single-byte flips in headers)
    seeds = [_u4(33333, 5001, pay(64)),
             eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(64))), 0x0800),
             eth(ipv6(PEER6, L6A, 6, tcp(6, PEER6, L6A, 41000, 443, pay(64))), 0x86DD)]
    for _ in range(600):
        b = bytearray(rnd.choice(seeds))
        k = rnd.randrange(12, 14 + 60)
        b[k] ^= 1 << rnd.randrange(8)
        add(bytes(b))
    # TCP timestamp-option fast layout (tcp_rx.c:4537-4543): doff 8 with the
    # options word NOP NOP TS 10; near misses (doff 7/9, other option words),
    # a bad checksum, VLAN, IPv6, frames long enough to need the body.
    for doff, opts in TSO_VARIANTS:
        for n in (0, 13, 1200):
            add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(n), doff=doff,
                                            options=opts)), 0x0800))
            add(eth(ipv6(PEER6, L6A, 6, tcp(6, PEER6, L6A, 41000, 443, pay(n), doff=doff,
                                            options=opts)), 0x86DD))
        add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(5), doff=doff,
                                        options=opts)), 0x0800, vlan=7))
        for n in (5, 1500):
            add(eth(ipv4(PEER4, L4A, 6, tcp(4, PEER4, L4A, 40000, 80, pay(n), doff=doff,
                                            options=opts, csum="bad")), 0x0800))
    return out


def pack(frames: list[tuple[bytes, int]], align: int = 64, shift: int = 0):
    """Pack frames into one buffer: offsets aligned to `align` plus `shift`."""
    desc = np.zeros(len(frames), dtype=_abi.DESC_DTYPE)
    off = 0
    chunks = []
    for i, (f, intf) in enumerate(frames):
        start = off + shift
        desc[i]["frame_off"] = start
        desc[i]["len"] = len(f)
        desc[i]["intf_i"] = intf
        slot = ((shift + len(f) + align - 1) // align) * align
        chunks.append(b"\xee" * shift + f + b"\xee" * (slot - shift - len(f)))
        off += slot
    buf = np.frombuffer(b"".join(chunks) + b"\xee" * 64, dtype=np.uint8).copy()
    return buf, desc
