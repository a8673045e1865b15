# SPDX-License-Identifier: BSD-2-Clause
"""Seeded filter-table scripts for pinning the table half of the oracle, the
host mirror (onload_amd/csrc/oo_gpu_rx.cpp) and the device table kernels
against the reference's own netif_table.c / netif_table_ip6.c
(oracle/_ref/ref_table, tests/golden/make_table_golden.py).

A script is fully determined by its name (numpy PCG64 streams): the sockets,
the insert/remove sequence, the checkpoints and the queries are regenerated
here on any machine; the fixture holds only what the reference answered --
each operation's return code, the table dump at each checkpoint (rows, or a
SHA-256 for the large tables), slot-lookup results and per-stage match
walks (count, first socket, hash)."""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass, field

import numpy as np

SCRIPTS = {
    # name: (seed, ip4_log2, ip6_log2, nsocks, n_ops, p_insert, hwports)
    "mixed": (11, 16, 6, 700, 6000, 0.62, (0, 1, 3, 2)),
    "churn": (12, 16, 8, 4000, 60000, 0.55, (0, 2)),
    "ip6_full": (13, 16, 4, 64, 400, 0.8, (0,)),
    "ip4_full": (14, 16, 4, 8, 0, 0.0, (0,)),  # ops built separately: fill to -ENOBUFS
}
CHECKPOINTS = 3


@dataclass
class Sock:
    id: int
    af: int
    proto: int
    lport: int          # BE value in a host integer
    rport: int
    raddr: bytes        # 4 or 16 bytes, zeros when unconnected
    connected: bool
    b2d: bool = False
    hwports: int = 0
    vlan: int = 0
    laddrs: set = field(default_factory=set)


def be(port: int) -> int:
    return ((port & 0xff) << 8) | (port >> 8)


def _pools(rng):
    l4 = [bytes([10, 0, int(a), int(b)]) for a, b in rng.integers(0, 256, (48, 2))]
    r4 = [bytes([192, 168, int(a), int(b)]) for a, b in rng.integers(0, 256, (512, 2))]
    l6 = [bytes([0xfd, 0, 0, 0]) + bytes(rng.integers(0, 256, 12, dtype=np.uint8))
          for _ in range(24)]
    r6 = [bytes([0xfd, 9, 0, 0]) + bytes(rng.integers(0, 256, 12, dtype=np.uint8))
          for _ in range(256)]
    return l4, r4, l6, r6


def build(name: str):
    """-> (cfg dict, socks list, ops list).  An op is a tuple:
    ("A"|"R", af, sock, laddr, lport, raddr|None, rport, proto)
    ("C", k)                      checkpoint k (dump + queries)."""
    seed, log4, log6, nsocks, n_ops, p_ins, hw = SCRIPTS[name]
    rng = np.random.default_rng(seed)
    l4, r4, l6, r6 = _pools(rng)
    cfg = dict(log4=log4, log6=log6, nsocks=nsocks, hwports=hw)
    socks = []
    for i in range(nsocks):
        af = 6 if (name == "ip6_full" or rng.random() < 0.3) and name != "ip4_full" else 4
        proto = 6 if rng.random() < 0.5 else 17
        lport = be(int(rng.integers(1, 400)) + (5000 if proto == 17 else 8000))
        connected = rng.random() < 0.5
        raddr = ((r6 if af == 6 else r4)[int(rng.integers(0, 256 if af == 6 else 512))]
                 if connected else bytes(16 if af == 6 else 4))
        rport = be(int(rng.integers(30000, 61000))) if connected else 0
        s = Sock(i, af, proto, lport, rport, raddr, connected)
        if rng.random() < 0.05:
            s.b2d = True
            s.hwports = int(rng.integers(1, 16))
            s.vlan = int(rng.choice([0, 7]))
        socks.append(s)
    ops = []
    live = []  # (sock, laddr)
    if name == "ip4_full":
        # 2^16 + 1 distinct connected 4-tuples over the 8 sockets' fields:
        # the last insert finds the table full (-ENOBUFS, netif_table.c:375)
        for k in range((1 << log4) + 1):
            s = socks[k % nsocks]
            la = struct.pack(">I", 0x0a000000 + k)  # distinct laddr per filter
            ops.append(("A", 4, s.id, la, s.lport, s.raddr if s.connected else None,
                        s.rport, s.proto))
            if k in (1 << 15, 1 << 16):
                ops.append(("C", len([o for o in ops if o[0] == "C"])))
        ops.append(("C", 2))
        return cfg, socks, ops
    per = max(1, n_ops // CHECKPOINTS)
    for k in range(n_ops):
        if live and rng.random() >= p_ins:
            if rng.random() < 0.05:  # remove of an absent filter (a no-op, :476-481)
                s = socks[int(rng.integers(0, nsocks))]
                la = (l6 if s.af == 6 else l4)[int(rng.integers(0, len(l6 if s.af == 6 else l4)))]
                if la in s.laddrs:
                    continue
            else:
                j = int(rng.integers(0, len(live)))
                sid, la = live[j]
                live[j] = live[-1]
                live.pop()
                s = socks[sid]
                s.laddrs.discard(la)
            ops.append(("R", s.af, s.id, la, s.lport, s.raddr if s.connected else None,
                        s.rport, s.proto))
        else:
            s = socks[int(rng.integers(0, nsocks))]
            pool = l6 if s.af == 6 else l4
            if not s.connected and rng.random() < 0.15:
                la = bytes(16 if s.af == 6 else 4)  # wildcard laddr
            else:
                la = pool[int(rng.integers(0, len(pool)))]
            if la in s.laddrs:  # one entry per (socket, laddr) (netif_table.c:357-358)
                continue
            s.laddrs.add(la)
            live.append((s.id, la))
            ops.append(("A", s.af, s.id, la, s.lport, s.raddr if s.connected else None,
                        s.rport, s.proto))
        if (k + 1) % per == 0:
            ops.append(("C", len([o for o in ops if o[0] == "C"])))
    return cfg, socks, ops


def queries(name: str, socks, live_filters, k: int):
    """Queries for checkpoint k: exact slot lookups and packet-shaped match
    tuples (af, proto, laddr, lport, raddr, rport, intf, vlan)."""
    seed = SCRIPTS[name][0]
    rng = np.random.default_rng([seed, 1000 + k])
    l4, r4, l6, r6 = _pools(np.random.default_rng(seed))
    nintf = len(SCRIPTS[name][6])
    looks, matches = [], []
    lf = list(live_filters)
    for _ in range(600):
        if lf and rng.random() < 0.7:
            af, sid, la, lp, ra, rp, proto = lf[int(rng.integers(0, len(lf)))]
        else:
            s = socks[int(rng.integers(0, len(socks)))]
            af, la, lp, proto = s.af, (l6 if s.af == 6 else l4)[int(rng.integers(0, 8))], s.lport, s.proto
            ra, rp = (s.raddr, s.rport) if rng.random() < 0.5 else (None, 0)
        looks.append((af, la, lp, ra, rp, proto))
    for _ in range(900):
        if lf and rng.random() < 0.8:
            af, sid, la, lp, ra, rp, proto = lf[int(rng.integers(0, len(lf)))]
            s = socks[sid]
            if ra is None:  # listener / unconnected: any peer
                ra = (r6 if af == 6 else r4)[int(rng.integers(0, 256))]
                rp = be(int(rng.integers(30000, 61000)))
            if not any(la):  # wildcard laddr: any local address
                la = (l6 if af == 6 else l4)[int(rng.integers(0, 8))]
            if rng.random() < 0.1:
                rp = be(int(rng.integers(30000, 61000)))
        else:
            af = 6 if rng.random() < 0.3 else 4
            proto = 6 if rng.random() < 0.5 else 17
            la = (l6 if af == 6 else l4)[int(rng.integers(0, 8))]
            lp = be(int(rng.integers(1, 400)) + (5000 if proto == 17 else 8000))
            ra = (r6 if af == 6 else r4)[int(rng.integers(0, 256))]
            rp = be(int(rng.integers(30000, 61000)))
        intf = int(rng.integers(0, nintf))
        vlan = int(rng.choice([0, 0, 7]))
        matches.append((af, proto, la, lp, ra, rp, intf, vlan))
    return looks, matches


def live_at(ops, upto: int):
    """Filters inserted and not removed by ops[:upto] (whatever the inserts
    returned), as (af, sock, laddr, lport, raddr, rport, proto): the query
    generator's view, independent of the answers."""
    live = {}
    for o in ops[:upto]:
        if o[0] == "A":
            live[(o[2], o[3])] = (o[1], o[2], o[3], o[4], o[5], o[6], o[7])
        elif o[0] == "R":
            live.pop((o[2], o[3]), None)
    return list(live.values())


def match_stages(q):
    """The lookup stages a packet of query q makes (udp_rx.c:271-306,
    tcp_rx.c:4786-4835): (laddr, lport, raddr|None, rport) per stage."""
    af, proto, la, lp, ra, rp, intf, vlan = q
    z = bytes(16 if af == 6 else 4)
    st = [(la, lp, ra, rp), (la, lp, None, 0)]
    if proto == 6:
        st.append((z, lp, None, 0))
    return st


def hexs(a):
    return "-" if a is None else a.hex()


def dump_digest(rows4: np.ndarray, rows6: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(rows4, dtype="<i8").tobytes())
    h.update(np.ascontiguousarray(rows6, dtype="<i8").tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------------------
# Replaying a script on a stack (GpuRxStack, OracleStack) and reading it back.

def sock_struct(s: Sock):
    from onload_amd import _abi
    o = _abi.Sock()
    o.protocol = s.proto
    o.lport_be16 = s.lport
    o.rport_be16 = s.rport
    if s.af == 4:
        o.raddr_be32 = int.from_bytes(s.raddr, "little")
    else:
        for i, b in enumerate(s.raddr):
            o.raddr6[i] = b
    o.flags = (_abi.SOCK_CONNECTED if s.connected else 0) | (_abi.SOCK_BIND2DEV if s.b2d else 0)
    o.bind2dev_hwports = s.hwports
    o.bind2dev_vlan = s.vlan
    return o


def replay(stack, socks, ops, at_checkpoint=None, upto=None):
    """Sockets, then the inserts/removes in order; returns their return codes.
    at_checkpoint(k, i) runs at each checkpoint (i = op index)."""
    for s in socks:
        assert stack.sock_set(s.id, sock_struct(s)) == 0
    rcs = []
    for i, o in enumerate(ops[:upto]):
        if o[0] == "A":
            rcs.append(stack.filter_insert_raw(o[2], o[1], o[3], o[4], o[5], o[6], o[7]))
        elif o[0] == "R":
            rc = stack.filter_remove_raw(o[2], o[1], o[3], o[4], o[5], o[6], o[7])
            rcs.append(0 if rc is None else rc)
        elif at_checkpoint is not None:
            at_checkpoint(o[1], i)
    return rcs


def image_rows(img) -> np.ndarray:
    """The sparse dump rows of a table image (oo_gpu_rx_table_export)."""
    from onload_amd import _abi
    p = _abi.parse_image(img)
    s4, rc4, s6 = p["slot4"], p["rc4"].astype(np.int64), p["slot6"]
    ids = s4["id_state"].astype(np.int64)
    la = s4["laddr"].astype(np.int64)
    lp = s4["lport"].astype(np.int64)
    keep = (ids != 0x80000000) | (la != 0) | (rc4 != 0) | (lp != 0)
    i4 = np.nonzero(keep)[0]
    r4 = np.stack([np.full(len(i4), 4), i4, ids[i4], la[i4], rc4[i4], lp[i4]], axis=1)
    la6 = np.ascontiguousarray(s6["laddr"]).view(np.int64).reshape(-1, 2)
    id6 = s6["id"].astype(np.int64)
    rc6 = s6["route_count"].astype(np.int64)
    keep6 = (id6 != -2) | (rc6 != 0) | (la6[:, 0] != 0) | (la6[:, 1] != 0)
    i6 = np.nonzero(keep6)[0]
    r6 = np.stack([np.full(len(i6), 6), i6, id6[i6], rc6[i6], la6[i6, 0], la6[i6, 1]], axis=1)
    return np.concatenate([r4.reshape(-1, 6), r6.reshape(-1, 6)]).astype(np.int64)


def check_dump(rows: np.ndarray, golden, name: str, k: int):
    key = f"{name}/dump{k}"
    if key in golden:
        want = golden[key]
        assert rows.shape == want.shape, (rows.shape, want.shape)
        bad = np.nonzero((rows != want).any(axis=1))[0]
        assert len(bad) == 0, f"first differing rows: got {rows[bad[:3]]} want {want[bad[:3]]}"
    else:
        d = dump_digest(rows[rows[:, 0] == 4], rows[rows[:, 0] == 6])
        assert d == golden[f"{name}/digest{k}"].tobytes().decode()


def folded_lookup(stack, look) -> int:
    """What the fixture's slot lookup answers (ci_ip6_netif_filter_lookup,
    or __ci_ip4_netif_filter_lookup: the exact tuple, then (laddr, lport,
    0, 0), else -ENOENT; netif_table.c:617-645) from a stack's exact
    lookups (oo_gpu_rx_table_lookup / the oracle's)."""
    af, la, lp, ra, rp, proto = look
    if af == 6:
        return stack.filter_lookup_raw(6, la, lp, ra, rp, proto)
    rc = stack.filter_lookup_raw(4, la, lp, ra if ra is not None else bytes(4), rp, proto)
    if rc >= 0:
        return rc
    rc = stack.filter_lookup_raw(4, la, lp, bytes(4), 0, proto)
    return rc if rc >= 0 else -2  # -ENOENT


def frame_for(q) -> bytes:
    """A well-formed frame whose demux asks exactly query q's stages: the
    peer (raddr, rport) sends to (laddr, lport), tagged with q's VLAN."""
    from frames import eth, ipv4, ipv6, tcp, udp
    af, proto, la, lp, ra, rp, intf, vlan = q
    sport, dport = be(rp), be(lp)
    pay = bytes(range(37))
    l4 = (udp(af, ra, la, sport, dport, pay) if proto == 17
          else tcp(af, ra, la, sport, dport, pay))
    l3 = ipv4(ra, la, proto, l4) if af == 4 else ipv6(ra, la, proto, l4)
    return eth(l3, 0x0800 if af == 4 else 0x86DD, vlan=vlan if vlan else None)


def expected_records(matches, m):
    """Per query: (stage, sock, nmatch, hash3) from the reference's per-stage
    walks m[j] = [(n, first, hash)] * 3 -- the first stage with a match
    decides (udp_rx.c:292-306, tcp_rx.c:4814-4835); hash3 is stage 1's.  The
    harness walks to the end with a callback that accepts nothing; TCP's
    callbacks accept the first match and so end the walk there
    (tcp_rx.c:4644-4657), so a TCP query counts one match."""
    out = []
    for j, q in enumerate(matches):
        st, sock, n = 0, -1, 0
        for s in range(len(match_stages(q))):
            if m[j, s, 0] > 0:
                st, sock, n = s + 1, int(m[j, s, 1]), int(m[j, s, 0])
                if q[1] == 6:
                    n = 1
                break
        out.append((st, sock, n, int(m[j, 0, 2]) & 0xffffffff))
    return out
