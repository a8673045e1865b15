# SPDX-License-Identifier: BSD-2-Clause
"""Test side of the batched RX branch (include/oo_rx_poll.h).

``Recorder`` is the fake callback table: it logs every call in order and
declines chosen futures (a full recvq).  ``expect`` restates, from the
reference, what the poll loop does with each event and record -- the
dispatch decision and the counters -- independently of the shim's code:

* per event: netif_event.c:1715-1742 (plain RX: rx_evs, whole-buffer test
  :1729-1736) and discard_rx_multi_pkts :1131-1191 (class counter
  :1164-1172, checksum class + not fragmented :1155-1162, release :1175-1183,
  double count :1189-1190);
* per record: handle_rx_csum_bad's drop counters :1031-1116, handle_rx_pkt's
  not_fast split :293-303 and counters :282/:327/:332/:384/:394/:400,
  ci_ip_options_parse's ip_options :181, the future rules
  tcp_rx.h:150-184 / udp_internal.h:41-103 and their in_segs / in_dgrams,
  post-future fallbacks tcp_rx.h:198-214 / udp_internal.h:116-134."""
from __future__ import annotations

from collections import Counter

import numpy as np

from hostmem import page_buffer, whole_pages
from onload_amd import _abi, poll

CSUM_CLASS = poll.DISCARD_L3_CSUM_ERR | poll.DISCARD_L4_CSUM_ERR | poll.DISCARD_L3_CLASS_OTHER


class Recorder:
    def __init__(self, decline=lambda rq_id: False):
        self.calls = []
        self.recs = []  # every record a callback received, in call order
        self.decline = decline

    def post_future(self, i, r, f):
        self.recs.append(r)
        if self.decline(i):
            self.calls.append(("declined", i, r["sock"]))
            return 1
        self.calls.append(("future", i, r["sock"], f["hash"], f["seq"], f["ack"], f["pay_len"],
                           f["l4_off"], f["ip_paylen"]))
        return 0

    def full_handler(self, i, r):
        if not self.calls or self.calls[-1][:2] != ("declined", i):
            self.recs.append(r)
        self.calls.append(("full", i, r["reason"]))

    def pkt_handler(self, i, r):
        self.recs.append(r)
        self.calls.append(("pkt", i, r["reason"]))

    def release(self, i, r):
        if r is not None:
            self.recs.append(r)
        self.calls.append(("release", i, None if r is None else r["reason"]))

    def other_ev(self, e):
        self.calls.append(("other", int(e["rq_id"])))


def in_pool(e, buf_size, pool_bytes):
    """The frame lies inside its own buffer of the pool."""
    off = int(e["rq_id"]) * buf_size + int(e["ofs"])
    return int(e["ofs"]) + int(e["len"]) <= buf_size and off + int(e["len"]) <= pool_bytes


def udp_pre_future(stages):
    """ci_udp_handle_rx_pre_future (udp_internal.h:58-103) over the matches of
    its two lookups -- (laddr, lport, raddr, rport) then (laddr, lport), each
    a list of socket ids in walk order -- with ci_udp_rx_deliver_to_future
    (:41-52) as the callback, every recvq having room (a full one is the
    declined-future case): the socket the future resolves, or None."""
    sock = None
    for matches in stages:
        dealt = False
        for s in matches:
            if sock is not None:  # :47-50 a second socket: give the future up
                sock = None
                dealt = True
                break
            sock = s              # :52-53 keep walking for another
        if dealt:                 # the walk returned 1: stage 2 is skipped (:93-97)
            break
    return sock


def udp_stage_matches(oracle, r, intf_i):
    """The two IPv4 UDP lookups of a record's packet, on the oracle's tables
    (ci_netif_filter_for_each_match restated): lists of socket ids with the
    first one known (only the first and the count matter to the rule)."""
    out = []
    for ra, rp in ((int(r["saddr_be"]), int(r["sport_be"])), (0, 0)):
        n, first = oracle.walk4(int(r["daddr_be"]), int(r["dport_be"]), ra, rp, 17, intf_i,
                                int(r["vlan"]))
        out.append([first] + [-2] * (n - 1) if n else [])
    return out


def transformed(e, sw_verify, buf_size, pool_bytes) -> bool:
    whole = (int(e["flags"]) & (poll.EV_SOP | poll.EV_CONT)) == poll.EV_SOP
    ok = whole and in_pool(e, buf_size, pool_bytes)
    if int(e["discard"]) == 0:
        return bool(sw_verify and ok)
    return bool(int(e["discard"]) & CSUM_CLASS and ok)


def expect(evs, recs, pool, buf_size, sw_verify, decline, oracle):
    """The calls and counters the reference loop would produce.  recs: the
    oracle's records of the transformed events, in event order; oracle: an
    OracleStack holding the same tables (the UDP future rule walks them).
    rx_evs of the events handed back (other_ev) is the caller loop's to count
    (netif_event.c:1718), not the shim's."""
    st = Counter()
    calls = []
    k = 0
    for e in evs:
        i, d = int(e["rq_id"]), int(e["discard"])
        if d == 0:
            if transformed(e, sw_verify, buf_size, pool.nbytes):
                st["rx_evs"] += 1
        elif d & poll.DISCARD_ETH_LEN_ERR:
            st["rx_discard_len_err"] += 1
        elif d & poll.DISCARD_ETH_FCS_ERR:
            st["rx_discard_crc_bad"] += 1
        elif d & (poll.DISCARD_L3_CSUM_ERR | poll.DISCARD_L4_CSUM_ERR):
            st["rx_discard_csum_bad"] += 1
        else:
            st["rx_discard_other"] += 1
        if not transformed(e, sw_verify, buf_size, pool.nbytes):
            calls.append(("other", i) if d == 0 else ("release", i, None))
            continue
        r = recs[k]
        k += 1
        reason = int(r["reason"])
        if reason >= _abi.R_DROP_BASE:
            st[{_abi.R_SHORT_L2: "in_hdr_errs", _abi.R_IP4_LEN: "in_hdr_errs",
                _abi.R_IP4_CSUM: "in_hdr_errs", _abi.R_IP6_LEN: "in6_hdr_errs",
                _abi.R_UDP_CSUM: "udp_in_errs"}.get(reason, "none")] += 1
            calls.append(("release", i, reason))
            continue
        if d:
            st["rx_evs"] += 1
            st["rx_sw_csum_pass"] += 1
        if reason in (_abi.R_IP4_FRAG, _abi.R_IP4_OPTS_BAD):
            calls.append(("pkt", i, reason))
            continue
        is6 = bool(r["flags"] & _abi.F_IP6)
        st["in6_recvs" if is6 else "in_recvs"] += 1
        pre_l3 = 18 if r["flags"] & _abi.F_VLAN else 14
        if not is6 and r["l4_off"] > pre_l3 + 20:
            st["ip_options"] += 1
        # The future seam (IPv4 only): TCP's pre-future walks stage 1 alone
        # (tcp_rx.h:150-184); UDP's walks both stages with the give-up rule.
        fut = False
        if not is6 and reason in (_abi.R_DELIVER, _abi.R_NO_MATCH):
            if r["proto"] == 6:
                fut = reason == _abi.R_DELIVER and r["stage"] == 1
            elif r["proto"] == 17:
                sock = udp_pre_future(udp_stage_matches(oracle, r, int(e["intf_i"])))
                fut = sock is not None
                assert not fut or sock == int(r["sock"]), (sock, r)
        if fut and not decline(i):
            frame = pool[int(e["rq_id"]) * buf_size + int(e["ofs"]):]
            l4 = int(r["l4_off"])
            be32 = lambda o: int.from_bytes(frame[l4 + o:l4 + o + 4].tobytes(), "big")  # noqa
            if r["proto"] == 6:
                f = (int(r["hash3"]), be32(4), be32(8), int(r["ip_paylen"]))
                st["tcp_in_segs"] += 1
            else:
                udp_len = int.from_bytes(frame[l4 + 4:l4 + 6].tobytes(), "big")
                f = (0, 0, 0, (udp_len - 8) & 0xffffffff)
                st["udp_in_dgrams"] += 1
            calls.append(("future", i, int(r["sock"])) + f + (l4, int(r["ip_paylen"])))
        else:
            if fut:
                calls.append(("declined", i, int(r["sock"])))
            calls.append(("full", i, reason))
        st["in6_delivers" if is6 else "in_delivers"] += 1
    st.pop("none", None)
    return calls, st


def onload_stats(stats: dict) -> Counter:
    """The Onload-named counters of oo_rx_poll_stats (the n_* tallies are the
    shim's own)."""
    return Counter({k: v for k, v in stats.items() if v and not k.startswith("n_")})


def events_for(frames, buf_size, rng, discard_mix=True):
    """A pool with one frame per buffer and one event per frame: mostly
    whole-buffer RX events; with discard_mix, also discard events of every
    class, multi-buffer events and events pointing outside the pool."""
    n = len(frames)
    pool = page_buffer(whole_pages((n + 1) * buf_size))  # whole pages: registrable
    evs = np.zeros(n, dtype=poll.EV_DTYPE)
    for i, (f, intf) in enumerate(frames):
        ofs = int(rng.choice([192, 192, 193, 256, 0, 255]))
        assert ofs + len(f) <= buf_size
        pool[i * buf_size + ofs:i * buf_size + ofs + len(f)] = np.frombuffer(f, np.uint8)
        evs[i] = (i, ofs, len(f), poll.EV_SOP, 0, intf, 0)
        if not discard_mix:
            continue
        u = rng.random()
        if u < 0.25:
            evs[i]["discard"] = int(rng.choice([
                poll.DISCARD_L4_CSUM_ERR, poll.DISCARD_L3_CSUM_ERR, poll.DISCARD_L3_CLASS_OTHER,
                poll.DISCARD_L4_CSUM_ERR | poll.DISCARD_ETH_LEN_ERR,
                poll.DISCARD_L3_CSUM_ERR | poll.DISCARD_ETH_FCS_ERR,
                poll.DISCARD_ETH_FCS_ERR, poll.DISCARD_ETH_LEN_ERR, 0x10]))
        elif u < 0.28:
            evs[i]["flags"] = int(rng.choice([poll.EV_SOP | poll.EV_CONT, poll.EV_CONT, 0]))
        elif u < 0.29:
            evs[i]["rq_id"] = n + 5  # outside the pool
    return pool, evs
