# SPDX-License-Identifier: BSD-2-Clause
"""The reference-run L4 fixtures (tests/golden/ref_l4_golden.npz, made by
tests/golden/make_l4_golden.py from the reference's own netif_event.c,
udp_rx.c, tcp_rx.c and filter tables): the corpora they were run on, and the
comparison of a batch of records against them.

What the reference's run pins, per frame:
  handled   handle_rx_csum_bad's return (netif_event.c:1014-1128): every
            checksum / length gate's drop-or-not decision;
  entry     whether an L4 handler ran, with its l4 offset and ip_paylen
            (handle_rx_pkt :250-451: the IPv4 frag / tot_len / option-walk
            tests pass to the kernel before it);
  stages    per lookup stage ci_{udp,tcp}_handle_rx ran: the real table
            walk's match count and first socket (udp_rx.c:271-306,
            tcp_rx.c:4786-4835), so the deciding stage, socket and nmatch;
            TCP stage 1's hash (rxp.hash);
  kernel    ci_netif_pkt_pass_to_kernel was called (NO_MATCH, IP4_FRAG,
            IP4_OPTS_BAD, TCP_SCATTERED);
  fut       the socket ci_udp_handle_rx_pre_future / ci_tcp_handle_rx_pre_
            future resolve (udp_internal.h:41-103, tcp_rx.h:150-184; IPv4);
  tso       the TCP timestamp-option fast layout (OO_RX_F_TSO):
            ci_tcp_rx_deliver_to_conn's own layout test (tcp_rx.c:4534-4546),
            run on the stage-1 match in a forked child of the harness (1 / 0;
            -1 the child ended before the test; -2 not a TCP stage-1 match);
  obs       which of handle_rx_csum_bad's drop branches a dropped frame took
            (netif_event.c:1024-1127), from what the run shows: the
            address-family branch that ran, which checksum functions ran and
            their verdicts, whether pf.udp.pay_len was written, the protocol
            byte (OBS; ref_drop_reasons);
  stats     every stack counter the frame changed and by how much
            (ip_stats_ops.h:165-291, stats_def.h via CITP_STATS_NETIF_INC):
            the drop counters of handle_rx_csum_bad, handle_rx_pkt's
            in_recvs / in_delivers / in_discards / ip_options, the handlers'
            udp_in_dgrams / tcp_in_segs / no-match counters (expected_stats).
"""
from __future__ import annotations

import hashlib

import numpy as np

from onload_amd import _abi
from onload_amd.rx import htons

COLS = ("handled", "kernel", "entry", "l4off", "ip_paylen", "n1", "f1", "n2", "f2", "n3", "f3",
        "hash", "fut", "tso")
HWPORTS = (0, 1, 3, 2, 5)
CORPORA = ("edge", "edge99", "c2", "c3", "c4", "c5")
CONFIG_SAMPLE = 3000  # frames per configuration sample


def _norm_edge():
    from frames import edge_world
    socks, filters = edge_world()
    fl = [(i, af, bytes(la), htons(lp), None if ra is None else bytes(ra), htons(rp), proto)
          for (i, af, la, lp, ra, rp, proto) in filters]
    return dict(socks), fl


def _norm_pktgen(cfg):
    from onload_amd import pktgen
    filters, socks = pktgen.world(cfg)
    fl = []
    for f in filters:
        n = 4 if f.af == 4 else 16
        fl.append((f.sock, f.af, bytes(f.laddr)[:n], f.lport_be,
                   None if f.raddr_any else bytes(f.raddr)[:n], f.rport_be, f.proto))
    return dict(enumerate(socks)), fl


def corpus(name: str):
    """(socks {id: Sock}, filters [(id, af, laddr, lport_be, raddr|None,
    rport_be, proto)], hwports, frames [(bytes, intf_i)])."""
    if name.startswith("edge"):
        from frames import edge_frames
        socks, filters = _norm_edge()
        return socks, filters, HWPORTS, edge_frames(seed=1234 if name == "edge" else 99)
    cfg = int(name[1:])
    from onload_amd import pktgen
    socks, filters = _norm_pktgen(cfg)
    buf, desc = pktgen.generate(cfg, CONFIG_SAMPLE, first=7000)
    frames = [(buf[int(d["frame_off"]):int(d["frame_off"]) + int(d["len"])].tobytes(),
               int(d["intf_i"])) for d in desc]
    return socks, filters, (0,), frames


def frames_sha(frames) -> str:
    h = hashlib.sha256()
    for f, intf in frames:
        h.update(len(f).to_bytes(4, "little") + intf.to_bytes(2, "little", signed=True) + f)
    return h.hexdigest()


def world_script(socks, filters, hwports):
    """The harness's I / S / A lines for a world."""
    af_of = {f[0]: f[1] for f in filters}
    nsocks = max(list(socks) + [f[0] for f in filters]) + 1
    lines = [f"I 16 14 {max(nsocks, 64)} {len(hwports)} " + " ".join(str(h) for h in hwports)]
    for i, s in sorted(socks.items()):
        af = af_of.get(i, 4)
        ra = (int(s.raddr_be32).to_bytes(4, "little") if af == 4 else bytes(s.raddr6)).hex()
        flags = (1 if s.flags & _abi.SOCK_CONNECTED else 0) | (2 if s.flags & _abi.SOCK_BIND2DEV
                                                                  else 0)
        lines.append(f"S {i} {af} {s.protocol} {s.lport_be16} {s.rport_be16} {ra} {flags} "
                     f"{s.bind2dev_hwports} {s.bind2dev_vlan}")
    for (i, af, la, lp, ra, rp, proto) in filters:
        lines.append(f"A {af} {i} {la.hex()} {lp} {'-' if ra is None else ra.hex()} {rp} {proto}")
    return lines


def load(golden, name):
    return golden[f"{name}/out"], bytes(golden[f"{name}/sha256"]).hex()


OBS = ("eth", "ipcsum", "udp", "udpset", "tcp", "proto")


def load_stats(golden, name):
    """(obs (n, 6), [{counter: delta}] per frame) of a corpus."""
    names = [str(x) for x in golden["stats_names"]]
    st = golden[f"{name}/stats"]
    return golden[f"{name}/obs"], [{k: int(v) for k, v in zip(names, row) if v} for row in st]


def ref_drop_reasons(o, st) -> set:
    """The drop reasons handle_rx_csum_bad's observed run allows
    (netif_event.c:1024-1127): its branches by the counter they bump
    (in_hdr_errs :1031/:1048/:1055, in6_hdr_errs :1069, udp_in_errs :1116),
    the address-family branch that ran (it writes CI_PKT_FLAG_IS_IP6 first,
    :1043/:1063), whether ci_ip_csum_partial ran (:1053), the checksum
    functions' verdicts (:1091, :1109), whether pf.udp.pay_len was written
    (:1105) and the protocol byte.  TCP's two gates before its checksum
    function (ip_paylen < 20, :1087; doff < 5 or hlen > ip_paylen inside
    ci_tcp_csum_correct, :107-110) leave the same trace: that pair is
    allowed either way."""
    o = dict(zip(OBS, (int(x) for x in o)))
    if st.get("ip.in_hdr_errs"):
        if o["eth"] == 0:
            return {_abi.R_SHORT_L2}
        return {_abi.R_IP4_CSUM} if o["ipcsum"] else {_abi.R_IP4_LEN}
    if st.get("ip.in6_hdr_errs"):
        return {_abi.R_IP6_LEN}
    if st.get("udp.udp_in_errs") or o["udp"] == 0:
        return {_abi.R_UDP_CSUM}
    if o["eth"] == 0:
        return {_abi.R_NOT_IP}
    if o["udpset"] and o["udp"] == -1:
        return {_abi.R_UDP_SHORT}
    if o["tcp"] == 0:
        return {_abi.R_TCP_CSUM}
    if o["proto"] == 6:
        return {_abi.R_TCP_SHORT, _abi.R_TCP_CSUM}
    if o["proto"] not in (6, 17):
        return {_abi.R_PROTO_OTHER}
    return set()


def expected_stats(r) -> dict:
    """The stack counters the reference's per-event path changes for a frame
    whose record is r: handle_rx_csum_bad's drop counters, then for a handled
    frame handle_rx_pkt (netif_event.c:282-373 / :384-404: in_recvs, the
    option parse's ip_options or rx_discard_ip_options_bad + in_hdr_errs
    :179-183, in_discards + the pass to the kernel for the slow path,
    in_delivers) and the handler (udp_rx.c:263 udp_in_dgrams, :322-327
    no-match to the kernel; tcp_rx.c:4692 tcp_in_segs, :4842-4857 no match
    or scattered to the kernel).  The poll shim keeps the ones it replaces
    (INTEGRATION.md §2); tests pin this against the reference's run."""
    reason = int(r["reason"])
    d = {}
    if reason >= _abi.R_DROP_BASE:
        if reason in (_abi.R_SHORT_L2, _abi.R_IP4_LEN, _abi.R_IP4_CSUM):
            d["ip.in_hdr_errs"] = 1
        elif reason == _abi.R_IP6_LEN:
            d["ip.in6_hdr_errs"] = 1
        elif reason == _abi.R_UDP_CSUM:
            d["udp.udp_in_errs"] = 1
        return d
    is6 = bool(int(r["flags"]) & _abi.F_IP6)
    d["ip.in6_recvs" if is6 else "ip.in_recvs"] = 1
    if reason in (_abi.R_IP4_FRAG, _abi.R_IP4_OPTS_BAD):
        d["ip.in_discards"] = 1
        d["ni.no_match_pass_to_kernel_ip_other"] = 1
        if reason == _abi.R_IP4_OPTS_BAD:
            d["ip.in_hdr_errs"] = 1
            d["ni.rx_discard_ip_options_bad"] = 1
        return d
    d["ip.in6_delivers" if is6 else "ip.in_delivers"] = 1
    pre_l3 = 18 if int(r["flags"]) & _abi.F_VLAN else 14
    if not is6 and int(r["l4_off"]) > pre_l3 + 20:
        d["ni.ip_options"] = 1
    if int(r["proto"]) == 17:
        d["udp.udp_in_dgrams"] = 1
        if reason == _abi.R_NO_MATCH:
            d["ni.no_match_pass_to_kernel_udp"] = 1
    else:
        d["tcp.tcp_in_segs"] = 1
        if reason in (_abi.R_NO_MATCH, _abi.R_TCP_SCATTERED):
            d["ni.no_match_pass_to_kernel_tcp"] = 1
    return d


def stats_mismatches(recs, obs, stats, limit: int = 8) -> list[str]:
    """Where the records' drop reasons or counter changes disagree with the
    reference's run (empty: none)."""
    bad = []
    for i, (r, o, st) in enumerate(zip(recs, obs, stats)):
        err = []
        reason = int(r["reason"])
        if reason >= _abi.R_DROP_BASE and reason not in ref_drop_reasons(o, st):
            err.append(f"drop reason {reason} not in {sorted(ref_drop_reasons(o, st))}")
        want = expected_stats(r)
        if want != st:
            err.append(f"stats {want} != reference {st}")
        if err:
            bad.append(f"[{i}] {', '.join(err)}: rec={r} obs={dict(zip(OBS, o.tolist()))}")
            if len(bad) >= limit:
                break
    return bad


KERNEL = (_abi.R_NO_MATCH, _abi.R_IP4_FRAG, _abi.R_IP4_OPTS_BAD, _abi.R_TCP_SCATTERED)


def mismatches(recs: np.ndarray, out: np.ndarray, limit: int = 8) -> list[str]:
    """Where the records disagree with the reference's run (empty: none)."""
    bad = []
    for i, (r, row) in enumerate(zip(recs, out)):
        g = dict(zip(COLS, (int(x) for x in row)))
        reason = int(r["reason"])
        err = []
        if bool(g["handled"]) != (reason < _abi.R_DROP_BASE):
            err.append("handled")
        elif g["handled"]:
            if bool(g["kernel"]) != (reason in KERNEL):
                err.append("kernel")
            if g["entry"] == 0:
                if reason not in (_abi.R_IP4_FRAG, _abi.R_IP4_OPTS_BAD):
                    err.append("no L4 entry")
            else:
                if (g["entry"], g["l4off"], g["ip_paylen"] & 0xffff) != (
                        int(r["proto"]), int(r["l4_off"]), int(r["ip_paylen"])):
                    err.append("entry")
                ran = [(g[f"n{k}"], g[f"f{k}"]) for k in (1, 2, 3) if g[f"n{k}"] >= 0]
                dec = next((k for k, (n, _) in enumerate(ran) if n > 0), None)
                tcp = g["entry"] == 6
                if dec is None:
                    want = _abi.R_TCP_SCATTERED if (tcp and not ran) else _abi.R_NO_MATCH
                    if reason != want:
                        err.append(f"reason {reason} want {want}")
                else:
                    n, first = ran[dec]
                    if (reason, int(r["stage"]), int(r["sock"]), int(r["nmatch"])) != (
                            _abi.R_DELIVER, dec + 1, first, 1 if tcp else n):
                        err.append(f"deliver want stage {dec + 1} sock {first} n {n}")
                if tcp and ran and int(r["hash3"]) != g["hash"]:
                    err.append("hash3")
                if g["fut"] != -2:  # IPv4: the pre-future ran
                    if tcp:
                        fut = (reason == _abi.R_DELIVER and int(r["stage"]) == 1)
                    else:
                        fut = (reason == _abi.R_DELIVER and int(r["nmatch"]) == 1 and
                               not r["flags"] & _abi.F_UDP_S2)
                    if fut != (g["fut"] >= 0) or (fut and g["fut"] != int(r["sock"])):
                        err.append(f"future want {g['fut']}")
                if g["tso"] == -1:
                    err.append("tso probe ended before the layout test")
                elif g["tso"] >= 0 and bool(int(r["flags"]) & _abi.F_TSO) != bool(g["tso"]):
                    err.append(f"tso want {g['tso']}")
        if err:
            bad.append(f"[{i}] {', '.join(err)}: rec={r} ref={g}")
            if len(bad) >= limit:
                break
    return bad
