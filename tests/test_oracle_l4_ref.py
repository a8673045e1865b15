# SPDX-License-Identifier: BSD-2-Clause
"""The oracle against the reference's own receive path (tests/l4_ref.py,
tests/golden/ref_l4_golden.npz): for every frame of the edge corpora and of
configuration samples 2-5, the gates, the L4 entry, each lookup stage's
matches and socket, the pass-to-kernel decisions and the UDP / TCP future
sockets the reference computed -- handle_rx_csum_bad, handle_rx_pkt,
ci_udp_handle_rx, ci_tcp_handle_rx, ci_netif_filter_for_each_match and the
pre-future helpers, compiled unmodified (oracle/ref_l4_harness.c).  When the
harness binary is present (this container) the fixtures are also re-derived
live."""
import os
import subprocess

import numpy as np
import pytest

import l4_ref
from frames import pack
from onload_amd import _abi
from oracle_lib import OracleStack

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "ref_l4_golden.npz")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_l4")


def oracle_records(name):
    socks, filters, hwports, frames = l4_ref.corpus(name)
    o = OracleStack(intf_hwport=hwports)
    for i, s in socks.items():
        assert o.sock_set(i, s) == 0
    for (i, af, la, lp, ra, rp, proto) in filters:
        assert o.filter_insert_raw(i, af, la, lp, ra, rp, proto) == 0
    buf, desc = pack(frames)
    return o.handle_rx_batch(buf, desc, nthreads=4), frames


@pytest.mark.parametrize("name", l4_ref.CORPORA)
def test_oracle_matches_reference_run(name):
    golden = np.load(GOLDEN)
    out, sha = l4_ref.load(golden, name)
    recs, frames = oracle_records(name)
    assert l4_ref.frames_sha(frames) == sha, "the generator no longer makes the fixture's frames"
    assert len(recs) == len(out)
    bad = l4_ref.mismatches(recs, out)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("name", l4_ref.CORPORA)
def test_oracle_drop_reasons_and_counters_match_reference_run(name):
    """Every dropped frame's reason is the branch handle_rx_csum_bad took
    (TCP's two pre-checksum gates: either of their two reasons), and every
    frame changes exactly the stack counters the reference's run changed."""
    golden = np.load(GOLDEN)
    obs, stats = l4_ref.load_stats(golden, name)
    recs, _ = oracle_records(name)
    bad = l4_ref.stats_mismatches(recs, obs, stats)
    assert not bad, "\n".join(bad)


def test_fixture_covers_every_drop_branch():
    """The corpora reach all ten drop branches, told apart by the reference's
    own run, and every counter the rules name."""
    golden = np.load(GOLDEN)
    seen, names = set(), set()
    for n in l4_ref.CORPORA:
        out, _ = l4_ref.load(golden, n)
        obs, stats = l4_ref.load_stats(golden, n)
        for row, o, st in zip(out, obs, stats):
            names |= set(st)
            if row[0] == 0:
                rs = l4_ref.ref_drop_reasons(o, st)
                assert rs, (o, st)
                seen |= rs
    assert seen == set(range(_abi.R_DROP_BASE, _abi.R_UDP_CSUM + 1))
    assert {"ip.in_hdr_errs", "ip.in6_hdr_errs", "udp.udp_in_errs", "ip.in_recvs",
            "ip.in_delivers", "ip.in6_recvs", "ip.in6_delivers", "ip.in_discards",
            "ni.ip_options", "ni.rx_discard_ip_options_bad", "udp.udp_in_dgrams",
            "tcp.tcp_in_segs", "ni.no_match_pass_to_kernel_udp",
            "ni.no_match_pass_to_kernel_tcp", "ni.no_match_pass_to_kernel_ip_other"} <= names


def test_fixture_covers_the_rules():
    """The corpora reach every decision the fixture pins: all three TCP
    stages, both UDP stages with multi-match, the UDP future given up by a
    stage-2 match after a single stage-1 one, kernel hand-offs with and
    without an L4 entry, the TCP timestamp-option layout test both ways
    (every probe reached it)."""
    golden = np.load(GOLDEN)
    out = np.concatenate([l4_ref.load(golden, n)[0] for n in l4_ref.CORPORA])
    c = {k: out[:, i] for i, k in enumerate(l4_ref.COLS)}
    tcp, udp = c["entry"] == 6, c["entry"] == 17
    assert ((c["n1"] > 0) & tcp).any() and ((c["n2"] > 0) & tcp).any() and \
        ((c["n3"] > 0) & tcp).any()
    assert ((c["n1"] > 0) & udp).any() and ((c["n2"] > 1) & udp).any()
    assert ((c["n1"] == 1) & udp & (c["fut"] == -1)).any()   # given up: stage 2 matched too
    assert ((c["n1"] == 1) & udp & (c["fut"] >= 0)).any()
    assert ((c["kernel"] == 1) & (c["entry"] == 0)).any()
    assert ((c["kernel"] == 1) & tcp & (c["n1"] < 0)).any()   # TCP scattered
    assert ((c["tso"] == 1) & tcp).any() and ((c["tso"] == 0) & tcp).any()
    assert not (c["tso"] == -1).any() and not ((c["tso"] >= 0) & ~tcp).any()


@pytest.mark.skipif(not os.path.exists(HARNESS), reason="oracle/_ref/ref_l4 is built only "
                    "where /root/reference is (this container)")
@pytest.mark.parametrize("name", ("edge", "c5"))
def test_fixture_rederived_live(name):
    socks, filters, hwports, frames = l4_ref.corpus(name)
    lines = l4_ref.world_script(socks, filters, hwports) + \
        [f"P {intf} {f.hex()}" for f, intf in frames]
    p = subprocess.run([HARNESS], input="\n".join(lines) + "\n", capture_output=True, text=True,
                       check=True)
    lines = [x for x in p.stdout.splitlines() if x.startswith("r ")]
    golden = np.load(GOLDEN)
    rows = np.array([list(map(int, x.split("|")[0].split()[1:])) for x in lines], dtype=np.int64)
    obs = np.array([list(map(int, x.split("|")[1].split())) for x in lines], dtype=np.int64)
    stats = [{k: int(v) for k, v in (t.split("=") for t in x.split("|")[2].split())}
             for x in lines]
    np.testing.assert_array_equal(rows, l4_ref.load(golden, name)[0])
    gobs, gstats = l4_ref.load_stats(golden, name)
    np.testing.assert_array_equal(obs, gobs)
    assert stats == gstats
