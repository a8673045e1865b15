# SPDX-License-Identifier: BSD-2-Clause
"""The table half of the oracle and of the product's host mirror, pinned
against the reference's own filter-table code (netif_table.c:323-505,
netif_table_ip6.c:192-345 inserts/removes, :86-143 / :13-66 slot lookups,
:234-319 / :110-189 match walks), through the fixtures that
tests/golden/make_table_golden.py made by running it (oracle/_ref/ref_table):

* every insert/remove return code, -ENOBUFS on a full table included;
* the whole table at each checkpoint -- slot, state, socket id, laddr,
  route count and lport, tombstones and the route counts a failed insert
  leaves behind (netif_table.c:344-376) -- row for row, or by SHA-256 for
  the 2^16-slot tables;
* exact-tuple slot lookups (the reference's wildcard fold, :617-645);
* for the oracle, the demux of a frame per packet-shaped query against the
  reference's per-stage walks (deciding stage, first socket, match count,
  hash3), intf/VLAN bind2dev checks included.
The device side (table kernels + demux walks) is tests/test_gpu_table_ref.py."""
import os

import numpy as np
import pytest

import table_scripts as ts
from frames import pack
from onload_amd.rx import GpuRxStack
from oracle_lib import OracleStack

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                      "ref_table_golden.npz")


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


def _check_script(stack, name, golden, rows_of, frames_check):
    cfg, socks, ops = ts.build(name)

    def at(k, i):
        ts.check_dump(rows_of(stack), golden, name, k)
        looks, matches = ts.queries(name, socks, ts.live_at(ops, i), k)
        got = np.array([ts.folded_lookup(stack, lk) for lk in looks], np.int32)
        want = golden[f"{name}/look{k}"]
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (k, [(looks[j], got[j], want[j]) for j in bad[:3]])
        if frames_check:
            frames_check(stack, matches, golden[f"{name}/match{k}"])

    rcs = ts.replay(stack, socks, ops, at)
    want = golden[f"{name}/rc"]
    np.testing.assert_array_equal(np.array(rcs, np.int32), want)


def _stack_kw(name):
    cfg = ts.build(name)[0]
    return dict(ip4_log2=cfg["log4"], ip6_log2=cfg["log6"], max_socks=cfg["nsocks"],
                intf_hwport=cfg["hwports"])


def oracle_frames_check(stack, matches, m):
    buf, desc = pack([(ts.frame_for(q), q[6]) for q in matches])
    rec = stack.handle_rx_batch(buf, desc, nthreads=4)
    want = ts.expected_records(matches, m)
    for j, (r, w) in enumerate(zip(rec, want)):
        got = (int(r["stage"]), int(r["sock"]), int(r["nmatch"]), int(r["hash3"]))
        assert got == w, (j, matches[j], got, w)


@pytest.mark.parametrize("name", list(ts.SCRIPTS))
def test_oracle_tables_match_reference(golden, name):
    o = OracleStack(**_stack_kw(name))
    _check_script(o, name, golden, lambda s: s.dump(), oracle_frames_check)
    o.close()


@pytest.mark.parametrize("name", list(ts.SCRIPTS))
def test_host_mirror_matches_reference(golden, name):
    g = GpuRxStack(device=-1, **_stack_kw(name))
    _check_script(g, name, golden, lambda s: ts.image_rows(s.image_host()), None)
    g.close()
