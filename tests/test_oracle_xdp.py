# SPDX-License-Identifier: BSD-2-Clause
"""The oracle's AF_XDP ring batch (efxdp_ef_eventq_poll, efxdp_vi.c:309-358,
with netif_event.c:1715-1736) against its plain-descriptor batch on the same
frames: an entry is the frame at UMEM + addr, of length len mod 2^16, on
the ring's interface."""
import numpy as np

from frames import edge_frames, edge_world, install, pack
from onload_amd import _abi
from oracle_lib import OracleStack
from xdp_util import ring_of, to_umem

HWPORTS = (0, 1, 3, 2, 5)


def _stack():
    st = OracleStack(intf_hwport=HWPORTS)
    install(st, edge_world())
    return st


def test_ring_equals_descriptor_batch():
    st = _stack()
    frames = [f for f, _ in edge_frames()]
    umem, ents = to_umem(frames, seed=3)
    for intf in (0, 2):
        for log2, cons in ((12, 0), (12, 4000), (13, (1 << 32) - 37)):
            ring, mask = ring_of(ents, log2, cons, seed=log2)
            got = st.handle_xdp_batch(umem, ring, mask, cons, len(ents), intf)
            buf, desc = pack([(f, intf) for f in frames])
            want = st.handle_rx_batch(buf, desc)
            assert got.tobytes() == want.tobytes(), (intf, log2, cons)


def test_length_is_sixteen_bits_and_outside_is_empty():
    """ef_event's rx.len is 16 bits (ef_vi.h:154): a u32 len of 2^16 + L
    reads L bytes.  An entry past the UMEM end is an empty frame."""
    st = _stack()
    frames = [f for f, _ in edge_frames()][:64]
    umem, ents = to_umem(frames, seed=5)
    ents2 = ents.copy()
    ents2["len"] = ents["len"].astype(np.uint32) + np.uint32(1 << 16)
    ring, mask = ring_of(ents2, 7, 0)
    got = st.handle_xdp_batch(umem, ring, mask, 0, len(ents2), 0)
    ring0, _ = ring_of(ents, 7, 0)
    want = st.handle_xdp_batch(umem, ring0, mask, 0, len(ents), 0)
    assert got.tobytes() == want.tobytes()

    bad = ents[:3].copy()
    bad[0]["addr"] = umem.nbytes                      # starts at the end
    bad[1]["addr"] = umem.nbytes - 10                 # runs past it
    bad[1]["len"] = 60
    bad[2]["addr"] = (1 << 63) + 5                    # far outside
    ring, mask = ring_of(bad, 2, 1)
    got = st.handle_xdp_batch(umem, ring, mask, 1, 3, 0)
    empty = st.handle_rx_batch(np.zeros(64, np.uint8), np.zeros(1, _abi.DESC_DTYPE))[0]
    for r in got:
        assert r.tobytes() == empty.tobytes()
        assert r["reason"] == _abi.R_SHORT_L2
