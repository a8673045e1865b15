# SPDX-License-Identifier: BSD-2-Clause
"""A transport for oo_gpu_rx_group_join_transport whose ranks are threads of
this process (test infrastructure): every collective is a rendezvous of all
ranks on a barrier, moving host memory with ctypes.memmove.  Failures are
injected per rank and per call: the rank still takes part in the rendezvous
(as a real rank whose local copy failed would still have entered the
collective) but its call returns -EIO and, for a broadcast, leaves its buffer
as it was.  A rank that never enters a collective the others entered shows
up as a barrier timeout, reported as -ETIMEDOUT by the others (a hang, in a
real communicator)."""
from __future__ import annotations

import ctypes
import errno
import threading

from onload_amd.group import BCAST, GATHER, REDUCE, Transport

TIMEOUT_S = 10.0


class ThreadXport:
    def __init__(self, nranks: int):
        self.n = nranks
        self.bar = threading.Barrier(nranks, timeout=TIMEOUT_S)
        self.slot = [None] * nranks
        self.fail = {}  # (rank, kind, index) -> True: that call returns -EIO
        self.count = [dict() for _ in range(nranks)]  # rank -> kind -> calls so far
        self.timeouts = 0
        self.calls = [[] for _ in range(nranks)]

    def _next(self, rank, kind):
        k = self.count[rank].get(kind, 0)
        self.count[rank][kind] = k + 1
        self.calls[rank].append(kind)
        return self.fail.get((rank, kind, k), False)

    def _wait(self):
        try:
            self.bar.wait()
            return True
        except threading.BrokenBarrierError:
            self.timeouts += 1
            return False

    def transport(self, rank: int) -> Transport:
        def bcast(arg, p, nbytes):
            bad = self._next(rank, "bcast")
            self.slot[rank] = (p, nbytes)
            if not self._wait():
                return -errno.ETIMEDOUT
            src, sb = self.slot[0]
            if rank != 0 and not bad:
                ctypes.memmove(p, src, min(nbytes, sb))
            if not self._wait():
                return -errno.ETIMEDOUT
            return -errno.EIO if bad or sb != nbytes else 0

        def reduce(op, kind):
            def f(arg, v, n):
                bad = self._next(rank, kind)
                self.slot[rank] = [int(v[i]) for i in range(n)]
                if not self._wait():
                    return -errno.ETIMEDOUT
                res = [op(self.slot[r][i] for r in range(self.n)) & 0xFFFFFFFF for i in range(n)]
                if not self._wait():
                    return -errno.ETIMEDOUT
                if bad:
                    return -errno.EIO
                for i in range(n):
                    v[i] = res[i]
                return 0
            return f

        def gather(arg, src, nbytes, dst, bytes_of):
            bad = self._next(rank, "gather")
            self.slot[rank] = (src, nbytes)
            if not self._wait():
                return -errno.ETIMEDOUT
            if rank == 0:
                at = 0
                for r in range(self.n):
                    want = int(bytes_of[r])
                    s, sb = self.slot[r]
                    if sb != want:
                        bad = True
                    elif want:
                        ctypes.memmove(dst + at, s, want)
                    at += want
            if not self._wait():
                return -errno.ETIMEDOUT
            return -errno.EIO if bad else 0

        return Transport(None, BCAST(bcast), REDUCE(reduce(max, "max")),
                         REDUCE(reduce(sum, "sum")), GATHER(gather))


def run_ranks(fn, nranks: int, timeout: float = 3 * TIMEOUT_S):
    """fn(rank) on one thread per rank; their results (an exception is a
    result).  A thread still running after `timeout` is a hang: AssertionError."""
    out = [None] * nranks

    def body(r):
        try:
            out[r] = fn(r)
        except Exception as e:  # noqa: BLE001 - reported as the rank's result
            out[r] = e

    ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(nranks)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), "a rank hung in a collective"
    return out
