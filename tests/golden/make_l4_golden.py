# SPDX-License-Identifier: BSD-2-Clause
"""Generates tests/golden/ref_l4_golden.npz from the reference's own receive
path: oracle/_ref/ref_l4 (oracle/ref_l4_harness.c) runs handle_rx_csum_bad ->
handle_rx_pkt -> ci_{udp,tcp}_handle_rx -> ci_netif_filter_for_each_match
and the UDP / TCP pre-future lookups, all compiled unmodified from
/root/reference by oracle/Makefile (this container only).

For each corpus (a socket world + frames from this repo's generators) it
stores what the reference answered for every frame:

  <corpus>/out     int64 (n, 14): handled, kernel, entry (0 / 6 / 17), l4off,
                   ip_paylen, n1, first1, n2, first2, n3, first3, hash (TCP
                   stage 1), fut (pre-future socket; -1 none, -2 not run),
                   tso (the timestamp-option fast layout test of
                   ci_tcp_rx_deliver_to_conn on the stage-1 match: 1 / 0,
                   -1 not reached, -2 not probed)
                   -- columns as tests/l4_ref.py names them
  <corpus>/obs     int64 (n, 6): what tells handle_rx_csum_bad's drop
                   branches apart -- eth, ipcsum, udp, udpset, tcp, proto
                   (tests/l4_ref.py OBS; oracle/ref_l4_harness.c)
  <corpus>/stats   int64 (n, K): each stack counter's change over the frame
                   (columns: stats_names)
  <corpus>/sha256  SHA-256 of the frames (the test regenerates them and
                   checks this first: the fixture holds no frame bytes)
  stats_names      the K counter names ("ip.in_recvs", "ni.ip_options", ...)

Run: python tests/golden/make_l4_golden.py   (after `make -C oracle`)."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import l4_ref  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_l4")


def run(corpus: str):
    socks, filters, hwports, frames = l4_ref.corpus(corpus)
    lines = l4_ref.world_script(socks, filters, hwports)
    for f, intf in frames:
        lines.append(f"P {intf} {f.hex()}")
    p = subprocess.run([HARNESS], input="\n".join(lines) + "\n", capture_output=True,
                       text=True, check=True)
    out = p.stdout.splitlines()
    nset = len(lines) - len(frames)
    assert len(out) == len(lines), (len(out), len(lines), p.stderr[-500:])
    assert all(x in ("ok", "0") for x in out[:nset]), [x for x in out[:nset] if x not in ("ok", "0")]
    assert all(x.startswith("r ") for x in out[nset:])
    rows, obs, stats = [], [], []
    for x in out[nset:]:
        a, b, c = x.split("|")
        rows.append(list(map(int, a.split()[1:])))
        obs.append(list(map(int, b.split())))
        stats.append({k: int(v) for k, v in (t.split("=") for t in c.split())})
    return (np.array(rows, dtype=np.int64), np.array(obs, dtype=np.int64), stats,
            l4_ref.frames_sha(frames))


def main() -> None:
    res, runs = {}, {}
    for name in l4_ref.CORPORA:
        runs[name] = run(name)
    names = sorted({k for r in runs.values() for d in r[2] for k in d})
    res["stats_names"] = np.array(names)
    for name, (out, obs, stats, sha) in runs.items():
        res[f"{name}/out"] = out
        res[f"{name}/obs"] = obs
        res[f"{name}/stats"] = np.array([[d.get(k, 0) for k in names] for d in stats],
                                        dtype=np.int64).reshape(len(stats), len(names))
        res[f"{name}/sha256"] = np.frombuffer(bytes.fromhex(sha), np.uint8)
        handled = out[:, 0].sum()
        print(f"{name}: {len(out)} frames, {handled} handled, "
              f"{(out[:, 2] != 0).sum()} reached an L4 handler, {(out[:, 12] >= 0).sum()} futures")
    np.savez_compressed(os.path.join(HERE, "ref_l4_golden.npz"), **res)


if __name__ == "__main__":
    main()
