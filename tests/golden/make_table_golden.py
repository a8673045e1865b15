# SPDX-License-Identifier: BSD-2-Clause
"""Generates tests/golden/ref_table_golden.npz from the reference's own
filter-table code (netif_table.c + netif_table_ip6.c compiled unmodified into
oracle/_ref/ref_table by oracle/Makefile; this container only).

For each script of tests/table_scripts.py it feeds the reference the socket
fields, the insert/remove sequence and, at each checkpoint, a table dump, the
exact-tuple slot lookups and the per-stage match walks of the checkpoint's
packet-shaped queries, and stores what the reference answered:

  <name>/rc          int32 per insert/remove (0, -ENOBUFS, ...)
  <name>/dumpK       sparse dump rows (af, slot, a, b, c, d) for the small
                     tables, or <name>/digestK (SHA-256 of the rows) for
                     the 2^16-slot ones
  <name>/lookK       int32 per slot lookup
  <name>/matchK      (n, first, hash) per query and stage (-1 rows where a
                     query has no third stage)

Run: python tests/golden/make_table_golden.py   (after `make -C oracle`)."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import table_scripts as ts  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_table")
ROWS_LIMIT = 20000  # dumps larger than this are stored as a digest


def script_text(name):
    cfg, socks, ops = ts.build(name)
    lines = [f"I {cfg['log4']} {cfg['log6']} {cfg['nsocks']} {len(cfg['hwports'])} "
             + " ".join(str(h) for h in cfg["hwports"])]
    for s in socks:
        flags = (1 if s.connected else 0) | (2 if s.b2d else 0)
        lines.append(f"S {s.id} {s.af} {s.proto} {s.lport} {s.rport} {s.raddr.hex()} {flags} "
                     f"{s.hwports} {s.vlan}")
    plan = []  # ("rc",) per op, ("C", k, nlook, nmatch) per checkpoint
    for i, o in enumerate(ops):
        if o[0] in "AR":
            kind, af, sid, la, lp, ra, rp, proto = o
            lines.append(f"{kind} {af} {sid} {la.hex()} {lp} {ts.hexs(ra)} {rp} {proto}")
            plan.append(("rc",))
        else:
            k = o[1]
            looks, matches = ts.queries(name, socks, ts.live_at(ops, i), k)
            lines.append("D")
            for (af, la, lp, ra, rp, proto) in looks:
                lines.append(f"L {af} {la.hex()} {lp} {ts.hexs(ra)} {rp} {proto}")
            for q in matches:
                for (la, lp, ra, rp) in ts.match_stages(q):
                    lines.append(f"M {q[0]} {la.hex()} {lp} {ts.hexs(ra)} {rp} {q[1]} {q[6]} {q[7]}")
            plan.append(("C", k, len(looks), matches))
    return lines, plan


def run(name):
    lines, plan = script_text(name)
    p = subprocess.run([HARNESS], input="\n".join(lines) + "\n", capture_output=True,
                       text=True, check=True)
    out = p.stdout.splitlines()
    pos = 1 + ts.SCRIPTS[name][3]  # init + socket lines answer "ok"
    assert all(x == "ok" for x in out[:pos]), out[:pos]
    res = {}
    rc = []
    for item in plan:
        if item[0] == "rc":
            rc.append(int(out[pos]))
            pos += 1
            continue
        _, k, nlook, matches = item
        rows = []
        while out[pos] != "end":
            f = out[pos].split()
            if f[0] == "d4":
                rows.append((4, int(f[1]), int(f[2]), int(f[3]), int(f[4]), int(f[5])))
            else:
                la = bytes.fromhex(f[4])
                rows.append((6, int(f[1]), int(f[2]), int(f[3]),
                             int.from_bytes(la[:8], "little", signed=True),
                             int.from_bytes(la[8:], "little", signed=True)))
            pos += 1
        pos += 1
        rows = np.array(rows, dtype=np.int64).reshape(-1, 6)
        if len(rows) > ROWS_LIMIT:
            res[f"{name}/digest{k}"] = np.frombuffer(
                ts.dump_digest(rows[rows[:, 0] == 4], rows[rows[:, 0] == 6]).encode(), np.uint8)
        else:
            res[f"{name}/dump{k}"] = rows
        res[f"{name}/look{k}"] = np.array([int(x) for x in out[pos:pos + nlook]], np.int32)
        pos += nlook
        m = np.full((len(matches), 3, 3), -1, dtype=np.int64)
        for j, q in enumerate(matches):
            for st in range(len(ts.match_stages(q))):
                n, first, h = out[pos].split()
                m[j, st] = (int(n), int(first), int(h))
                pos += 1
        res[f"{name}/match{k}"] = m
    assert pos == len(out)
    res[f"{name}/rc"] = np.array(rc, np.int32)
    return res


def main():
    if not os.path.exists(HARNESS):
        sys.exit(f"{HARNESS} missing: run `make -C oracle` where /root/reference exists")
    res = {}
    for name in ts.SCRIPTS:
        r = run(name)
        res.update(r)
        rcs = r[f"{name}/rc"]
        print(name, "ops", len(rcs), "ENOBUFS", int((rcs == -105).sum()),
              "checkpoints", sum(1 for k in r if "/look" in k))
    np.savez_compressed(os.path.join(HERE, "ref_table_golden.npz"), **res)


if __name__ == "__main__":
    main()
