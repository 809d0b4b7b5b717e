#!/usr/bin/env python
"""Per-step kernel summary from a rocprofv3 SQLite database (rocpd schema,
the default ``--kernel-trace`` output of ROCm 7).

Steps are delimited by a marker kernel that runs once per training step (the
L2-norm packing of the prefetched batch by default).  Over the steps in
[--first, --last) it prints the wall time per step, the GPU-busy time (union of
kernel intervals over all streams), the idle gap, and the per-kernel totals.

    python scripts/prof_db_summary.py gpurun_out/prof/run_results.db --first 20 --last 100
"""
import argparse
import sqlite3
from collections import defaultdict


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="l2norm_rows_kernel")
    ap.add_argument("--first", type=int, default=20)
    ap.add_argument("--last", type=int, default=100)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    marks = [r[1] for r in rows if a.marker in r[0]]
    if len(marks) < a.last + 1:
        a.last = len(marks) - 1
    t0, t1 = marks[a.first], marks[a.last]
    nsteps = a.last - a.first
    win = [r for r in rows if r[1] >= t0 and r[2] <= t1]
    busy, cur_s, cur_e = 0, None, None
    for _, s, e, _ in sorted(win, key=lambda r: r[1]):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    per = defaultdict(lambda: [0, 0])
    for n, s, e, _ in win:
        per[n][0] += e - s
        per[n][1] += 1
    wall = (t1 - t0) / nsteps / 1e6
    lines = [f"steps {a.first}..{a.last} (marker {a.marker}): wall {wall:.3f} ms/step, "
             f"GPU busy (union over streams) {busy / nsteps / 1e6:.3f} ms/step, "
             f"idle {wall - busy / nsteps / 1e6:.3f} ms/step", "",
             "| ms/step | calls/step | kernel |", "|---:|---:|---|"]
    for n, (d, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:a.top]:
        lines.append(f"| {d / nsteps / 1e6:.3f} | {c / nsteps:.1f} | `{n[:90]}` |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
