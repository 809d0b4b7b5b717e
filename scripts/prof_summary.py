#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace of ``bench.py`` over the timed steps only.

The first W warmup steps include MIOpen solver search, so dispatches are kept
from the start of step W (located by the per-step count of a marker kernel).

    python scripts/prof_summary.py gpurun_out/prof/hip_kernel_trace.csv --warmup 3 --steps 5 [--out profiles/x.md]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--marker", default="l2norm_rows_kernel")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    per_step = len(marks) // (a.warmup + a.steps)
    first = marks[a.warmup * per_step] if per_step else 0
    # the window ends at the marker of the first step after the timed ones (when
    # the traced program runs more after them, e.g. bench_inloc's eager breakdown)
    end = marks[(a.warmup + a.steps) * per_step] if per_step and len(marks) > (a.warmup + a.steps) * per_step else None
    sel = rows[first:end]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        name = r["Kernel_Name"]
        for pre in ("void ", "ncnet::"):
            name = name.replace(pre, "")
        name = name.split("(")[0][:90]
        agg[name][0] += d
        agg[name][1] += 1
    busy = sum(v[0] for v in agg.values())
    lines = [f"timed window: {(t1 - t0) / 1e6 / a.steps:.3f} ms/step wall, kernel-busy {busy / 1e6 / a.steps:.3f} ms/step",
             "", "| ms/step | % busy | calls/step | kernel |", "|---:|---:|---:|---|"]
    for name, (d, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
        lines.append(f"| {d / 1e6 / a.steps:.3f} | {100.0 * d / busy:.1f} | {c / a.steps:.1f} | `{name}` |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
