#!/usr/bin/env python
"""One training step of a rocprofv3 kernel trace as a timeline: every kernel
of the step in start order with its offset, duration and stream, so the
critical path of the pipelined step (main stream, weight-gradient side stream,
trunk prefetch stream) can be read off.

A step is the window between two consecutive dispatches of ``--marker``
(default: the correlation GEMM, once per step on the main stream).

    python scripts/prof_timeline.py gpurun_out/prof/run_kernel_trace.csv --step 4 [--out profiles/x.md]
"""
import argparse
import csv


def short(name: str) -> str:
    for pre in ("void ", "ncnet::", "at::native::"):
        name = name.replace(pre, "")
    return name.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=4, help="which marker interval (0-based)")
    ap.add_argument("--marker", default="corr_gemm_kernel")
    ap.add_argument("--min-us", type=float, default=0.0, help="hide kernels shorter than this")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
    t0, t1 = marks[a.step], marks[a.step + 1]
    qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    sel = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
    queues = {}
    for r in sel:
        queues.setdefault(r[qkey], len(queues))
    lines = [f"step {a.step}: {(t1 - t0) / 1e3:.1f} us between `{a.marker}` dispatches; "
             f"{len(sel)} kernels on {len(queues)} streams ({qkey})", "",
             "| start us | dur us | end us | stream | kernel |", "|---:|---:|---:|---:|---|"]
    busy = {}
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = queues[r[qkey]]
        busy[q] = busy.get(q, 0) + (e - s)
        if (e - s) / 1e3 < a.min_us:
            continue
        lines.append(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {(e - t0) / 1e3:.1f} | {q} | `{short(r['Kernel_Name'])}` |")
    lines.append("")
    lines.append("busy per stream (us): " + ", ".join(f"{q}: {v / 1e3:.0f}" for q, v in sorted(busy.items())))
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
