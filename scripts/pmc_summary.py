#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc CSVs per kernel (mean over dispatches) into a table.

    python scripts/pmc_summary.py gpurun_out/pmc_1 gpurun_out/pmc_2 [--out profiles/x.md]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ncnet::", "")[:60]
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    lines = []
    for k, cs in vals.items():
        lines.append(f"### `{k}`")
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(m):
            lines.append(f"- {c}: {m[c]:.4g}")
        busy = m.get("GRBM_GUI_ACTIVE")
        if "SQ_LDS_IDX_ACTIVE" in m and "SQ_BUSY_CYCLES" in m:
            lines.append(f"- LDS_IDX_ACTIVE / SQ_BUSY_CYCLES: {m['SQ_LDS_IDX_ACTIVE'] / max(m['SQ_BUSY_CYCLES'], 1):.3f}")
        if "SQ_WAVE_CYCLES" in m:
            w = m["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    lines.append(f"- {c} / WAVE_CYCLES: {m[c] / w:.3f}")
        if busy and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            lines.append(f"- MFMA_BUSY / GRBM_GUI_ACTIVE: {m['SQ_VALU_MFMA_BUSY_CYCLES'] / busy:.4g}")
        lines.append("")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
