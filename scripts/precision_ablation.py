#!/usr/bin/env python
"""Per-stage precision ablation of the fp32-accurate (bf16x3) training mode
(VERDICT r4 item 4): which stages must stay bf16x3 for the weak-loss training
to learn in the offline regime (random-init trunk, known-correspondence
pairs, scripts/train_quality.py), and which can drop to plain bf16.

Each configuration trains the HIP model for --steps from the same init on 4
seeds and reports the mean / per-seed PCK@0.1 before and after; "learns" =
mean PCK gain >= 0.1 with every seed's loss decreasing (the bar of
tests/test_gpu_quality.py::test_training_tracks_fp32_reference).

    python scripts/precision_ablation.py --out profiles/r5/ablation/ablation.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

# (name, --hip-trunk, x3 stages dropped to bf16); the all-bf16 default mode is
# the "bf16" row (nc_precision bf16: no split operands anywhere)
CONFIGS = [
    ("x3_all", "fp32", ""),
    ("bf16_trunk", "bf16", ""),
    ("bf16_corr", "fp32", "corr"),
    ("bf16_nc_in", "fp32", "nc_in"),
    ("bf16_nc_w", "fp32", "nc_w"),
    ("bf16_nc_act", "fp32", "nc_act"),
    ("bf16_nc_grad", "fp32", "nc_grad"),
    ("x3_in_only", "bf16", "nc_w,nc_act,nc_grad"),
    ("bf16", None, ""),
    # combinations: the cheap stages together
    ("bf16_corr_grad", "fp32", "corr,nc_grad"),
    ("bf16_corr_grad_wbwd", "fp32", "corr,nc_grad,nc_w_bwd"),
    ("bf16_corr_grad_act", "fp32", "corr,nc_grad,nc_act"),
    ("bf16_corr_grad_trunk", "bf16", "corr,nc_grad"),
    ("bf16_corr_grad_wbwd_trunk", "bf16", "corr,nc_grad,nc_w_bwd"),
    # the shipped nc_precision='mixed' mode (its own kernels; bf16x3 trunk)
    ("mixed", "mixed", ""),
    # the fp32 trunk's implementation: bf16x3 plan vs MIOpen true fp32
    ("mixed_miopen_trunk", "mixed", "miopen"),
    ("x3_all_x3_trunk", "fp32", "x3"),
]


def main(argv=None):
    import train_quality
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2, 3])
    ap.add_argument("--only", type=str, default="", help="comma list of config names")
    ap.add_argument("--out", type=str, default="")
    a = ap.parse_args(argv)
    only = set(x for x in a.only.split(",") if x)
    rows = []
    for name, trunk, drop in CONFIGS:
        if only and name not in only:
            continue
        runs = []
        for seed in a.seeds:
            t0 = time.time()
            args = ["--steps", str(a.steps), "--batch", "4", "--image-size", "240", "--eval-batches", "4",
                    "--seed", str(seed), "--no-ref"]
            if trunk == "mixed":
                args += ["--nc-precision", "mixed"] + (["--fp32-trunk", drop] if drop else [])
            elif trunk is not None and drop in ("x3", "miopen"):
                args += ["--nc-precision", "fp32", "--hip-trunk", trunk, "--fp32-trunk", drop]
            elif trunk is not None:
                args += ["--nc-precision", "fp32", "--hip-trunk", trunk, "--x3-drop", drop]
            res = train_quality.main(args)
            s = res["summary"]
            runs.append({"seed": seed, "pck_init": res["pck_init_hip"], "pck_final": res["pck_final_hip"],
                         "loss_first": s["loss_first_hip"], "loss_last": s["loss_last_hip"],
                         "seconds": round(time.time() - t0, 1)})
            print(json.dumps({"config": name, **runs[-1]}), flush=True)
        mean = lambda k: sum(r[k] for r in runs) / len(runs)  # noqa: E731
        row = {"config": name, "hip_trunk": trunk, "x3_drop": drop, "pck_init": round(mean("pck_init"), 3),
               "pck_final": round(mean("pck_final"), 3),
               "loss_decreases": all(r["loss_first"] - r["loss_last"] > 0 for r in runs), "runs": runs}
        row["learns"] = row["loss_decreases"] and row["pck_final"] > row["pck_init"] + 0.1
        rows.append(row)
        print(json.dumps({k: v for k, v in row.items() if k != "runs"}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
