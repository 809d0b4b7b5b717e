#!/usr/bin/env python
"""Measure the fused training path's gradient error against the quantized
fp64 oracle (engine/quantized_oracle.py training_grad_errors) over several
operating-point seeds, each run twice in one process: the spread across seeds
sets test_gpu_quality's bounds, the repeat shows whether one build is
run-to-run deterministic at a fixed point.

    python scripts/oracle_tolerance.py [--seeds 0 10 20 30] [--repeats 2] [--out F.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 10, 20, 30])
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--out", default="")
    args = ap.parse_args(argv)
    from ncnet_amd import config as _config
    from ncnet_amd.engine.quantized_oracle import training_grad_errors
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    rows = []
    with _config.override(trunk_conv="native"):
        for fe in (0, 1):
            for s in args.seeds:
                for r in range(args.repeats):
                    e = training_grad_errors(fe_finetune=fe, point_seed=s)
                    rows.append({"fe_finetune": fe, "point_seed": s, "repeat": r, **e})
                    print(json.dumps(rows[-1]), flush=True)
    summary = {}
    for fe in (0, 1):
        sel = [x for x in rows if x["fe_finetune"] == fe]
        keys = [k for k in sel[0] if k not in ("fe_finetune", "point_seed", "repeat")]
        nc = [max(v for k, v in x.items() if k.startswith("layer")) for x in sel]
        spread = 0.0
        for s in args.seeds:
            rs = [x for x in sel if x["point_seed"] == s]
            for k in keys:
                spread = max(spread, max(x[k] for x in rs) - min(x[k] for x in rs))
        summary[f"fe{fe}"] = {"max_layer": max(nc), "layer_by_point": nc, "max_vols": max(x["vols"] for x in sel),
                              "max_d_raw": max((x.get("d_raw_features", 0.0) for x in sel)),
                              "max_repeat_spread": spread}
    print(json.dumps({"summary": summary}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"rows": rows, "summary": summary}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
