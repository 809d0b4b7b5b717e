#!/usr/bin/env python
"""InLoc 3200 px bf16 pair latency with MIOpen's solver search on or off
(torch.backends.cudnn.benchmark): picks the state eval_inloc.py and bench.py's
InLoc secondaries share (eval/inloc.py INLOC_CUDNN_BENCHMARK).

    python scripts/inloc_cudnn_ab.py --benchmark 0|1 [--size 3200]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--benchmark", type=int, default=0)
    ap.add_argument("--size", type=int, default=3200)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    import bench_inloc
    r = bench_inloc.run_single(a.size, pairs=20, warmup=10, panos_per_query=10, precision="bf16")
    print(json.dumps({"cudnn_benchmark": a.benchmark, "size": a.size, "ms_per_pair": r["value"],
                      "stages_ms": r["stages_ms"]}), flush=True)


if __name__ == "__main__":
    main()
