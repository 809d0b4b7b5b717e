#!/usr/bin/env python
"""bench.py's headline step at a given batch, then the caching allocator's
counters (alloc retries, cudaMalloc / cudaFree calls, reserved vs allocated
peak): tells allocator churn apart from kernel time at large batches.

    python scripts/alloc_probe.py --batch 512 --steps 4 --warmup 3
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch

    import bench
    argv = sys.argv[1:] + ["--inloc", "0"]
    rc = bench.main(argv)
    st = torch.cuda.memory_stats()
    keys = ("num_alloc_retries", "num_ooms", "num_device_alloc", "num_device_free",
            "reserved_bytes.all.peak", "allocated_bytes.all.peak", "reserved_bytes.all.current")
    print(json.dumps({"alloc_conf": os.environ.get("PYTORCH_HIP_ALLOC_CONF", os.environ.get("PYTORCH_CUDA_ALLOC_CONF")),
                      **{k: st.get(k) for k in keys}}), flush=True)
    # reserved segments by (stream, graph pool): where the cache sits
    by = {}
    for seg in torch.cuda.memory_snapshot():
        k = (str(seg.get("stream")), str(seg.get("segment_pool_id")))
        e = by.setdefault(k, {"segments": 0, "reserved_gb": 0.0, "active_gb": 0.0, "largest_gb": 0.0})
        e["segments"] += 1
        e["reserved_gb"] += seg["total_size"] / 2 ** 30
        e["active_gb"] += seg.get("active_size", seg.get("allocated_size", 0)) / 2 ** 30
        e["largest_gb"] = max(e["largest_gb"], seg["total_size"] / 2 ** 30)
    for k, e in sorted(by.items(), key=lambda kv: -kv[1]["reserved_gb"]):
        print(json.dumps({"stream": k[0], "pool": k[1], **{a: round(b, 2) if isinstance(b, float) else b
                                                            for a, b in e.items()}}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
