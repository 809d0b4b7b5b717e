#!/usr/bin/env python
"""Host-side input pipeline capacity (no GPU): DataLoader decode + packed
uint8 collate (train.py's real-data path: ImagePairDataset(gpu_resize=True) +
collate_uint8_pairs; resize / normalise run on the GPU afterwards) over a
synthetic JPEG pair set, for several worker counts.

Reports images/s for the loader as a whole and per worker, and the number of
decode cores a node needs to feed ``--ranks`` ranks at ``--pairs-per-s`` image
pairs/s each (2 images per pair).  Reference loader: /root/reference/lib/dataloader.py:162-183
(worker processes), /root/reference/train.py:88-99 (num_workers 0 train / 4 test).

    python scripts/loader_throughput.py [--pairs 400] [--workers 1 2 4 8] [--batches 40]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=400)
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dir", default="")
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--pairs-per-s", type=float, default=700.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)

    import torch
    from torch.utils.data import DataLoader, RandomSampler

    from ncnet_amd.data.datasets import ImagePairDataset, collate_uint8_pairs

    root = a.dir or os.path.join(tempfile.gettempdir(), "ncnet_jpeg_pairs")
    if not os.path.exists(os.path.join(root, "image_pairs", "train_pairs.csv")):
        import make_jpeg_pairs  # noqa: E402  (scripts/)
        make_jpeg_pairs.main(["--out", root, "--pairs", str(a.pairs)])
    ds = ImagePairDataset(os.path.join(root, "image_pairs"), "train_pairs.csv", root, output_size=(400, 400),
                          gpu_resize=True)
    torch.set_num_threads(1)
    rows = []
    for w in a.workers:
        sampler = RandomSampler(ds, replacement=True, num_samples=a.batch * (a.batches + 4 * max(w, 1)))
        dl = DataLoader(ds, batch_size=a.batch, sampler=sampler, num_workers=w, collate_fn=collate_uint8_pairs,
                        drop_last=True, persistent_workers=False, prefetch_factor=4 if w else None)
        it = iter(dl)
        for _ in range(2 * max(w, 1)):           # worker start-up + queue fill
            next(it)
        t0 = time.perf_counter()
        n = 0
        for _ in range(a.batches):
            b = next(it)
            n += 2 * b["pixel_meta"].shape[0] // 2
        dt = time.perf_counter() - t0
        del it, dl
        ips = n / dt
        rows.append({"workers": w, "images_per_s": round(ips, 1), "per_worker": round(ips / max(w, 1), 1)})
        print(json.dumps(rows[-1]), flush=True)
    per_core = max(r["per_worker"] for r in rows)
    need = a.ranks * a.pairs_per_s * 2
    rep = {"cpus_here": os.cpu_count(), "rows": rows, "images_per_s_per_core": per_core,
           "node_need_images_per_s": need, "cores_needed": round(need / per_core, 1),
           "per_rank_workers_needed": round(need / per_core / a.ranks, 1)}
    print(json.dumps(rep), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
