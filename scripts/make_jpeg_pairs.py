#!/usr/bin/env python
"""Write N random JPEG pairs in PF-Pascal size ranges (longest side 300-500 px,
4:3 / 3:4 / square) plus train/val pair CSVs in the reference layout
(``source_image,target_image,class,flip``) -- the real-data input path's
benchmark set when the datasets cannot be downloaded.

    python scripts/make_jpeg_pairs.py --out /tmp/jpeg_pairs --pairs 1000
"""
import argparse
import os

import numpy as np
from PIL import Image


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--pairs", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    rng = np.random.default_rng(a.seed)
    img_dir = os.path.join(a.out, "images")
    os.makedirs(img_dir, exist_ok=True)
    os.makedirs(os.path.join(a.out, "image_pairs"), exist_ok=True)
    names = []
    for i in range(2 * a.pairs):
        long = int(rng.integers(300, 501))
        short = int(long * rng.choice([0.75, 1.0]))
        h, w = (short, long) if rng.random() < 0.6 else (long, short)
        # smooth colour field + noise: JPEG decode cost like a photo, not like flat colour
        base = rng.integers(0, 256, size=(h // 16 + 2, w // 16 + 2, 3), dtype=np.uint8)
        im = Image.fromarray(base).resize((w, h), Image.BICUBIC)
        arr = np.asarray(im).astype(np.int16) + rng.integers(-20, 21, size=(h, w, 3))
        name = f"img_{i:05d}.jpg"
        Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8)).save(os.path.join(img_dir, name), quality=90)
        names.append("images/" + name)
    rows = [f"{names[2 * i]},{names[2 * i + 1]},{i % 20 + 1},{i % 2}" for i in range(a.pairs)]
    nval = max(1, a.pairs // 10)
    for fn, part in (("train_pairs.csv", rows[nval:]), ("val_pairs.csv", rows[:nval])):
        with open(os.path.join(a.out, "image_pairs", fn), "w") as f:
            f.write("source_image,target_image,class,flip\n" + "\n".join(part) + "\n")
    print(f"wrote {2 * a.pairs} JPEGs to {img_dir}")


if __name__ == "__main__":
    main()
