"""Acquire the datasets and trained models the reference's download scripts fetch.

Parity map (reference file -> target here):
  datasets/pf-pascal/download.sh:1-2   -> ``pf-pascal``  (zip, JPEGImages only)
  datasets/ivd/make_dirs.sh:1-3        -> ``ivd``        (directory tree from dirs.txt)
  datasets/ivd/download.sh:1           -> ``ivd``        (3,708 images from urls.txt, 8 parallel fetches)
  datasets/inloc/download.sh:1-2       -> ``inloc``      (cutouts + iPhone7 query tarballs)
  trained_models/download.sh:1-2       -> ``models``     (ncnet_pfpascal / ncnet_ivd checkpoints)

The pair lists (``datasets/*/image_pairs/*.csv``), ``ivd/dirs.txt`` and
``ivd/urls.txt`` ship in the repository, so ``train.py`` with the reference's
default flags finds its CSVs; only images and weights are fetched.  Fetches are
resumable: a file that already exists with non-zero size is skipped.  This
needs network access (the build/GPU boxes have none: use ``--dry-run`` there).

    python scripts/fetch_assets.py pf-pascal ivd inloc models [--jobs 8] [--dry-run]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import sys
import tarfile
import urllib.request
import zipfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DATASETS = ROOT / "datasets"

PF_ZIP = "https://www.di.ens.fr/willow/research/proposalflow/dataset/PF-dataset-PASCAL.zip"
INLOC = ("http://www.ok.sc.e.titech.ac.jp/INLOC/materials/cutouts.tar.gz",
         "http://www.ok.sc.e.titech.ac.jp/INLOC/materials/iphone7.tar.gz")
MODELS = ("https://www.di.ens.fr/willow/research/ncnet/models/ncnet_pfpascal.pth.tar",
          "https://www.di.ens.fr/willow/research/ncnet/models/ncnet_ivd.pth.tar")


def _fetch(url: str, dst: Path, dry: bool) -> str:
    if dst.exists() and dst.stat().st_size > 0:
        return f"skip {dst}"
    if dry:
        return f"would fetch {url} -> {dst}"
    dst.parent.mkdir(parents=True, exist_ok=True)
    tmp = dst.with_suffix(dst.suffix + ".part")
    with urllib.request.urlopen(url, timeout=120) as r, open(tmp, "wb") as f:
        shutil.copyfileobj(r, f, 1 << 20)
    os.replace(tmp, dst)
    return f"ok {dst}"


def read_pairs_file(path: Path):
    """Lines of ``<relative path> <url>`` (ivd/urls.txt) or ``<dir>`` (dirs.txt)."""
    out = []
    for line in path.read_text().splitlines():
        parts = line.split()
        if parts:
            out.append(parts)
    return out


def pf_pascal(dry: bool, jobs: int) -> None:
    base = DATASETS / "pf-pascal"
    z = base / "PF-dataset-PASCAL.zip"
    print(_fetch(PF_ZIP, z, dry))
    if dry:
        return
    with zipfile.ZipFile(z) as zf:
        members = [m for m in zf.namelist() if m.startswith("PF-dataset-PASCAL/JPEGImages/")]
        zf.extractall(base, members)
    print(f"extracted {len(members)} JPEGs under {base / 'PF-dataset-PASCAL'}")


def ivd(dry: bool, jobs: int) -> None:
    base = DATASETS / "ivd"
    for parts in read_pairs_file(base / "dirs.txt"):
        if not dry:
            (base / parts[0]).mkdir(parents=True, exist_ok=True)
    todo = [(url, base / rel) for rel, url in read_pairs_file(base / "urls.txt")]
    print(f"ivd: {len(todo)} images, {jobs} parallel fetches")
    fails = 0
    with cf.ThreadPoolExecutor(jobs) as ex:
        for fut in cf.as_completed([ex.submit(_fetch, u, d, dry) for u, d in todo]):
            try:
                msg = fut.result()
                if dry:
                    continue
            except Exception as e:  # keep going, report at the end (xargs -P semantics)
                fails += 1
                msg = f"FAILED {e!r}"
                print(msg, file=sys.stderr)
    if fails:
        print(f"ivd: {fails} downloads failed; re-run to resume", file=sys.stderr)


def inloc(dry: bool, jobs: int) -> None:
    base = DATASETS / "inloc"
    for url in INLOC:
        dst = base / url.rsplit("/", 1)[1]
        print(_fetch(url, dst, dry))
        if not dry:
            with tarfile.open(dst) as tf:
                tf.extractall(base, filter="data")


def models(dry: bool, jobs: int) -> None:
    for url in MODELS:
        print(_fetch(url, ROOT / "trained_models" / url.rsplit("/", 1)[1], dry))


TARGETS = {"pf-pascal": pf_pascal, "ivd": ivd, "inloc": inloc, "models": models}


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("targets", nargs="+", choices=sorted(TARGETS))
    p.add_argument("--jobs", type=int, default=8)
    p.add_argument("--dry-run", action="store_true")
    a = p.parse_args(argv)
    for t in a.targets:
        TARGETS[t](a.dry_run, a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
