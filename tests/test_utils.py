import os

import numpy as np
import torch

from ncnet_amd.data.transforms import normalize_image
from ncnet_amd.utils.plot import denormalize_image, plot_image, save_plot
from ncnet_amd.utils.torch_util import (BatchToDevice, collate_custom, create_file_path, expand_dim, softmax_1d,
                                        str_to_bool)


def test_collate_custom_keeps_lists():
    b = [{"a": torch.ones(2), "pts": [1, 2]}, {"a": torch.zeros(2), "pts": [3]}]
    out = collate_custom(b)
    assert out["a"].shape == (2, 2)
    assert out["pts"] == [[1, 2], [3]]


def test_batch_to_device_softmax_expand(tmp_path):
    out = BatchToDevice("cpu")({"x": torch.ones(3), "name": "q"})
    assert out["name"] == "q" and out["x"].device.type == "cpu"
    x = torch.randn(4, 5)
    assert torch.allclose(softmax_1d(x, 1), torch.softmax(x, 1))
    assert expand_dim(torch.ones(1, 3), 0, 4).shape == (4, 3)
    p = tmp_path / "a" / "b" / "c.txt"
    create_file_path(str(p))
    assert os.path.isdir(p.parent)
    assert str_to_bool("yes") and not str_to_bool("0")


def test_plot_roundtrip(tmp_path):
    img = torch.rand(3, 8, 10)
    arr = plot_image(normalize_image(img), return_im=True)
    assert arr.shape == (8, 10, 3) and arr.dtype == np.uint8
    assert np.abs(arr.astype(float) - img.permute(1, 2, 0).numpy() * 255).max() <= 1.0
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    plt.figure()
    plt.imshow(denormalize_image(normalize_image(img)))
    save_plot(str(tmp_path / "x.png"))
    plt.close("all")
    assert (tmp_path / "x.png").exists()


def test_runtime_config_from_env():
    from ncnet_amd.config import RuntimeConfig
    c = RuntimeConfig.from_env({"NCNET_TRUNK_GRAPH": "0", "NCNET_BWD_OVERLAP": "0", "NCNET_GP_TPW": "3",
                                "NCNET_TRUNK_CONV": "native"})
    assert not c.trunk_graph and c.trunk_plan and not c.bwd_overlap and c.gp_tpw == 3 and c.trunk_conv == "native"
    assert set(c.as_dict()) >= {"trunk_prefetch", "allow_torch_fallback", "nc_fp8", "stats2d", "nt_store"}
    assert set(c.tuning()) == set(RuntimeConfig.TUNING)


def test_runtime_override_restores():
    from ncnet_amd import config
    before = config.RUNTIME
    with config.override(nc_fp8=True, gp_tpw=2) as c:
        assert config.RUNTIME is c and c.nc_fp8 and c.gp_tpw == 2
    assert config.RUNTIME is before


def test_no_environment_reads_outside_config():
    """the NCNET_* switches are read once, in ncnet_amd/config.py;
    the package reads no other environment variable but the launcher's
    (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* / TORCHELASTIC_RUN_ID) and the
    build script's."""
    import pathlib
    import re
    root = pathlib.Path(__file__).resolve().parents[1] / "ncnet_amd"
    allowed = {"WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR", "TORCHELASTIC_RUN_ID"}
    bad = []
    for f in list(root.rglob("*.py")) + list(root.rglob("*.hip")) + list(root.rglob("*.h")) + list(root.rglob("*.cpp")):
        if f.name in ("config.py", "build.py"):
            continue
        for n, line in enumerate(f.read_text().splitlines(), 1):
            for m in re.finditer(r'(?:os\.environ(?:\.get|\.setdefault)?\(?\[?|getenv\()\s*"([A-Z_]+)"', line):
                if m.group(1) not in allowed:
                    bad.append(f"{f.name}:{n}: {m.group(1)}")
            if "getenv(" in line and "getenv(\"" not in line:
                bad.append(f"{f.name}:{n}: getenv")
    assert not bad, bad


def test_segment_timer_cpu():
    from ncnet_amd.utils.timing import SegmentTimer, segment, set_active
    t = SegmentTimer(device="cpu")
    set_active(t)
    try:
        for _ in range(3):
            with segment("a"):
                torch.ones(10).sum()
        with segment("b"):
            pass
    finally:
        set_active(None)
    ms = t.collect()
    assert set(ms) == {"a", "b"} and all(v >= 0 for v in ms.values())
    assert t.collect() == {}
    with segment("ignored"):   # no active timer: null context
        pass


def test_affine_tnf_identity_and_resize():
    from ncnet_amd.data.transforms import AffineTnf, gpu_normalize_resize, resize_bilinear
    img = torch.rand(2, 3, 12, 16)
    out = AffineTnf(12, 16)(img)
    assert torch.allclose(out, img, atol=1e-5)            # identity theta, align_corners=True
    r = resize_bilinear(img, 6, 8)
    assert torch.allclose(AffineTnf(6, 8)(img), r, atol=1e-5)
    u8 = (torch.rand(1, 3, 12, 16) * 255).to(torch.uint8)
    n = gpu_normalize_resize(u8, 12, 16)
    assert torch.allclose(normalize_image(u8.float() / 255.0), n, atol=1e-5)


def test_train_segment_timing_and_profile(tmp_path):
    import json
    import train
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        train.main(["--synthetic", "4", "--batch_size", "2", "--image_size", "64", "--ncons_kernel_sizes", "3", "3",
                    "--ncons_channels", "16", "1", "--max_steps", "2", "--segment_timing", "--profile", "prof",
                    "--metrics", "m.jsonl"])
        assert os.path.exists("prof/train_profile.txt") and os.path.exists("prof/train_trace.json")
        train.main(["--synthetic", "4", "--batch_size", "2", "--image_size", "64", "--ncons_kernel_sizes", "3", "3",
                    "--ncons_channels", "16", "1", "--num_epochs", "1", "--segment_timing", "--metrics", "m.jsonl",
                    "--result-model-dir", "models"])
        recs = [json.loads(x) for x in open("m.jsonl")]
        seg = [r["segments_ms"] for r in recs if r["mode"] == "train" and "segments_ms" in r]
        assert seg and {"backbone", "correlation", "neigh_consensus", "backward", "optimizer"} <= set(seg[0])
    finally:
        os.chdir(old)


def test_reference_pair_lists_ship():
    """The reference's pair CSVs (datasets/*/image_pairs) are in the
    tree at train.py's default --dataset_csv_path, with the reference counts."""
    import os

    from ncnet_amd.data.datasets import ImagePairDataset, PFPascalDataset

    root = os.path.join(os.path.dirname(__file__), "..", "datasets")
    pf = os.path.join(root, "pf-pascal", "image_pairs")
    assert len(ImagePairDataset(pf, "train_pairs.csv", "unused")) == 2940
    assert len(ImagePairDataset(pf, "val_pairs.csv", "unused")) == 308
    ivd = os.path.join(root, "ivd", "image_pairs")
    tr = ImagePairDataset(ivd, "train_pairs.csv", "unused")
    assert len(tr) == 6932 and int(tr.flip.sum()) == 3466
    assert len(ImagePairDataset(ivd, "val_pairs.csv", "unused")) == 758
    test = PFPascalDataset(os.path.join(pf, "test_pairs.csv"), "unused", output_size=(400, 400))
    assert len(test) == 299


def test_fetch_assets_dry_run(capsys):
    import importlib.util
    import os

    p = os.path.join(os.path.dirname(__file__), "..", "scripts", "fetch_assets.py")
    spec = importlib.util.spec_from_file_location("fetch_assets", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.main(["pf-pascal", "models", "--dry-run"]) == 0
    out = capsys.readouterr().out
    assert "PF-dataset-PASCAL.zip" in out and "ncnet_ivd.pth.tar" in out
    assert len(m.read_pairs_file(m.DATASETS / "ivd" / "urls.txt")) == 3708


def test_gpu_resize_path_matches_cpu_resize(tmp_path):
    """The uint8 decode-only dataset + batched resize/normalise (train.py's GPU
    path, run here on CPU tensors) equals the reference-style per-sample CPU
    resize + NormalizeImageDict."""
    import sys

    import torch

    sys.path.insert(0, str(tmp_path.parent))
    from ncnet_amd.data.datasets import ImagePairDataset, collate_uint8_pairs, gpu_pair_batch
    from ncnet_amd.data.transforms import NormalizeImageDict
    import importlib.util
    import os
    p = os.path.join(os.path.dirname(__file__), "..", "scripts", "make_jpeg_pairs.py")
    spec = importlib.util.spec_from_file_location("mkj", p)
    mkj = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mkj)
    mkj.main(["--out", str(tmp_path), "--pairs", "6"])
    csv = str(tmp_path / "image_pairs")
    norm = NormalizeImageDict(["source_image", "target_image"])
    a = ImagePairDataset(csv, "train_pairs.csv", str(tmp_path), output_size=(64, 80), transform=norm)
    b = ImagePairDataset(csv, "train_pairs.csv", str(tmp_path), output_size=(64, 80), transform=norm, gpu_resize=True)
    sa = [a[i] for i in range(3)]
    batch = gpu_pair_batch(collate_uint8_pairs([b[i] for i in range(3)]), "cpu", 64, 80)
    for k in ("source_image", "target_image"):
        want = torch.stack([s[k] for s in sa])
        assert batch[k].shape == want.shape == (3, 3, 64, 80)
        assert torch.allclose(batch[k], want, atol=1e-4)
    assert torch.equal(batch["source_im_size"], torch.stack([s["source_im_size"] for s in sa]))
