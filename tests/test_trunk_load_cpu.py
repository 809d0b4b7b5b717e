"""Strict loading of a local feature_extraction_model_file (models/backbones.py
load_trunk_state): the whole torchvision model's keys or the trunk's own keys
load; layers past the truncation are dropped; a missing, unknown or misshaped
tensor raises naming it (reference: lib/model.py:37-44 truncates a pretrained
torchvision resnet101)."""
import pytest
import torch

from ncnet_amd.models.backbones import ResNet, build_trunk, load_trunk_state, vgg16_trunk
from ncnet_amd.models.immatchnet import FeatureExtraction


def _full_resnet_sd(seed=0):
    torch.manual_seed(seed)
    net = ResNet((3, 4, 6, 3))
    sd = dict(net.state_dict())
    sd["fc.weight"] = torch.randn(10, 2048)
    sd["fc.bias"] = torch.randn(10)
    return sd


def test_full_torchvision_keys_load(tmp_path):
    sd = _full_resnet_sd()
    f = tmp_path / "r50.pth"
    torch.save(sd, f)
    fe = FeatureExtraction(feature_extraction_cnn="resnet50", feature_extraction_model_file=str(f), use_cuda=False)
    got = fe.model.state_dict()
    assert torch.equal(got["0.weight"], sd["conv1.weight"])
    assert torch.equal(got["6.5.conv3.weight"], sd["layer3.5.conv3.weight"])
    assert torch.equal(got["4.0.downsample.1.running_var"], sd["layer1.0.downsample.1.running_var"])


def test_trunk_keys_and_prefixes_load():
    trunk, _, _ = build_trunk("resnet50")
    src, _, _ = build_trunk("resnet50")
    sd = {"module.model." + k: v.clone() + 1 for k, v in src.state_dict().items()}
    load_trunk_state(trunk, sd, "resnet50")
    assert torch.equal(trunk.state_dict()["1.bias"], src.state_dict()["1.bias"] + 1)


def test_missing_key_is_named():
    sd = _full_resnet_sd()
    del sd["layer2.1.bn2.weight"]
    trunk, _, _ = build_trunk("resnet50")
    with pytest.raises(RuntimeError, match=r"missing 1: 5\.1\.bn2\.weight"):
        load_trunk_state(trunk, sd, "resnet50")


def test_unexpected_and_shape_errors():
    trunk, _, _ = build_trunk("resnet50")
    sd = _full_resnet_sd()
    sd["layer3.0.extra"] = torch.zeros(1)
    with pytest.raises(RuntimeError, match=r"unexpected 1: 6\.0\.extra"):
        load_trunk_state(trunk, sd, "resnet50")
    sd = _full_resnet_sd()
    sd["conv1.weight"] = torch.zeros(64, 3, 3, 3)
    with pytest.raises(RuntimeError, match=r"shape mismatch 1: 0\.weight"):
        load_trunk_state(trunk, sd, "resnet50")


def test_vgg_features_keys():
    full = vgg16_trunk("pool5")
    sd = {"features." + k: v for k, v in full.state_dict().items()}
    sd["classifier.0.weight"] = torch.zeros(4096, 25088)
    trunk, _, _ = build_trunk("vgg")
    load_trunk_state(trunk, sd, "vgg")
    assert torch.equal(trunk.state_dict()["21.weight"], full.state_dict()["21.weight"])


def test_file_without_num_batches_tracked_loads():
    """ImageNet checkpoints older than BatchNorm's counter have no
    num_batches_tracked keys; BN's own loader fills them with 0, and so must
    the strict trunk load."""
    sd = {k: v for k, v in _full_resnet_sd().items() if not k.endswith("num_batches_tracked")}
    trunk, _, _ = build_trunk("resnet50")
    load_trunk_state(trunk, sd, "resnet50")
    got = trunk.state_dict()
    assert torch.equal(got["6.5.conv3.weight"], sd["layer3.5.conv3.weight"])
    assert int(got["1.num_batches_tracked"]) == 0


def test_densenet_legacy_keys_load():
    """The legacy torchvision densenet file names 'denselayerN.norm.1.weight';
    the load remaps it to 'norm1' as torchvision's densenet loader does."""
    import re
    src, _, _ = build_trunk("densenet201")
    pat = re.compile(r"^(.*denselayer\d+\.(?:norm|relu|conv))((?:[12])\.(?:weight|bias|running_mean|running_var))$")
    sd = {}
    for k, v in src.state_dict().items():
        if k.endswith("num_batches_tracked"):
            continue
        m = pat.match(k)
        sd[(m.group(1) + "." + m.group(2)) if m else k] = v.clone() + 1
    assert any(".norm.1." in k for k in sd)
    trunk, _, _ = build_trunk("densenet201")
    load_trunk_state(trunk, sd, "densenet201")
    k = next(k for k in trunk.state_dict() if "denselayer" in k and k.endswith("norm1.weight"))
    assert torch.equal(trunk.state_dict()[k], src.state_dict()[k] + 1)
