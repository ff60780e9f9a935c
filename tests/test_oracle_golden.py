"""CPU: the oracle reproduces the committed golden vectors, and the reference's shape
contracts hold (TP:823-836, 861-862, 898-899, 921, 1006-1009, 1088-1090)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as G  # noqa: E402

from oracle import ref_cpu as R  # noqa: E402


def _load(name):
    return dict(np.load(os.path.join(HERE, "golden", f"{name}.npz")))


def _cmp(got, want, rtol=2e-4):
    got = got.detach().numpy() if torch.is_tensor(got) else got
    scale = max(np.abs(want).max(), 1e-12)
    assert np.abs(got - want).max() <= rtol * scale


@pytest.mark.parametrize("case", ["fusion", "resnet18", "resnet50", "bert2"])
def test_oracle_matches_golden(case):
    torch.set_num_threads(4)
    fn = {"fusion": G.fusion_case, "resnet18": lambda: G.resnet_case("resnet18"),
          "resnet50": lambda: G.resnet_case("resnet50"), "bert2": G.bert_case}[case]
    got = fn()
    want = _load(case)
    assert set(got) == set(want)
    for k in want:
        _cmp(got[k], want[k])


@pytest.mark.parametrize("case,image,seed", [("c1", "e1.jpg", 14), ("c1_e2", "e2.jpg", 15)])
def test_c1_golden_logits(case, image, seed):
    """C1 on both of the reference's sample images (backend/sample_images/e1.jpg, e2.jpg)."""
    torch.set_num_threads(4)
    got = G.c1_case(image, seed)
    want = _load(case)
    _cmp(got["x"], want["x"], 1e-6)
    _cmp(got["logits"], want["logits"])
    assert want["logits"].shape == (1, 13)


def test_reference_shape_contracts():
    torch.manual_seed(0)
    img = R.RefImageEncoderCNN("resnet18")
    x = torch.randn(2, 3, 64, 64)
    out = img(x)
    assert tuple(out["embeddings"].shape) == (2, 1024)   # TP:861
    assert tuple(out["logits"].shape) == (2, 13)         # TP:862
    fus = R.RefFusion()
    o = fus(torch.randn(2, 1024), torch.randn(2, 512))
    assert tuple(o["disease_logits"].shape) == (2, 13)   # TP:1088
    assert o["gen"] is None                              # TP:595 (report_labels=None)


def test_resnet_topology_matches_torchvision_counts():
    # torchvision resnet18/50 total params 11,689,512 / 25,557,032 (fc included)
    for arch, total in (("resnet18", 11689512), ("resnet50", 25557032)):
        children, _ = R.resnet_children(arch)
        assert sum(p.numel() for m in children for p in m.parameters()) == total
