"""ViT-B/16 tower (C5) on the HIP path vs the oracle's torchvision restatement.
Two encoder layers (the per-layer arithmetic is identical across layers), B = 2, 224x224.
fp32: features rel err <= 1e-4; every parameter gradient 1 - cos <= 1e-4.
bf16: features rel err <= 5e-2."""
import pytest
import torch

from mmdx.vit import VitTrunk
from oracle import ref_cpu as R
from parity_util import cosine, rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
def test_vit_trunk_parity(dev, dt):
    torch.manual_seed(0)
    ref = R.RefVitTrunk(layers=2)
    mine = VitTrunk(layers=2)
    mine.load_state_dict(ref.state_dict())
    mine.compute_dtype = dt
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 3, 224, 224, generator=g)
    f_ref = ref(x)
    dy = torch.randn(f_ref.shape, generator=g)
    f_ref.backward(dy)
    mine.to(dev)
    f = mine(x.to(dev))
    assert tuple(f.shape) == (2, 768)
    assert rel_err(f, f_ref) <= (1e-4 if dt == torch.float32 else 5e-2)
    if dt == torch.bfloat16:
        return
    f.float().backward(dy.to(dev))
    gm = dict(mine.named_parameters())
    bad = []
    # fp16 (C5's "fp16 MFMA"): gradients 1 - cos <= 1e-2 against the fp32 oracle
    tol = 1e-4 if dt == torch.float32 else 1e-2
    for n, p in ref.named_parameters():
        assert torch.isfinite(gm[n].grad).all(), n
        c = cosine(gm[n].grad, p.grad)
        if 1 - c > tol:
            bad.append((n, 1 - c))
    assert not bad, bad
