"""two_tower_backward == loss.backward() (grads of every parameter, bit-exact on CPU)."""
import torch
import torch.nn as nn

from mmdx.schedule import two_tower_backward


def _model(seed):
    torch.manual_seed(seed)
    img = nn.Sequential(nn.Linear(12, 16), nn.GELU(), nn.Linear(16, 8))
    txt = nn.Sequential(nn.Embedding(50, 8), nn.Flatten(), nn.Linear(8 * 5, 4))
    head = nn.Sequential(nn.Linear(12, 10), nn.GELU(), nn.LayerNorm(10), nn.Linear(10, 3))
    return img, txt, head


def _loss(img, txt, head, x, ids, y):
    z_img, z_txt = img(x), txt(ids)
    logits = head(torch.cat([z_img, z_txt], -1))
    return nn.functional.binary_cross_entropy_with_logits(logits, y), z_img, z_txt


def test_two_tower_backward_matches_plain_backward():
    g = torch.Generator().manual_seed(0)
    x, ids = torch.randn(6, 12, generator=g), torch.randint(0, 50, (6, 5), generator=g)
    y = (torch.rand(6, 3, generator=g) < 0.3).float()
    ref = _model(1)
    loss, _, _ = _loss(*ref, x, ids, y)
    loss.backward()
    mine = _model(1)
    loss2, z_img, z_txt = _loss(*mine, x, ids, y)
    two_tower_backward(loss2, z_img, z_txt, mine[2].parameters())
    for a, b in zip(ref, mine):
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            assert torch.equal(p.grad, q.grad), n
    assert z_img.grad is None and z_txt.grad is None


def test_two_tower_forward_threads_match_sequential():
    """TwoTowerForward (text tower issued from a worker thread) builds the same autograd
    graph as issuing the towers one after the other: identical outputs and gradients."""
    from mmdx.schedule import TwoTowerForward
    g = torch.Generator().manual_seed(0)
    x, ids = torch.randn(6, 12, generator=g), torch.randint(0, 50, (6, 5), generator=g)
    y = (torch.rand(6, 3, generator=g) < 0.3).float()
    ref = _model(2)
    loss, _, _ = _loss(*ref, x, ids, y)
    loss.backward()
    mine = _model(2)
    towers = TwoTowerForward()
    try:
        for _ in range(2):  # the worker thread is reused across steps
            for p in (q for m in mine for q in m.parameters()):
                p.grad = None
            z_img, z_txt = towers(lambda: mine[0](x), lambda: mine[1](ids))
            logits = mine[2](torch.cat([z_img, z_txt], -1))
            nn.functional.binary_cross_entropy_with_logits(logits, y).backward()
            for a, b in zip(ref, mine):
                for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
                    assert torch.equal(p.grad, q.grad), n
        with torch.no_grad():  # grad mode follows the caller into the worker thread
            _, z = towers(lambda: mine[0](x), lambda: mine[1](ids))
            assert not z.requires_grad
    finally:
        towers.close()
