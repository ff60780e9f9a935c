"""DP parity on one GPU (SURVEY §8(e) check (i)): two ranks (gloo, both on cuda:0), each
with half of the batch, all-reduce-averaged gradients == single-process full-batch
gradients, with BatchNorm in eval mode so per-replica statistics do not enter.
fp32 path; tolerance per tensor (reduction order only): 1 - cosine <= 1e-6 and the norm
ratio |g|/|g_ref| within 1e-5 of 1 (cosine alone would miss a lost or doubled 1/world)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(kind="resnet"):
    sys.path.insert(0, HERE)
    from parity_util import build_pair
    if kind == "stack":   # C5's towers: the ViT-B/16 and BERT encoder stacks (launch plans)
        _, img, txt, fus = build_pair("vit_b_16", "bert-base-uncased", bert_layers=4)
        # train-mode BERT dropout draws fresh masks every step: off, so two backwards agree
        txt.encoder.config.hidden_dropout_prob = 0.0
        txt.encoder.config.attention_probs_dropout_prob = 0.0
    else:
        _, img, txt, fus = build_pair("resnet18", "embed-mean")
    return img, txt, fus


def _grads(img, txt, fus, x, ids, mask, y):
    import mmdx
    from parity_util import mmdx_forward
    dev = torch.device("cuda", 0)
    for m in (img, txt, fus):
        m.to(dev)
    img.unfreeze_backbone()
    img.backbone.eval()  # BN on running statistics: no per-replica batch statistics
    txt.train()
    fus.train()
    logits = mmdx_forward(img, txt, fus, x.to(dev), ids.to(dev), mask.to(dev))
    mmdx.BCEWithLogitsLoss()(logits, y.to(dev)).backward()
    return [(n, p) for mod in (img, txt, fus) for n, p in mod.named_parameters()]


def _worker(rank, world, port, out, early):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx import resnet as RN
    from mmdx.dist import GradAllReducer, shard_batch
    from parity_util import synth_batch
    x, ids, mask, y = synth_batch(4, 16, hw=64)
    a, b = shard_batch(4, rank, world)
    img, txt, fus = _model()
    red = GradAllReducer([p for mod in (img, txt, fus) for p in mod.parameters()], world)
    tails = []
    if early == "event":  # layers 4, 3, 2 reduced from the plan's mid-backward events
        def hook(g, regions):
            tails.extend((lo, hi, g.numel()) for lo, hi, _ in regions)
            red.trunk_hook(g, regions)
        RN.TRUNK_GRAD_HOOK = hook
    elif early == "seg":  # ... in place, issued between the backward plan's segments
        def seg(g, lo, hi):
            assert torch.cuda.current_stream() != torch.cuda.default_stream()
            tails.append((lo, hi, g.numel()))
            red.trunk_segment(g, lo, hi)
        RN.TRUNK_SEGMENT_HOOK = seg
    named = _grads(img, txt, fus, x[a:b], ids[a:b], mask[a:b], y[a:b])
    red.reduce()
    RN.TRUNK_GRAD_HOOK = RN.TRUNK_SEGMENT_HOOK = None
    if early:  # three contiguous slices ending at the arena's end, in backward order
        assert len(tails) == 3, tails
        assert tails[0][1] == tails[0][2] and tails[1][1] == tails[0][0], tails
        assert tails[2][1] == tails[1][0] and 0 < tails[2][0] < tails[2][1], tails
    torch.cuda.synchronize()
    out[rank] = {n: p.grad.detach().cpu() for n, p in named if p.grad is not None}
    dist.destroy_process_group()


@pytest.mark.parametrize("early", [False, "event", "seg"])
def test_dp_two_ranks_match_full_batch(dev, early):
    from parity_util import cosine, norm_ratio, synth_batch
    x, ids, mask, y = synth_batch(4, 16, hw=64)
    img, txt, fus = _model()
    ref = {n: p.grad.detach().cpu() for n, p in _grads(img, txt, fus, x, ids, mask, y)
           if p.grad is not None}
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out, early)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    for r in range(2):
        g = out[r]
        assert set(g) == set(ref)
        for n in ref:
            c = cosine(g[n], ref[n])
            assert 1 - c <= 1e-6, f"rank {r} {n}: 1-cos {1 - c:.2e}"
            nr = norm_ratio(g[n], ref[n])
            assert abs(nr - 1) <= 1e-5, f"rank {r} {n}: norm ratio {nr:.7f}"


def _rccl_worker(port, out, early):
    """One-rank RCCL group: the nccl-backend path of GradAllReducer (AVG collectives, the
    arena found by storage and reduced in place, optional early trunk tail on a comm
    stream or in place between the backward plan's segments, bucket unpack) must leave every gradient exactly as the local backward made it
    (the mean over one rank is the identity)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from mmdx import resnet as RN
    from mmdx import xplan as XP
    from mmdx.dist import GradAllReducer
    from parity_util import synth_batch
    kind = "stack" if early == "stack" else "resnet"
    x, ids, mask, y = synth_batch(2, 16, hw=224) if kind == "stack" else synth_batch(4, 16, hw=64)
    img, txt, fus = _model(kind)
    params = [p for mod in (img, txt, fus) for p in mod.parameters()]
    _grads(img, txt, fus, x, ids, mask, y)
    ref = {id(p): p.grad.detach().clone() for p in params if p.grad is not None}
    for p in params:
        p.grad = None
    if kind == "stack":   # run-to-run determinism of the local backward itself
        _grads(img, txt, fus, x, ids, mask, y)
        out["base_diff"] = [(i, (p.grad - ref[id(p)]).abs().max().item())
                            for i, p in enumerate(params)
                            if p.grad is not None and not torch.equal(p.grad, ref[id(p)])][:8]
        for p in params:
            p.grad = None
    red = GradAllReducer(params, 1, rehearse=True)
    assert red._avg
    if early == "event":
        RN.TRUNK_GRAD_HOOK = red.trunk_hook
    elif early == "seg":
        RN.TRUNK_SEGMENT_HOOK = red.trunk_segment
    elif early == "stack":   # the encoder stacks' backward segments (xplan.STACK_SEGMENT_HOOK)
        XP.STACK_SEGMENT_HOOK = red.trunk_segment
    _grads(img, txt, fus, x, ids, mask, y)
    RN.TRUNK_GRAD_HOOK = RN.TRUNK_SEGMENT_HOOK = XP.STACK_SEGMENT_HOOK = None
    if kind == "stack":
        out["segments"] = len(red._pending)   # 3 ViT groups + 1 BERT group, issued mid-backward
        trunk_p = {id(p) for p in list(img.backbone.encoder.layers.parameters())
                   + list(txt.encoder.encoder.layer.parameters())}
    else:
        trunk_p = {id(p) for p in img.backbone.parameters()}
    trunk = {id(p.grad) for p in params if id(p) in trunk_p and p.grad is not None}
    red.launch()
    packed = sum(1 for b, *_ in red._pending if b is not None for _, t in b if id(t) in trunk)
    red.finish()
    torch.cuda.synchronize()
    bad = []
    for i, p in enumerate(params):
        if p.grad is None:
            continue
        g, r = p.grad, ref[id(p)]
        if id(p) in trunk_p:  # the arena: reduced in place, must be untouched bit for bit
            ok = torch.equal(g, r)
        else:  # (the text embedding's gradient is an atomic scatter: its bits vary per run)
            ok = torch.allclose(g, r, rtol=1e-6, atol=1e-7)
        if not ok:
            bad.append(i)
            out["diff"] = out.get("diff", []) + [(i, (g - r).abs().max().item(),
                                                  r.abs().max().item())][:8]
    out["packed"] = packed
    out["bad"] = bad
    out["n"] = len(ref)
    dist.destroy_process_group()


@pytest.mark.parametrize("early", [False, "event", "seg", "stack"])
def test_dp_rccl_one_rank_identity(dev, early):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    p = ctx.Process(target=_rccl_worker, args=(_port(), out, early))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0
    assert out["n"] > 50
    assert out["packed"] == 0, "trunk arena gradients went through a packed bucket"
    assert out["bad"] == [], (out["bad"][:10], out.get("base_diff"), out.get("diff"))
    if early == "stack":
        assert out["segments"] == 4, out["segments"]
