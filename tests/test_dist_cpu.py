"""CPU: the DP gradient all-reduce (mmdx.dist.GradAllReducer) over gloo, world_size 2."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import mmdx
    from mmdx.dist import GradAllReducer, shard_batch
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(s)) for s in ((300, 70), (70,), (13, 5), (4,))]
    g = torch.Generator().manual_seed(100 + rank)
    for p in params:
        p.grad = torch.randn(p.shape, generator=g)
    red = GradAllReducer(params, world, bucket_bytes=4096)
    red.reduce()
    out[rank] = [p.grad.clone() for p in params]
    assert shard_batch(1024, rank, world) == (rank * 512, (rank + 1) * 512)
    dist.destroy_process_group()


def test_grad_allreduce_mean_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    exp = []
    for r in range(world):
        g = torch.Generator().manual_seed(100 + r)
        exp.append([torch.randn(s, generator=g) for s in ((300, 70), (70,), (13, 5), (4,))])
    mean = [(a + b) / 2 for a, b in zip(*exp)]
    for r in range(world):
        for got, want in zip(out[r], mean):
            assert torch.allclose(got, want, atol=1e-6)


SHAPES2 = ((40, 3), (7,), (16,), (5, 5))


def _worker_frozen(rank, world, port, out):
    """A partially frozen trunk: one arena slot has no gradient (requires_grad=False), the
    early tail (trunk_hook) ran on the arena — the rest is reduced once, in place, and no
    arena gradient also goes through a packed bucket (it would be reduced twice)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx.dist import GradAllReducer
    params = [torch.nn.Parameter(torch.zeros(s)) for s in SHAPES2]
    params[1].requires_grad_(False)
    g = torch.Generator().manual_seed(400 + rank)
    flat = torch.randn(127, generator=g)
    params[0].grad = flat[:120].view(40, 3).detach()
    params[2].grad = torch.randn(16, generator=g)
    params[3].grad = torch.randn(5, 5, generator=g)
    red = GradAllReducer(params, world, bucket_bytes=64, small_arena_bytes=0)
    red.trunk_hook(flat, [(60, 120, None)])
    red.launch()
    assert all(b is None or id(params[0].grad) not in {id(g) for _, g in b}
               for b, *_ in red._pending), "arena gradient in a packed bucket"
    red.finish()
    out[rank] = [params[0].grad.clone(), params[2].grad.clone(), params[3].grad.clone()]
    dist.destroy_process_group()


def test_grad_allreduce_frozen_trunk_slot_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_frozen, args=(world, port, out), nprocs=world, join=True)
    exp = []
    for r in range(world):
        g = torch.Generator().manual_seed(400 + r)
        flat = torch.randn(127, generator=g)
        exp.append([flat[:120].view(40, 3), torch.randn(16, generator=g),
                    torch.randn(5, 5, generator=g)])
    mean = [(a + b) / 2 for a, b in zip(*exp)]
    for r in range(world):
        for got, want in zip(out[r], mean):
            assert torch.allclose(got, want, atol=1e-6)


def _worker_flat(rank, world, port, out, region=0, detach=False):
    """Gradients that are views of one flat buffer (the trunk's gradient arena) are reduced
    in place; the others through buckets; a subset is launched early (overlap path).
    detach: the views are stored detached, as autograd's AccumulateGrad stores a view a
    backward returns (.grad._base is None) — the arena is found by its storage."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx.dist import GradAllReducer
    params = [torch.nn.Parameter(torch.zeros(s)) for s in SHAPES2]
    g = torch.Generator().manual_seed(200 + rank)
    flat = torch.randn(40 * 3 + 7, generator=g)
    params[0].grad = flat[:120].view(40, 3)
    params[1].grad = flat[120:127]
    if detach:
        params[0].grad = params[0].grad.detach()
        params[1].grad = params[1].grad.detach()
        assert params[0].grad._base is None
    params[2].grad = torch.randn(16, generator=g)
    params[3].grad = torch.randn(5, 5, generator=g)
    red = GradAllReducer(params, world, bucket_bytes=64, small_arena_bytes=0)
    if region == 1:  # the buffer's tail first (the trunk's last layer)
        red.launch_region(flat, 100, flat.numel())
    elif region == 2:  # per-layer slices in backward order (resnet.TRUNK_GRAD_HOOK)
        red.trunk_hook(flat, [(100, 127, None), (60, 100, None), (30, 60, None)])
    elif region == 3:  # in place from between the plan's segments (resnet.TRUNK_SEGMENT_HOOK)
        for lo, hi in ((100, 127), (60, 100), (30, 60)):
            red.trunk_segment(flat, lo, hi)
    red.launch([params[2]])
    red.launch()
    arena = {id(params[0].grad), id(params[1].grad)}
    assert all(b is None or not arena & {id(g) for _, g in b} for b, *_ in red._pending), \
        "arena gradients went through a packed bucket"
    red.finish()
    if not detach:
        assert params[0].grad._base is flat  # reduced in place, still the same buffer
    assert params[0].grad.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
    out[rank] = [p.grad.clone() for p in params]
    dist.destroy_process_group()


@pytest.mark.parametrize("region,detach", [(0, False), (1, False), (2, False), (2, True),
                                           (3, False), (3, True)])
def test_grad_allreduce_flat_base_and_early_launch_gloo(region, detach):
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_flat, args=(world, port, out, region, detach), nprocs=world, join=True)
    exp = []
    for r in range(world):
        g = torch.Generator().manual_seed(200 + r)
        flat = torch.randn(127, generator=g)
        exp.append([flat[:120].view(40, 3), flat[120:127], torch.randn(16, generator=g),
                    torch.randn(5, 5, generator=g)])
    mean = [(a + b) / 2 for a, b in zip(*exp)]
    for r in range(world):
        for got, want in zip(out[r], mean):
            assert torch.allclose(got, want, atol=1e-6)


def _worker_small_arena(rank, world, port, out):
    """A whole flat buffer below small_arena_bytes (the BiLSTM's per-layer weight / bias
    pairs) travels in the packed bucket with the loose gradients — one collective — and every
    .grad is rebound to its view of the averaged bucket."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx import dist as D
    params = [torch.nn.Parameter(torch.zeros(s)) for s in SHAPES2]
    g = torch.Generator().manual_seed(200 + rank)
    flat = torch.randn(127, generator=g)
    params[0].grad = flat[:120].view(40, 3).detach()
    params[1].grad = flat[120:127].detach()
    params[2].grad = torch.randn(16, generator=g)
    params[3].grad = torch.randn(5, 5, generator=g)
    red = D.GradAllReducer(params, world)
    calls = []
    real = red._all_reduce
    red._all_reduce = lambda t, kind: (calls.append(kind), real(t, kind))[1]
    red.reduce()
    assert calls == ["bucket[4]"], calls
    assert all(p.grad.untyped_storage().data_ptr() != flat.untyped_storage().data_ptr()
               for p in params[:2])
    assert len({p.grad.untyped_storage().data_ptr() for p in params}) == 1
    out[rank] = [p.grad.clone() for p in params]
    dist.destroy_process_group()


def test_small_arena_packed_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_small_arena, args=(world, port, out), nprocs=world, join=True)
    exp = []
    for r in range(world):
        g = torch.Generator().manual_seed(200 + r)
        flat = torch.randn(127, generator=g)
        exp.append([flat[:120].view(40, 3), flat[120:127], torch.randn(16, generator=g),
                    torch.randn(5, 5, generator=g)])
    mean = [(a + b) / 2 for a, b in zip(*exp)]
    for r in range(world):
        for got, want in zip(out[r], mean):
            assert torch.allclose(got, want, atol=1e-6)


def test_complement_of_launched_regions():
    from mmdx.dist import _complement
    assert _complement([], 10) == [(0, 10)]
    assert _complement([(7, 10), (3, 7)], 10) == [(0, 3)]
    assert _complement([(2, 4), (6, 8)], 10) == [(0, 2), (4, 6), (8, 10)]
    assert _complement([(0, 10)], 10) == []


def _worker_bf16(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx.dist import GradAllReducer
    params = [torch.nn.Parameter(torch.zeros(s)) for s in SHAPES2]
    g = torch.Generator().manual_seed(300 + rank)
    for p in params:
        p.grad = torch.randn(p.shape, generator=g)
    red = GradAllReducer(params, world, bucket_bytes=64, bucket_dtype=torch.bfloat16)
    red.reduce()
    out[rank] = [p.grad.clone() for p in params]
    dist.destroy_process_group()


def test_grad_allreduce_bf16_buckets_gloo():
    """MMDX_DP_BUCKET_DTYPE=bf16: packed buckets travel in bf16; the fp32 mean is recovered
    to bf16 precision (rel 1e-2) and the grads stay fp32."""
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_bf16, args=(world, port, out), nprocs=world, join=True)
    exp = []
    for r in range(world):
        g = torch.Generator().manual_seed(300 + r)
        exp.append([torch.randn(s, generator=g) for s in SHAPES2])
    mean = [(a + b) / 2 for a, b in zip(*exp)]
    for r in range(world):
        for got, want in zip(out[r], mean):
            assert got.dtype == torch.float32
            assert (got - want).abs().max() <= 1e-2 * want.abs().max() + 1e-2


def test_whole_buffer_detection():
    """The arena test of GradAllReducer.launch: gradients that tile one whole storage (as
    detached views, the way autograd stores them) are one flat buffer; a gap, a foreign
    tensor, a dtype mix or a single tensor is not."""
    from mmdx.dist import _store_key, _whole_buffer
    buf = torch.arange(12.0)
    a, b = buf[:4].view(2, 2).detach(), buf[4:].detach()
    flat = _whole_buffer([a, b])
    assert flat is not None and flat.numel() == 12
    assert flat.untyped_storage().data_ptr() == buf.untyped_storage().data_ptr()
    flat.mul_(2)
    assert torch.equal(buf, torch.arange(12.0) * 2)
    assert _store_key(a) == _store_key(b)
    assert _whole_buffer([buf[:4], buf[6:]]) is None          # 2 elements uncovered
    assert _whole_buffer([a]) is None                          # a lone tensor: bucketed
    c = torch.zeros(12, dtype=torch.float64)
    assert _whole_buffer([c[:4], c[4:].float()]) is None       # not one storage / dtype


def _worker_stack(rank, world, port, out, sizes, regions):
    """A transformer stack's flat gradient buffer (xplan): the backward's segment hook
    (xplan.STACK_SEGMENT_HOOK -> GradAllReducer.trunk_segment) reduces each finished group of
    layers in place mid-backward, then launch() reduces the rest (layer 0's group) and the
    other gradients."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx.dist import GradAllReducer
    g = torch.Generator().manual_seed(500 + rank)
    flat = torch.randn(sum(sizes), generator=g)
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes] + \
        [torch.nn.Parameter(torch.zeros(9))]
    o = 0
    for p, n in zip(params, sizes):
        p.grad = flat[o:o + n].detach()
        o += n
    params[-1].grad = torch.randn(9, generator=g)
    red = GradAllReducer(params, world, bucket_bytes=64, small_arena_bytes=0)
    for lo, hi in regions:
        red.trunk_segment(flat, lo, hi)
    red.launch()
    stack = {id(p.grad) for p in params[:-1]}
    assert all(b is None or not stack & {id(g) for _, g in b} for b, *_ in red._pending)
    red.finish()
    out[rank] = [p.grad.clone() for p in params]
    dist.destroy_process_group()


def test_stack_segment_allreduce_gloo(monkeypatch):
    from mmdx import xplan
    from test_xplan_cpu import _small_vit_params
    monkeypatch.setattr(xplan, "SEG_LAYERS", 2)
    params = _small_vit_params(6)
    pl = xplan._build_vit(params, 2, 17, 64, 1, 128, 1e-6, torch.float16, torch.device("cpu"))
    assert len(pl.grad_regions) == 2
    sizes = [math.prod(sh) for _, sh, _ in sorted(pl.grads.items, key=lambda t: t[2])]
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_stack, args=(world, port, out, sizes, list(pl.grad_regions)),
             nprocs=world, join=True)
    exp = []
    for r in range(world):
        g = torch.Generator().manual_seed(500 + r)
        flat = torch.randn(sum(sizes), generator=g)
        exp.append(list(flat.split(sizes)) + [torch.randn(9, generator=g)])
    for r in range(world):
        for got, a, b in zip(out[r], exp[0], exp[1]):
            assert torch.allclose(got, (a + b) / 2, atol=1e-6)


SHAPES3 = ((16,), (5, 5), (60,))


def _worker_accum(rank, world, port, out, bf16):
    """Two reduces with ACCUMULATED gradients (zero_grad(set_to_none=False)): after the first,
    the packed gradients are views that tile the averaged bucket — a whole storage above
    small_arena_bytes — yet the second reduce must send them through the same packed bucket
    in the same dtype, not reduce that storage in place as an arena."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx.dist import GradAllReducer
    arena_p = [torch.nn.Parameter(torch.zeros(s)) for s in ((40, 3), (7,))]
    tens_p = [torch.nn.Parameter(torch.zeros(s)) for s in SHAPES3]
    params = arena_p + tens_p
    g = torch.Generator().manual_seed(600 + rank)
    flat = torch.randn(127, generator=g)
    arena_p[0].grad = flat[:120].view(40, 3).detach()
    arena_p[1].grad = flat[120:].detach()
    for p in tens_p:
        p.grad = torch.randn(p.shape, generator=g)
    red = GradAllReducer(params, world, small_arena_bytes=200,
                         bucket_dtype=torch.bfloat16 if bf16 else None)
    calls = []
    real = red._all_reduce
    red._all_reduce = lambda t, kind: (calls.append((kind, t.numel(), t.dtype)), real(t, kind))[1]
    red.reduce()
    first, calls[:] = list(calls), []
    for p in params:   # the second micro-step's gradients accumulate into the reduced ones
        p.grad.add_(torch.randn(p.shape, generator=g))
    red.reduce()
    out[rank] = {"calls": (first, list(calls)), "grads": [p.grad.clone() for p in params]}
    dist.destroy_process_group()


@pytest.mark.parametrize("bf16", [False, True])
def test_accumulated_grads_keep_bucket_path_gloo(bf16):
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_accum, args=(world, port, out, bf16), nprocs=world, join=True)
    bdt = torch.bfloat16 if bf16 else torch.float32
    want_calls = [("arena", 127, torch.float32), ("bucket[3]", 101, bdt)]
    first, second = out[0]["calls"]
    assert first == want_calls and second == want_calls, (first, second)
    draws = []
    for r in range(world):
        g = torch.Generator().manual_seed(600 + r)
        flat = torch.randn(127, generator=g)
        s1 = [flat[:120].view(40, 3), flat[120:]] + [torch.randn(s, generator=g) for s in SHAPES3]
        s2 = [torch.randn(t.shape, generator=g) for t in s1]
        draws.append((s1, s2))
    mean1 = [(a + b) / 2 for a, b in zip(draws[0][0], draws[1][0])]
    mean2 = [(m + (a + b) / 2) for m, a, b in zip(mean1, draws[0][1], draws[1][1])]
    tol = 2e-2 if bf16 else 1e-6
    for r in range(world):
        for got, want in zip(out[r]["grads"], mean2):
            assert got.dtype == torch.float32
            assert (got - want).abs().max() <= tol * max(1.0, want.abs().max())
