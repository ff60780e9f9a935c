"""CPU: the DP gradient all-reduce (mmdx.dist.GradAllReducer) over gloo, world_size 2."""
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


def _worker_flat(rank, world, port, out, region=False):
    """Gradients that are views of one flat buffer (the trunk's gradient arena) are reduced
    in place; the others through buckets; a subset is launched early (overlap path)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mmdx.dist import GradAllReducer
    params = [torch.nn.Parameter(torch.zeros(s)) for s in SHAPES2]
    g = torch.Generator().manual_seed(200 + rank)
    flat = torch.randn(40 * 3 + 7, generator=g)
    params[0].grad = flat[:120].view(40, 3)
    params[1].grad = flat[120:127]
    params[2].grad = torch.randn(16, generator=g)
    params[3].grad = torch.randn(5, 5, generator=g)
    red = GradAllReducer(params, world, bucket_bytes=64)
    if region:  # the buffer's tail first (the trunk's last layer, resnet.TRUNK_GRAD_HOOK)
        red.launch_region(flat, 100, flat.numel())
    red.launch([params[2]])
    red.reduce()
    assert params[0].grad._base is flat  # reduced in place, still the same buffer
    out[rank] = [p.grad.clone() for p in params]
    dist.destroy_process_group()


@pytest.mark.parametrize("region", [False, True])
def test_grad_allreduce_flat_base_and_early_launch_gloo(region):
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_flat, args=(world, port, out, region), nprocs=world, join=True)
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
