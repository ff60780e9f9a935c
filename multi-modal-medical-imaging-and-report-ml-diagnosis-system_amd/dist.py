"""Data parallelism for the multimodal train step (new capability; the reference is a
single CPU process).

One process per GPU; the (image, report) minibatch is sharded across ranks (weak scaling),
every rank holds a full replica, and the only exchange per step is the gradient
all-reduce: fp32 gradients are packed into ~64 MB buckets and reduced with
`torch.distributed.all_reduce` — RCCL over xGMI with the "nccl" backend on ROCm, gloo in
the CPU tests — then averaged.  Buckets are launched as soon as backward has produced
them: each bucket's all-reduce runs asynchronously (work handles) so RCCL moves bucket i
while the next is packed; `finish()` waits and scatters the averaged gradients back.
BatchNorm keeps per-replica batch statistics (DDP semantics, no SyncBN); clip_grad_norm_
runs after the all-reduce, so every rank clips identically.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

BUCKET_BYTES = 64 << 20


class GradAllReducer:
    def __init__(self, params, world_size: int | None = None, bucket_bytes: int = BUCKET_BYTES,
                 group=None):
        self.params = [p for p in params if p.requires_grad]
        self.world = world_size or dist.get_world_size(group)
        self.bucket_bytes = bucket_bytes
        self.group = group
        self._plan_key = None
        self._plan = None
        self._flat = None

    def _make_plan(self, grads):
        plan, cur, size = [], [], 0
        # reverse parameter order ~ order in which backward produces the gradients
        for g in reversed(grads):
            cur.append(g)
            size += g.numel() * g.element_size()
            if size >= self.bucket_bytes:
                plan.append(cur)
                cur, size = [], 0
        if cur:
            plan.append(cur)
        return plan

    def reduce(self):
        """All-reduce (mean) every existing .grad across ranks, in place."""
        grads = [p.grad for p in self.params if p.grad is not None]
        if not grads or self.world == 1:
            return
        key = tuple(g.data_ptr() for g in grads)
        if key != self._plan_key:
            self._plan = self._make_plan(grads)
            self._plan_key = key
        pending = []
        for bucket in self._plan:
            flat = torch._utils._flatten_dense_tensors(bucket)
            work = dist.all_reduce(flat, group=self.group, async_op=True)
            pending.append((bucket, flat, work))
        inv = 1.0 / self.world
        for bucket, flat, work in pending:
            work.wait()
            flat.mul_(inv)
            for g, s in zip(bucket, torch._utils._unflatten_dense_tensors(flat, bucket)):
                g.copy_(s)


def shard_batch(batch_size: int, rank: int, world: int):
    """Contiguous [start, stop) of the global batch owned by `rank` (global batch must
    divide evenly: C4 = 1024 over 8 ranks = 128 each)."""
    if batch_size % world:
        raise ValueError(f"global batch {batch_size} not divisible by world size {world}")
    per = batch_size // world
    return rank * per, (rank + 1) * per
