"""Backward scheduling for the two-tower train step (TP:1035/1056 `loss.backward()`).

The text tower runs on a side HIP stream concurrently with the image tower.
`two_tower_backward` computes the same gradients as `loss.backward()` in three engine
calls: the fusion head first (gradients of the two embeddings and of the fusion
parameters), then the image tower — its trunk backward is one native launch-plan call, so
the main stream (the critical path) is fed at once — then the text tower on its own
stream, whose host-side issue now overlaps the trunk's GPU work.  Every parameter's `.grad`
is identical to `loss.backward()`.
"""
from __future__ import annotations

import torch


def _tower(z: torch.Tensor) -> None:
    if z.requires_grad and z.grad is not None:
        g = z.grad
        z.backward(g)
        z.grad = None


def two_tower_backward(loss: torch.Tensor, z_img: torch.Tensor, z_txt: torch.Tensor,
                       head_params, text_stream=None, on_text_done=None) -> None:
    """`text_stream`: the stream the text tower's forward ran on.  Its backward is issued
    with that stream current, so the engine's end-of-backward stream sync does not make the
    image-trunk backward (current stream) wait for it; the current stream waits for the
    text stream only at the end, before the optimizer reads the gradients.
    `on_text_done()` is called with the text stream current once the text tower's and the
    fusion head's gradients are final (e.g. to start their data-parallel all-reduce while
    the image trunk is still in its backward)."""
    head = [p for p in head_params if p.requires_grad]
    inputs = [t for t in (z_img, z_txt) if t.requires_grad] + head
    loss.backward(inputs=inputs, retain_graph=True)
    if text_stream is None or not torch.cuda.is_available():
        _tower(z_img)
        _tower(z_txt)
        if on_text_done is not None:
            on_text_done()
        return
    main = torch.cuda.current_stream()
    text_stream.wait_stream(main)  # dL/dz_txt was produced on the current stream
    _tower(z_img)
    with torch.cuda.stream(text_stream):
        _tower(z_txt)
        if on_text_done is not None:
            on_text_done()
    main.wait_stream(text_stream)
