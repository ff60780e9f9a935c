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

import concurrent.futures
import os
import threading

import torch

from .trace import rng

# MMDX_TEXT_BWD_FIRST=1: issue the text tower's backward before the image trunk's (A/B)
TEXT_BWD_FIRST = os.environ.get("MMDX_TEXT_BWD_FIRST", "0") == "1"


class TwoTowerForward:
    """Issue the two encoder towers' forwards (TP:1000-1007 `image_encoder.encode` /
    `text_encoder.encode`) from two host threads at once.

    The image tower's host side is one native launch-plan call (the GIL is released while
    it enqueues), the text tower's is a sequence of Python-issued ops; on one thread one of
    them always starts late on the GPU by the other's issue time.  Here the text tower is
    issued by a persistent worker thread onto `text_stream` while the calling thread issues
    the image tower onto the current stream; both return their usual autograd outputs.
    `__call__(image_fn, text_fn)` -> (image_fn(), text_fn()).  The caller makes the current
    stream wait for `text_stream` before consuming the text output."""

    def __init__(self, text_stream=None):
        self.text_stream = text_stream
        self._pool = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="mmdx-text")
        self._lock = threading.Lock()

    def _text(self, fn, device, grad):
        with torch.set_grad_enabled(grad), rng("mmdx/text_fwd"):
            if self.text_stream is None:
                return fn()
            torch.cuda.set_device(device)
            with torch.cuda.stream(self.text_stream):
                return fn()

    def __call__(self, image_fn, text_fn):
        with self._lock:  # one step in flight per instance
            dev = torch.cuda.current_device() if self.text_stream is not None else None
            fut = self._pool.submit(self._text, text_fn, dev, torch.is_grad_enabled())
            try:
                with rng("mmdx/image_fwd"):
                    z_img = image_fn()
            finally:
                z_txt = fut.result()
            return z_img, z_txt

    def close(self):
        self._pool.shutdown(wait=True)


def _tower(z: torch.Tensor) -> None:
    if z.requires_grad and z.grad is not None:
        g = z.grad
        z.backward(g)
        z.grad = None


def two_tower_backward(loss: torch.Tensor, z_img: torch.Tensor, z_txt: torch.Tensor,
                       head_params, text_stream=None, on_text_done=None, mark=None) -> None:
    """`text_stream`: the stream the text tower's forward ran on.  Its backward is issued
    with that stream current, so the engine's end-of-backward stream sync does not make the
    image-trunk backward (current stream) wait for it; the current stream waits for the
    text stream only at the end, before the optimizer reads the gradients.
    `on_text_done()` is called with the text stream current once the text tower's and the
    fusion head's gradients are final (e.g. to start their data-parallel all-reduce while
    the image trunk is still in its backward).  `mark(name, stream)` (optional, diagnostics):
    called once each part is issued, with the stream that part runs on."""
    head = [p for p in head_params if p.requires_grad]
    inputs = [t for t in (z_img, z_txt) if t.requires_grad] + head
    with rng("mmdx/head_bwd"):
        loss.backward(inputs=inputs, retain_graph=True)
    if mark is not None:
        mark("head_bwd", torch.cuda.current_stream())
    if text_stream is None or not torch.cuda.is_available():
        with rng("mmdx/image_bwd"):
            _tower(z_img)
        with rng("mmdx/text_bwd"):
            _tower(z_txt)
        if on_text_done is not None:
            on_text_done()
        return
    main = torch.cuda.current_stream()
    text_stream.wait_stream(main)  # dL/dz_txt was produced on the current stream

    def text():
        with torch.cuda.stream(text_stream):
            with rng("mmdx/text_bwd"):
                _tower(z_txt)
            if mark is not None:
                mark("text_bwd", text_stream)
            if on_text_done is not None:
                on_text_done()
    if TEXT_BWD_FIRST:
        text()
    with rng("mmdx/image_bwd"):
        _tower(z_img)
    if mark is not None:
        mark("image_bwd", main)
    if not TEXT_BWD_FIRST:
        text()
    main.wait_stream(text_stream)
