"""Time mmdx_lstm_bwd (recurrence + dW_hh GEMMs) at the C4 shape, B=128 L=128 H=256 bf16.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.  MMDX_LIB_PATH picks a
variant build."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mmdx
from mmdx import _lib as L

B, Ls, H = 128, 128, 256
G4 = 4 * H
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
whh = (torch.randn(2 * G4, H, device=dev, generator=g) * 0.05).bfloat16()
hout = torch.randn(B, Ls, 2 * H, device=dev, generator=g).bfloat16()
cs = torch.randn(2, Ls, B, H, device=dev, generator=g)
gs = torch.rand(2, Ls, B, G4, device=dev, generator=g)
dh = torch.randn(B, Ls, 2 * H, device=dev, generator=g).bfloat16()
dxg = torch.empty(B, Ls, 2, G4, device=dev, dtype=torch.bfloat16)
dw = torch.empty(2 * G4 * H, device=dev)
wsn = L.lib().mmdx_lstm_workspace_size(1, B, Ls, H)
ws = torch.empty(wsn, dtype=torch.uint8, device=dev)
def run():
    L.call("mmdx_lstm_bwd", 1, L.ptr(whh), L.ptr(hout), L.ptr(cs), L.ptr(gs), L.ptr(dh), B, Ls, H,
           L.ptr(dxg), L.ptr(dw), L.ptr(ws), wsn, None, 0, 0, L.stream())
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    run()
e1.record()
torch.cuda.synchronize()
print(f"{os.environ.get('MMDX_LIB_PATH', 'default')}: mmdx_lstm_bwd {e0.elapsed_time(e1) / 10:.3f} ms")
