"""Which hipBLASLt kernels torch.matmul picks for the R50 conv GEMM shapes (run under
rocprofv3 --kernel-trace; the Tensile kernel names carry macro tile, MFMA shape, depth-U,
global split-U and workgroup mapping)."""
import torch
shapes = [(6272, 512, 4608), (6272, 2048, 512), (6272, 512, 2048), (25088, 256, 2304),
          (25088, 1024, 256), (25088, 256, 1024), (25088, 512, 1024), (100352, 256, 512),
          (100352, 512, 256), (401408, 256, 64)]
dev = torch.device("cuda", 0)
for M, N, K in shapes:
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    for _ in range(5):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
