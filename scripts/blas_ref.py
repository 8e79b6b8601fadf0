"""hipBLASLt (torch.matmul, bf16) on the step's GEMM shapes: what a vendor GEMM reaches on the
same M x N x K (the conv kernels' shapes as plain GEMMs; no im2col counted)."""
import torch

dev = "cuda"
SHAPES = [("dec qkv fwd", 24576, 768, 256), ("dec fc fwd", 24576, 256, 256),
          ("dec w2 fwd", 24576, 256, 1024), ("dec w2 dgrad", 24576, 1024, 256),
          ("dec qkv dgrad", 24576, 256, 768), ("dec k9 fwd", 24576, 1024, 2304),
          ("dec k9 dgrad", 24576, 256, 9216), ("postnet k5", 24576, 512, 2560),
          ("dec k9 wgrad", 1024, 2304, 24576)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(K, N, device=dev).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(10):
        torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            torch.matmul(a, b, out=c)
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / 20 * 1e3)
    fl = 2.0 * M * N * K
    print(f"{name:14s} M={M:6d} N={N:5d} K={K:6d}  {best:7.1f} us  {fl / best / 1e6:7.0f} TF/s", flush=True)
