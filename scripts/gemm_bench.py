"""Time the bf16 implicit-GEMM kernels on the training step's shapes (SYN-48 batch).

python scripts/gemm_bench.py  (variants chosen by FS2_GEMM_OLD / FS2_GEMM_STAGES env vars)
"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")

dev = "cuda:0"
K.lib.fs2_set_tuning(7, int(os.environ.get("WGRAD_HALO", "0")))  # -1: tap-major weight gradient
# --lens: pass the SYN-48 utterance lengths, as the step does (all-padding row tiles skipped)
LENS = "--lens" in sys.argv
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
_b = PKG.data.syn_batch(48, 128, seed=0)
MEL_LENS = torch.tensor(_b[7], device=dev) if LENS else None
SRC_LENS = torch.tensor(_b[4], device=dev) if LENS else None


def lens_for(M):
    return None if not LENS else (MEL_LENS if M == 24576 else SRC_LENS)


SHAPES = [  # name, rows, T, cin, cout, taps
    ("dec conv1 k9 fwd", 24576, 512, 256, 1024, 9),
    ("dec conv1 k9 dX", 24576, 512, 1024, 256, 9),
    ("dec conv2 k1 fwd", 24576, 512, 1024, 256, 1),
    ("dec conv2 k1 dX", 24576, 512, 256, 1024, 1),
    ("dec qkv", 24576, 512, 256, 768, 1),
    ("dec fc", 24576, 512, 256, 256, 1),
    ("enc conv1 k9 fwd", 6144, 128, 256, 1024, 9),
    ("enc conv1 k9 dX", 6144, 128, 1024, 256, 9),
    ("postnet k5 512", 24576, 512, 512, 512, 5),
    ("postnet k5 80->512", 24576, 512, 80, 512, 5),
    ("vp k3", 6144, 128, 256, 256, 3),
]
tot = 0.0
for name, M, T, cin, cout, k in SHAPES:
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    w = torch.randn(cout * cin * k, device=dev).to(torch.bfloat16)
    b = torch.randn(cout, device=dev)
    aux = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    run = lambda: K.conv_gemm(x, w, M, T, cin, cout, k, (k - 1) // 2, bias=b, out=y,
                              flags=K.EPI_ADD_AUX | K.EPI_AUX_BF16, aux=aux, out_dtype=torch.bfloat16,
                              lens=lens_for(M))
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / n * 1e3
    tot += us
    print(f"{name:22s} {us:8.1f} us  {2 * M * cout * cin * k / us / 1e6:7.1f} TF/s")
print(f"total {tot:.1f} us")

WSHAPES = [  # weight-gradient shapes: name, rows, T, cin, cout, taps
    ("dec conv1 k9 dW", 24576, 512, 256, 1024, 9),
    ("dec conv2 k1 dW", 24576, 512, 1024, 256, 1),
    ("dec qkv dW", 24576, 512, 256, 768, 1),
    ("dec fc dW", 24576, 512, 256, 256, 1),
    ("enc conv1 k9 dW", 6144, 128, 256, 1024, 9),
    ("postnet k5 dW", 24576, 512, 512, 512, 5),
    ("vp k3 dW", 6144, 128, 256, 256, 3),
]
tot = 0.0
for name, M, T, cin, cout, k in WSHAPES:
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    dw = torch.zeros(cout, cin, k, device=dev)
    db = torch.zeros(cout, device=dev)
    run = lambda: K.conv_wgrad(dy, x, dw, M, T, cin, cout, k, (k - 1) // 2, db=db,
                               lens=lens_for(M))
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / n * 1e3
    tot += us
    print(f"{name:22s} {us:8.1f} us  {2 * M * cout * cin * k / us / 1e6:7.1f} TF/s")
print(f"wgrad total {tot:.1f} us")
