"""Sweep the large-grid fwd/dX tile (FS2_TUNE_NT_BIG) x LDS stages on the step's shapes."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
_b = PKG.data.syn_batch(48, 128, seed=0)
LENS = torch.tensor(_b[7], device=dev)
SHAPES = [
    ("dec conv1 k9 fwd", 24576, 512, 256, 1024, 9, K.EPI_RELU),
    ("dec conv2 k1 dX", 24576, 512, 256, 1024, 1, 0),
    ("dec qkv", 24576, 512, 256, 768, 1, 0),
    ("postnet k5 512", 24576, 512, 512, 512, 5, 0),
]


def timeit(run, n=20):
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for name, M, T, cin, cout, k, fl in SHAPES:
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout * cin * k, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(cout, device=dev)
    ref = None
    line = []
    for big in (0, 1, 2):
        for st in (1, 2):
            K.lib.fs2_set_tuning(6, big)
            K.lib.fs2_set_tuning(0, st)
            y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
            run = lambda: K.conv_gemm(x, w, M, T, cin, cout, k, (k - 1) // 2, bias=b, out=y,
                                      flags=fl, out_dtype=torch.bfloat16, lens=LENS)
            us = timeit(run)
            if ref is None:
                ref = y.float().clone()
            err = (y.float() - ref).abs().max().item()
            line.append(f"big{big}/s{st} {us:6.1f}us {2 * M * cout * cin * k / us / 1e6:6.0f}TF"
                        + ("" if err == 0 else f" ERR{err:.2e}"))
    print(f"{name:18s} " + " | ".join(line), flush=True)
K.lib.fs2_set_tuning(6, 0)
K.lib.fs2_set_tuning(0, 0)
