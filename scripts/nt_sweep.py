"""Sweep the fwd/dX GEMM tile-group knob (n-tiles per L2 group) and stages on the step's shapes."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
dev = "cuda:0"
STAGES, GROUP = 0, 5
SHAPES = [
    ("dec conv1 k9 fwd", 24576, 512, 256, 1024, 9),
    ("dec conv1 k9 dX", 24576, 512, 1024, 256, 9),
    ("dec conv2 k1 fwd", 24576, 512, 1024, 256, 1),
    ("dec conv2 k1 dX", 24576, 512, 256, 1024, 1),
    ("dec qkv", 24576, 512, 256, 768, 1),
    ("dec qkv dX", 24576, 512, 768, 256, 1),
    ("enc conv1 k9 fwd", 6144, 128, 256, 1024, 9),
    ("enc conv1 k9 dX", 6144, 128, 1024, 256, 9),
    ("postnet k5 512", 24576, 512, 512, 512, 5),
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


for name, M, T, cin, cout, k in SHAPES:
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout * cin * k, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(cout, device=dev)
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    run = lambda: K.conv_gemm(x, w, M, T, cin, cout, k, (k - 1) // 2, bias=b, out=y,
                              flags=K.EPI_RELU, out_dtype=torch.bfloat16)
    res = []
    for st in (0, 1, 2, 3, 4):
        for g in (0,):
            K.lib.fs2_set_tuning(STAGES, st)
            K.lib.fs2_set_tuning(GROUP, g)
            res.append((timeit(run), st, g))
    K.lib.fs2_set_tuning(STAGES, 0)
    K.lib.fs2_set_tuning(GROUP, 0)
    auto = res[0]
    fl = 2 * M * cout * cin * k
    print(f"{name:18s} auto {auto[0]:7.1f}us ({fl / auto[0] / 1e6:5.0f} TF) | best " +
          "  ".join(f"{t:7.1f}us st{s} g{g}" for t, s, g in sorted(res)[:4]), flush=True)
