"""Timing of the decoder k=9 GEMMs with and without padding-tile skipping (SYN-48 lengths)."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
dev = "cuda:0"
b = PKG.data.syn_batch(48, 128, seed=0)
lens = torch.tensor(np.asarray(b[7]), device=dev)
M, T = 48 * 512, 512


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


for cin, cout, k in ((256, 1024, 9), (1024, 256, 9), (1024, 256, 1), (256, 768, 1)):
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout * cin * k, device=dev) * 0.02).to(torch.bfloat16)
    for L in (None, lens):
        t = timeit(lambda: K.conv_gemm(x, w, M, T, cin, cout, k, (k - 1) // 2, lens=L,
                                       out_dtype=torch.bfloat16))
        dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
        dw = torch.zeros(cout, cin, k, device=dev)
        tw = timeit(lambda: K.conv_wgrad(dy, x, dw, M, T, cin, cout, k, (k - 1) // 2, lens=L))
        print(f"{cin}->{cout} k{k} lens={'y' if L is not None else 'n'}: fwd {t:7.1f} us, "
              f"wgrad {tw:7.1f} us", flush=True)
