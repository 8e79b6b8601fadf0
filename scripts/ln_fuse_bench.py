"""fs2_conv_gemm_ln (GEMM + LayerNorm epilogue) vs fs2_conv_gemm + fs2_ln_fwd on the FFT blocks'
fc (K = 256) and w_2 (K = 1024) shapes at SYN-48 lengths, dropout on (p = 0.2).
    python scripts/ln_fuse_bench.py"""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
_b = PKG.data.syn_batch(48, 128, seed=0)
LENS = {512: torch.tensor(_b[7], device=dev), 128: torch.tensor(_b[4], device=dev)}
bf = torch.bfloat16


def timeit(run, reps=20):
    best = 1e9
    for _ in range(3):
        for _ in range(5):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            run()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1e3)
    return best


tot = {}
for name, T, cin, cnt in (("dec fc+ln1", 512, 256, 6), ("dec w2+ln2", 512, 1024, 6),
                          ("enc fc+ln1", 128, 256, 4), ("enc w2+ln2", 128, 1024, 4)):
    M, d = 48 * T, 256
    lens = LENS[T]
    x = torch.randn(M, cin, device=dev).to(bf)
    wf = (torch.randn(d, cin, device=dev) * 0.05).to(bf)
    b, res = torch.randn(d, device=dev), torch.randn(M, d, device=dev)
    g, bt = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    kw = dict(lens=lens, p_in=0.2, seed=torch.tensor([7], dtype=torch.int64, device=dev), site_in=3)

    def two():
        y = K.conv_gemm(x, wf, M, T, cin, d, 1, 0, bias=b, lens=lens)
        K.ln_fwd(y, g, bt, res=res, seq_len=T, copy=bf, **kw)

    row = [timeit(two)]
    for tile in (0, 1):
        K.lib.fs2_set_tuning(11, tile)
        row.append(timeit(lambda: K.conv_gemm_ln(x, wf, M, T, cin, d, 1, 0, g, bt, bias=b, res=res, **kw)))
        K.lib.fs2_set_tuning(11, 0)
    for i, t in enumerate(row):
        tot[i] = tot.get(i, 0.0) + cnt * t
    print(f"{name:12s} gemm+ln_fwd {row[0]:6.1f} us   fused 64x256 {row[1]:6.1f} us   "
          f"fused 128x256 {row[2]:6.1f} us", flush=True)
print(f"per step: two launches {tot[0]:.0f} us, fused 64x256 {tot[1]:.0f} us, 128x256 {tot[2]:.0f} us")
