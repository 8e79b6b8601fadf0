"""LayerNorm forward/backward in isolation at the decoder's SYN-48 shape (lens as the step
passes them), with and without dropout, and effective bandwidth over the valid rows."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
_b = PKG.data.syn_batch(48, 128, seed=0)
lens = torch.tensor(_b[7], device=dev)
M, T, d = 24576, 512, 256
V = int(lens.sum())


def timeit(run, n=50):
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


y, r = torch.randn(M, d, device=dev), torch.randn(M, d, device=dev)
g, b = torch.ones(d, device=dev), torch.zeros(d, device=dev)
SEED = torch.tensor([1], dtype=torch.int64, device=dev)  # device key, as the step passes it
for p in (0.0, 0.2):
    t = timeit(lambda: K.ln_fwd(y, g, b, res=r, lens=lens, seq_len=T, p_in=p, seed=SEED, site_in=3,
                                copy=torch.bfloat16))
    byt = V * d * (4 + 4 + 4 + 4 + 2) + (M - V) * d * 10
    print(f"ln_fwd  p={p}: {t:7.1f} us  {byt / t / 1e3:7.0f} GB/s", flush=True)
    out, out_t, xh, rs, _ = K.ln_fwd(y, g, b, res=r, lens=lens, seq_len=T, p_in=p, seed=SEED,
                                     site_in=3, copy=torch.bfloat16)
    dg, db, dbi = (torch.zeros(d, device=dev) for _ in range(3))
    dx2 = torch.randn(M, d, device=dev)
    dres = torch.empty(M, d, device=dev)
    run = lambda: K.ln_bwd(xh, rs, g, b, dg, db, dout=dx2, lens=lens, seq_len=T, p_in=p, seed=SEED,
                           site_in=3, dres=dres, dres_add=False, copy=torch.bfloat16,
                           dbias_in=dbi)
    t = timeit(run)
    byt = V * d * (4 + 4 + 4 + 2) + (M - V) * d * 6
    print(f"ln_bwd  p={p}: {t:7.1f} us  {byt / t / 1e3:7.0f} GB/s", flush=True)
    run = lambda: K.ln_bwd(xh, rs, g, b, dg, db, dout=dx2, lens=lens, seq_len=T, p_in=p, seed=SEED,
                           site_in=3, dres=dres, dres_add=True, copy=torch.bfloat16,
                           dbias_in=dbi)
    t = timeit(run)
    byt = V * d * (4 + 4 + 8 + 2) + (M - V) * d * 6
    print(f"ln_bwd+ p={p}: {t:7.1f} us  {byt / t / 1e3:7.0f} GB/s  (dres +=)", flush=True)
