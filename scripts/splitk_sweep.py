"""Encoder k=9 data gradient (Conv1d 1024 -> 256 over 48 x 128 frames, ADD_AUX epilogue, lens)
under the halo split-K knob: off, 64x64 split, 128x64 split with 2 / 4 / 6 splits."""
import importlib
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
_b = PKG.data.syn_batch(48, 128, seed=0)
lens = torch.tensor(_b[4], device=dev)
B, T, cin, cout, k = 48, 128, 1024, 256, 9
M = B * T
x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
w = torch.randn(cout, cin, k, device=dev) / math.sqrt(cin * k)
wf = torch.empty(cout * cin * k, device=dev, dtype=torch.bfloat16)
wb = torch.empty_like(wf)
K.weight_prep(w, cout, cin, k, wf, wb)
aux = torch.randn(M, cout, device=dev)
out = torch.empty(M, cout, device=dev)
run = lambda: K.conv_gemm(x, wf, M, T, cin, cout, k, 4, flags=K.EPI_ADD_AUX, aux=aux, out=out,
                          lens=lens)
valid = int(lens.sum())
for knob, name in ((-1, "off"), (-2, "64x64 auto"), (0, "auto"), (2, "128x64 kz2"),
                   (4, "128x64 kz4"), (6, "kz6")):
    K.lib.fs2_set_tuning(8, knob)
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(30):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 30 * 1e3
    print(f"{name:12s} {us:7.1f} us  {2 * valid * cin * cout * k / us / 1e6:6.0f} TFLOP/s (valid)",
          flush=True)
K.lib.fs2_set_tuning(8, 0)
