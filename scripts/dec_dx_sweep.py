"""Decoder FFN k=9 data gradient (Conv1d 1024 -> 256 over 48 x 512 frames, ADD_AUX, mel lens)
under the halo variants (FS2_TUNE_NT_HALO) and forced channel-block splits.
``--fwd``: the forward instead (Conv1d 256 -> 1024, bias + ReLU, bf16 out), the bench's
roofline launch."""
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
lens = torch.tensor(_b[7], device=dev)
FWD = "--fwd" in sys.argv
B, T, cin, cout, k = (48, 512, 256, 1024, 9) if FWD else (48, 512, 1024, 256, 9)
M = B * T
x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
w = torch.randn(cout, cin, k, device=dev) / math.sqrt(cin * k)
wf = torch.empty(cout * cin * k, device=dev, dtype=torch.bfloat16)
wb = torch.empty_like(wf)
K.weight_prep(w, cout, cin, k, wf, wb)
aux = torch.randn(M, cout, device=dev)
out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16 if FWD else torch.float32)
bias = torch.randn(cout, device=dev)
if FWD:
    run = lambda: K.conv_gemm(x, wf, M, T, cin, cout, k, 4, bias=bias, flags=K.EPI_RELU, out=out,
                              lens=lens)
else:
    run = lambda: K.conv_gemm(x, wf, M, T, cin, cout, k, 4, flags=K.EPI_ADD_AUX, aux=aux, out=out,
                              lens=lens)
valid = int(lens.sum())
for _ in range(400):  # clocks settle (the first ~0.3 s of launches run slow)
    run()
torch.cuda.synchronize()
ref = None
CONFIGS = ((0, 0, "auto"), (1, 0, "4-wave"), (4, 0, "3-slot"), (5, 0, "8w 256x128 3s"),
           (6, 0, "8w 128x128 3s"), (7, 0, "8w 256x128 2s"), (2, 0, "128x128"))
if not FWD:
    CONFIGS += ((0, 2, "128x64 kz2"), (0, 4, "128x64 kz4"), (2, 2, "128x128 kz2"),
                (2, 3, "128x128 kz3"), (2, 4, "128x128 kz4"))
DB = [0]
if "--db" in sys.argv:  # FS2_TUNE_HALO_DB: double-buffered halo stage on / off
    CONFIGS = tuple((0, 0, f"auto db {d_}", 0, d_) for d_ in (0, -1))
elif "--group" in sys.argv:  # FS2_TUNE_NT_GROUP: n-tiles per tile group (weight slice per XCD)
    CONFIGS = tuple((0, 0, f"auto group {g_}", g_, 0) for g_ in (0, 1, 2, 4))
else:
    CONFIGS = tuple(c + (0, 0) for c in CONFIGS)
for nt, sk, name, grp, db in CONFIGS + CONFIGS + CONFIGS:
    K.lib.fs2_set_tuning(6, nt)
    K.lib.fs2_set_tuning(8, sk)
    K.lib.fs2_set_tuning(5, grp)
    K.lib.fs2_set_tuning(10, db)
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(30):
        run()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 30 * 1e3
    keep = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
    if ref is None:
        ref = out[keep].clone()
    err = (out[keep].float() - ref.float()).abs().max().item()
    print(f"{name:16s} {us:7.1f} us  {2 * valid * cin * cout * k / us / 1e6:6.0f} TFLOP/s (valid)"
          f"  max|diff| {err:.2e}", flush=True)
K.lib.fs2_set_tuning(6, 0)
K.lib.fs2_set_tuning(8, 0)
K.lib.fs2_set_tuning(5, 0)
K.lib.fs2_set_tuning(10, 0)
