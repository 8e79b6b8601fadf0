"""Halo conv GEMM vs the tap-major kernel: agreement (fp32 outputs) and time, step shapes."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
_b = PKG.data.syn_batch(48, 128, seed=0)
MEL, SRC = torch.tensor(_b[7], device=dev), torch.tensor(_b[4], device=dev)
SHAPES = [  # name, rows, T, cin, cout, taps, lens
    ("dec k9 fwd", 24576, 512, 256, 1024, 9, MEL),
    ("dec k9 dX", 24576, 512, 1024, 256, 9, MEL),
    ("enc k9 fwd", 6144, 128, 256, 1024, 9, SRC),
    ("enc k9 dX", 6144, 128, 1024, 256, 9, SRC),
    ("postnet k5 512", 24576, 512, 512, 512, 5, None),
    ("postnet k5 512->80", 24576, 512, 512, 80, 5, None),
    ("vp k3", 6144, 128, 256, 256, 3, None),
    ("odd T k9 (fallback)", 4 * 300, 300, 256, 1024, 9, None),
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


for name, M, T, cin, cout, k, lens in SHAPES:
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout * cin * k, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(cout, device=dev)
    res = {}
    for mode in (-1, 3, 0, 4, 5, 6, 7):
        K.lib.fs2_set_tuning(6, mode)
        run = lambda: K.conv_gemm(x, w, M, T, cin, cout, k, (k - 1) // 2, bias=b, lens=lens)
        y = run()
        res[mode] = (y.clone(), timeit(run))
    K.lib.fs2_set_tuning(6, 0)
    (y0, t0), (y1, t1), (y3, t3), (y4, t4) = res[-1], res[0], res[3], res[4]
    errs = {md: ((res[md][0] - y1).abs().max() / y1.abs().max()).item() for md in (5, 6, 7)}
    print(f"    8-wave: 256x128/3 {res[5][1]:7.1f}us  128x128/3 {res[6][1]:7.1f}us  "
          f"256x128/2 {res[7][1]:7.1f}us  max rel diff vs default {errs}")
    # same tiles, same order: bitwise equal (128-row and 256-row tilings differ only in the
    # padded rows of partially valid tiles, which the 256-row kernels compute)
    assert torch.equal(y3, y4), name
    assert torch.equal(res[5][0], res[7][0]), name
    # torch fp32 reference on the same bf16 operands (per-utterance zero padding)
    W = w.float().view(cout, k, cin).permute(0, 2, 1)
    B_ = M // T
    yr = torch.nn.functional.conv1d(x.float().view(B_, T, cin).transpose(1, 2), W, b,
                                    padding=(k - 1) // 2).transpose(1, 2).reshape(M, cout)
    if lens is not None:  # compare valid rows (padded rows: skipped tiles or computed)
        keep = torch.cat([torch.arange(T, device=dev) < int(lens[u]) for u in range(B_)])
        y0, y1, yr = y0[keep], y1[keep], yr[keep]
    e0 = ((y0 - yr).abs().max() / yr.abs().max()).item()
    e1 = ((y1 - yr).abs().max() / yr.abs().max()).item()
    print(f"    vs torch: tap-major {e0:.1e} halo {e1:.1e}")
    err = ((y1 - y0).abs().max() / y0.abs().max()).item()
    fl = 2 * M * cout * cin * k
    print(f"{name:22s} tap-major {t0:7.1f}us {fl / t0 / 1e6:5.0f}TF | halo-1 {t3:7.1f}us "
          f"{fl / t3 / 1e6:5.0f}TF | halo-3 {t4:7.1f}us {fl / t4 / 1e6:5.0f}TF | halo {t1:7.1f}us "
          f"{fl / t1 / 1e6:5.0f}TF | rel err {err:.1e}", flush=True)
    assert e1 < 1e-5, name
