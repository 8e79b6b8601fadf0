"""Time the FFT block's three k = 1 weight gradients (QKV + bias, fc, w_2) at SYN-48 shapes:
three fs2_conv_wgrad launches (+ their split reduces) against one fs2_conv_wgrad_k1_multi
(grouped launch + one reduce), alone and beside a k = 9 data gradient on the main stream.

    python scripts/k1_multi_bench.py [--reps 20] [--probe]

--probe: 10 grouped launches at the decoder shape only (for rocprofv3 --pmc passes).
"""
import importlib
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
bf = torch.bfloat16
_b = PKG.data.syn_batch(48, 128, seed=0)
LENS = {512: torch.tensor(_b[7], device=dev), 128: torch.tensor(_b[4], device=dev)}
VALID = {512: int(np.sum(_b[7])), 128: int(np.sum(_b[4]))}


def timeit(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 20
    probe = "--probe" in sys.argv
    for T in ((512,) if probe else (512, 128)):
        M = 48 * T
        lens = LENS[T]
        valid = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
        jobs = []
        fl = 0.0
        for cin, cout, bias in ((256, 768, True), (256, 256, False), (1024, 256, False)):
            x = (torch.randn(M, cin, device=dev) * valid[:, None]).to(bf)
            dy = (torch.randn(M, cout, device=dev) * valid[:, None]).to(bf)
            jobs.append((dy, x, torch.zeros(cout, cin, device=dev),
                         torch.zeros(cout, device=dev) if bias else None, cin, cout))
            fl += 2.0 * VALID[T] * cin * cout / 1e6
        wsb = K.ws(max(K.lib.fs2_conv_wgrad_ws_bytes(M, cin, cout, 1) for _, _, _, _, cin, cout in jobs), dev)
        wsm = K.ws(K.conv_wgrad_k1_multi_ws_bytes(jobs, M), dev)

        def sep():
            for dy, x, dw, db, cin, cout in jobs:
                K.conv_wgrad(dy, x, dw, M, T, cin, cout, 1, 0, db=db, ws_buf=wsb, lens=lens)

        def grp():
            K.conv_wgrad_k1_multi(jobs, M, T, lens=lens, ws_buf=wsm)

        if probe:
            for _ in range(10):
                grp()
            torch.cuda.synchronize()
            return
        t_s, t_g = [], []
        for _ in range(3):
            t_s.append(timeit(sep, reps))
            t_g.append(timeit(grp, reps))
        hbm = sum((dy.numel() + x.numel()) * 2 for dy, x, *_ in jobs) / 1e6
        print(f"T={T}: three launches {min(t_s):6.1f} us ({fl / min(t_s):4.0f} TF/s)  grouped "
              f"{min(t_g):6.1f} us ({fl / min(t_g):4.0f} TF/s, {hbm / min(t_g):.2f} TB/s of the "
              f"{hbm:.0f} MB operands)", flush=True)


if __name__ == "__main__":
    main()
