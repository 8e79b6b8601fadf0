"""Launch one weight-gradient shape of the step 10 times (SYN-48 lengths), for PMC passes:

    bash scripts/pmc_kernel.sh wgrad python3 scripts/wgrad_probe.py <shape>

shapes: dec_qkv, dec_fc, dec_w2 (k = 1, tap-major kernel + wgrad_reduce_k1), dec_k9 (halo
kernel + wgrad_reduce_taps)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
SHAPES = {"dec_qkv": (512, 256, 768, 1, True), "dec_fc": (512, 256, 256, 1, False),
          "dec_w2": (512, 1024, 256, 1, False), "dec_k9": (512, 256, 1024, 9, True)}


def main():
    T, cin, cout, k, bias = SHAPES[sys.argv[1]]
    dev = "cuda:0"
    b = PKG.data.syn_batch(48, 128, seed=0)
    lens = torch.tensor(b[7] if T == 512 else b[4], device=dev)
    M = 48 * T
    valid = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
    x = (torch.randn(M, cin, device=dev) * valid[:, None]).to(torch.bfloat16)
    dy = (torch.randn(M, cout, device=dev) * valid[:, None]).to(torch.bfloat16)
    dw = torch.zeros(cout, cin, k, device=dev)
    db = torch.zeros(cout, device=dev) if bias else None
    for _ in range(10):
        K.conv_wgrad(dy, x, dw, M, T, cin, cout, k, (k - 1) // 2, db=db, lens=lens)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
