"""Cross-XCD visibility of a kernel's writes to the next kernel on the same stream
(fs2_debug_coherence): stale-line counts per size.  python scripts/coherence_probe.py"""
import importlib
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = importlib.import_module("mid-attribute-speaker-generation_amd._lib").lib
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
for n in (64, 1024, 65536, 1 << 20):
    x = torch.zeros(n, dtype=torch.int32, device="cuda")
    blocks = 2048
    bad = torch.zeros(blocks + 1, dtype=torch.int32, device="cuda")
    lib.fs2_debug_coherence(x.data_ptr(), n, 50, blocks, bad.data_ptr(), K.stream())
    torch.cuda.synchronize()
    b = bad[:blocks].cpu()
    print(f"n={n}: stale elements seen {int(b.sum())} in {int((b > 0).sum())} of {blocks} blocks "
          f"(50 rounds)", flush=True)
