"""Time the bf16 attention kernels on the decoder/encoder shapes with SYN-48 lengths."""
import importlib
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
dev = "cuda:0"
for kv in filter(None, os.environ.get("FS2_TUNE", "").split(",")):  # knob=value A/B
    K.lib.fs2_set_tuning(int(kv.split("=")[0]), int(kv.split("=")[1]))
b = PKG.data.syn_batch(48, 128, seed=0)


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


if "--probe" in sys.argv:  # PMC passes: 10 decoder-shaped forward + backward launches
    B, T, H, dh = 48, 512, 2, 128
    L = torch.tensor(np.asarray(b[7]), device=dev)
    qkv = (torch.randn(B * T, 3 * H * dh, device=dev) * 0.5).to(torch.bfloat16)
    o, lse = K.attn_fwd(qkv, L, B, T, H, dh, 1 / math.sqrt(dh))
    do = torch.randn(B * T, H * dh, device=dev).to(torch.bfloat16)
    for _ in range(10):
        K.attn_fwd(qkv, L, B, T, H, dh, 1 / math.sqrt(dh))
        K.attn_bwd(qkv, o, do, lse, L, B, T, H, dh, 1 / math.sqrt(dh))
    torch.cuda.synchronize()
    sys.exit(0)

for knob in ((0, 1, 2, 3, 0, 2) if "--variants" in sys.argv else tuple(int(v) for v in sys.argv[sys.argv.index("--knobs") + 1].split(",")) if "--knobs" in sys.argv else (0,)):
  K.lib.fs2_set_tuning(9, knob)  # FS2_TUNE_ATTN
  print(f"== FS2_TUNE_ATTN = {knob}")
  for name, T, lens in (("decoder", 512, np.asarray(b[7])), ("encoder", 128, np.asarray(b[4]))):
      B, H, dh = 48, 2, 128
      L = torch.tensor(lens, device=dev)
      qkv = (torch.randn(B * T, 3 * H * dh, device=dev) * 0.5).to(torch.bfloat16)
      o, lse = K.attn_fwd(qkv, L, B, T, H, dh, 1 / math.sqrt(dh))
      do = torch.randn(B * T, H * dh, device=dev).to(torch.bfloat16)
      tf = timeit(lambda: K.attn_fwd(qkv, L, B, T, H, dh, 1 / math.sqrt(dh)))
      tb = timeit(lambda: K.attn_bwd(qkv, o, do, lse, L, B, T, H, dh, 1 / math.sqrt(dh)))
      kv = np.ceil(lens / 64) * 64
      fl = float(np.sum(4.0 * H * kv * kv * dh))
      print(f"{name}: fwd {tf:6.1f} us ({fl / tf / 1e6:5.0f} TF)  bwd {tb:6.1f} us "
            f"({2.5 * fl / tb / 1e6:5.0f} TF)", flush=True)
K.lib.fs2_set_tuning(9, 0)
