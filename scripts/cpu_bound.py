"""Is the eager step CPU-bound?  Host enqueue time vs wall time of K steps."""
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
model = M.FastSpeech2(pp, mc, path, device="cuda:0", compute_dtype=torch.bfloat16)
model.train()
tr = TR.Trainer(model, pp, mc, tc)
batch = PKG.data.to_device(PKG.data.syn_batch(48, 128, seed=0), "cuda:0")
for overlap in (True, False):
    model.overlap_wgrad = overlap
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    K = 20
    t0 = time.perf_counter()
    for _ in range(K):
        tr.step(batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"overlap={overlap}: host enqueue {1e3 * (t1 - t0) / K:.2f} ms/step, "
          f"wall {1e3 * (t2 - t0) / K:.2f} ms/step", flush=True)
