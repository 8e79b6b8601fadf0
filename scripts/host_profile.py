"""Host-side (enqueue) profile of the eager training step: cProfile over 20 steps after
warm-up, top functions by own time.  The GPU runs behind the host (the step is GPU-bound),
so this is the Python + ctypes + launch cost the host pays per step.

    python scripts/host_profile.py [--py] [--one-thread]
(--py: per-kernel issue, model.C_BLOCKS off; --one-thread: the autograd backward runs on the
profiled thread instead of the device thread)"""
import cProfile
import importlib
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
dev = torch.device("cuda", 0)
if "--py" in sys.argv:
    M.C_BLOCKS = False
if "--one-thread" in sys.argv:  # backward on this thread, so cProfile sees its Python too
    torch.autograd.set_multithreading_enabled(False)
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
model.train()
tr = TR.Trainer(model, pp, mc, tc)
batch = PKG.data.to_device(PKG.data.syn_batch(48, 128, seed=0), dev)
for _ in range(5):
    tr.step(batch)
torch.cuda.synchronize()
N = 20
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    tr.step(batch)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
print(f"total host time per step: {st.total_tt / N * 1e3:.3f} ms (cProfile adds its own overhead)")
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumtime").print_stats(45)
