"""Host enqueue time vs GPU time per training step (is the step launch-bound?)."""
import importlib, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
dev = torch.device("cuda", 0)
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
model.train()
tr = TR.Trainer(model, pp, mc, tc)
batch = PKG.data.to_device(PKG.data.syn_batch(48, 128, seed=0), dev)
for _ in range(5):
    tr.step(batch)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    tr.step(batch)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step", flush=True)
# host-side profile of one step
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    tr.step(batch)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
