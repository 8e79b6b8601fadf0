"""cProfile of the host side of eager steps (where the Python enqueue time goes)."""
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
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
model = M.FastSpeech2(pp, mc, path, device="cuda:0", compute_dtype=torch.bfloat16)
model.train()
tr = TR.Trainer(model, pp, mc, tc)
batch = PKG.data.to_device(PKG.data.syn_batch(48, 128, seed=0), "cuda:0")
for _ in range(3):
    tr.step(batch)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    tr.step(batch)
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(28)
