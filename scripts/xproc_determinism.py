"""Cross-process determinism of the single-GPU training step: each child process builds the
model (fixed seeds, dropout off), runs 2 optimiser steps and prints a hash of the weights and
the losses; the parent (which never touches the GPU) compares children across schedules:
C-ABI blocks on / off, weight-gradient side stream on / off."""
import hashlib
import importlib
import os
import subprocess
import sys

CHILD = r'''
import importlib, sys, hashlib, torch
sys.path.insert(0, {repo!r})
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
T = importlib.import_module("mid-attribute-speaker-generation_amd.train")
M.C_BLOCKS = {cb}
dev = torch.device("cuda", 0)
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
torch.manual_seed(0)
junk = torch.randn({junk}, device=dev)  # leaves stale values in the caching allocator
del junk
model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
model.train(); model.dropout = False; model.overlap_wgrad = {side}
t = T.Trainer(model, pp, mc, tc)
batch = PKG.data.to_device(PKG.data.syn_batch(8, 32, seed=0), dev)
ls = [torch.stack(list(t.step(batch)[0])).cpu() for _ in range(2)]
torch.cuda.synchronize()
w = model.arena().flat.cpu().numpy().tobytes()
print("RESULT", hashlib.sha1(w).hexdigest()[:12], [round(float(x), 6) for x in ls[-1]])
'''
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for cb, side in ((True, True), (True, False), (False, True)):
    seen = {}
    for i in range(n):
        junk = [1, 1 << 20, 3 << 22, 1 << 24][i % 4]
        code = CHILD.format(repo=repo, cb=cb, side=side, junk=junk)
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
        r = line[0] if line else "ERROR " + out.stderr[-300:]
        seen.setdefault(r, []).append(i)
        print(f"C_BLOCKS={cb} side={side} child {i} (junk {junk}): {r}", flush=True)
    print(f"C_BLOCKS={cb} side={side}: {len(seen)} distinct results over {n} processes", flush=True)
