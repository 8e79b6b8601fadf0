"""HIP-event timeline of one training step (no profiler): forward, main-stream backward, the
side stream's drain, clip + Adam."""
import importlib, os, sys
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
E = lambda: torch.cuda.Event(enable_timing=True)
res = []
for it in range(10):
    ev = {k: E() for k in ("start", "fwd", "bwd", "side", "end")}
    ev["start"].record()
    output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
    ev["fwd"].record()
    losses = tr.Loss(batch[:12], output[:-2])
    losses[0].backward()
    eloss = tr.eLoss(output[-1], output[-2])
    (-eloss).backward()
    ev["bwd"].record()
    side = model.side_stream()
    ev["side"].record(side)
    tr.opt.clip_grad_norm_(tr.clip)
    tr.opt.step_and_update_lr()
    tr.opt.zero_grad()
    ev["end"].record()
    res.append(ev)
torch.cuda.synchronize()
t = np.array([[r["start"].elapsed_time(r[k]) for k in ("fwd", "bwd", "side", "end")] for r in res])
print("ms from step start (mean over 10): fwd end %.3f | main bwd end %.3f | side drained %.3f | step end %.3f"
      % tuple(t.mean(0)))
