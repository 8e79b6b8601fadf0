"""Nondeterminism probe of the single-GPU step: the same forward + both backwards from the same
weights, repeated; each repetition's flat gradient is compared bitwise with the first, and the
parameters whose gradients differ are named (arena order).  Dropout off, SYN-8 x 32 (the bitwise
tests' size) and SYN-48 shapes."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
T = importlib.import_module("mid-attribute-speaker-generation_amd.train")
dev = torch.device("cuda", 0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
for (B, Tm, drop) in ((8, 32, False), (48, 128, False), (48, 128, True)):
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    torch.manual_seed(0)
    model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
    model.train()
    model.dropout = drop
    tr = T.Trainer(model, pp, mc, tc)
    batch = PKG.data.to_device(PKG.data.syn_batch(B, Tm, seed=3), dev)
    arena = model.arena()
    names = {}
    for n, p in model.named_parameters():
        names[id(p)] = n
    order = [names.get(id(p), "?") for p in arena.params]
    ref = None
    bad = {}
    for r in range(reps):
        if drop:
            model.seed(25)
        tr.opt.zero_grad()
        output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
        losses = tr.Loss(batch[:12], output[:-2])
        losses[0].backward()
        eloss = tr.eLoss(output[-1], output[-2])
        (-eloss).backward()
        torch.cuda.synchronize()
        g = arena.grad.clone()
        if ref is None:
            ref = g
            continue
        if not torch.equal(g, ref):
            for i, p in enumerate(arena.params):
                o = arena.offsets[i]
                a, b = g[o:o + p.numel()], ref[o:o + p.numel()]
                if not torch.equal(a, b):
                    bad[order[i]] = bad.get(order[i], 0) + 1
            print(f"B={B} T={Tm} drop={drop} rep {r}: differs in "
                  f"{sorted(k for k in bad)[:12]}", flush=True)
    print(f"B={B} T={Tm} drop={drop}: {reps - 1} repetitions, parameters that differed: {bad}",
          flush=True)
