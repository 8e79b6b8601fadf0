"""Per-phase GPU (HIP events) and host (enqueue) time of one training step, no profiler:
forward | GMM speaker loss fwd+bwd | losses | main backward | side-stream drain | clip + Adam
(train_step's order)."""
import importlib, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
dev = torch.device("cuda", 0)
if "--py" in sys.argv:  # the per-kernel host path (model.C_BLOCKS off) for the A/B
    M.C_BLOCKS = False
# --modules: HIP events on the main stream around each autograd block's forward and backward
# (encoder, variance adaptor, decoder, mel head): where the step's main-stream time goes
MODS = {}
if "--modules" in sys.argv:
    for nm in ("EncoderFn", "VarianceAdaptorFn", "DecoderFn", "MelHeadFn"):
        cls = getattr(M, nm)
        for ph in ("forward", "backward"):
            f = getattr(cls, ph)

            def wrap(*a, _f=f, _k=f"{nm[:-2]}.{ph[:3]}"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = _f(*a)
                e1.record()
                MODS.setdefault(_k, []).append((e0, e1))
                return r
            setattr(cls, ph, staticmethod(wrap))
pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
model.train()
tr = TR.Trainer(model, pp, mc, tc)
batch = PKG.data.to_device(PKG.data.syn_batch(48, 128, seed=0), dev)
for _ in range(5):
    tr.step(batch)
torch.cuda.synchronize()
E = lambda: torch.cuda.Event(enable_timing=True)
names = ("fwd", "eloss", "loss", "bwd", "side", "end")
gpu, host = [], []
for it in range(12):
    ev = {k: E() for k in ("start",) + names}
    h = [time.perf_counter()]
    ev["start"].record()
    output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
    ev["fwd"].record(); h.append(time.perf_counter())
    eloss = tr.eLoss(output[-1], output[-2])  # train_step's order: the GMM loss first
    (-eloss).backward()
    ev["eloss"].record(); h.append(time.perf_counter())
    losses = tr.Loss(batch[:12], output[:-2])
    ev["loss"].record(); h.append(time.perf_counter())
    losses[0].backward()
    ev["bwd"].record(); h.append(time.perf_counter())
    ev["side"].record(model.side_stream()); h.append(time.perf_counter())
    tr.opt.clip_grad_norm_(tr.clip)
    tr.opt.step_and_update_lr()
    tr.opt.zero_grad()
    ev["end"].record(); h.append(time.perf_counter())
    gpu.append(ev); host.append(h)
torch.cuda.synchronize()
g = np.array([[r["start"].elapsed_time(r[k]) for k in names] for r in gpu[2:]])
hh = np.array([[(x - hr[0]) * 1e3 for x in hr[1:]] for hr in host[2:]])
print("GPU  ms from step start:", "  ".join(f"{n} {v:.3f}" for n, v in zip(names, g.mean(0))))
print("host ms from step start:", "  ".join(f"{n} {v:.3f}" for n, v in zip(names, hh.mean(0))))
print(f"C blocks: {M.C_BLOCKS}; host enqueue {hh.mean(0)[-1]:.3f} ms, GPU {g.mean(0)[-1]:.3f} ms per step")
if MODS:
    torch.cuda.synchronize()
    for k, v in MODS.items():
        t = [a.elapsed_time(b) for a, b in v[-10:]]
        print(f"  {k:24s} {np.mean(t):.3f} ms (main stream, last {len(t)} steps)")
