"""Stale-read probe: one training configuration under poisoned memory (run as a subprocess).

Every device allocation of the process comes from the library's debug allocator
(``fs2_debug_alloc``: no caching, each block filled with the poison byte) and every
workspace / split-K scratch the library reuses is re-filled with the byte before each use
(``fs2_debug_poison``); a freed block is poisoned again on its stream and never reused.
With ``--race`` the side streams trail the main stream by that many microseconds after every
cross-stream wait.  A kernel that reads memory nothing wrote this step, or memory freed before
it ran, therefore reads the byte: runs with two different bytes give different results instead of results that
depend on what ran earlier in the process.  ``tests/test_stale_reads.py`` compares them.

    python tests/stale_probe.py --poison 0 --out a.pt [--dtype bf16|f32] [--path c|kernel]
        [--fuse 0|1] [--batch 8x32] [--seed 25] [--race US [--race-mode 0|1]]

Writes {"grads": {name: tensor}, "losses1": ..., "flat": ..., "m": ..., "v": ...,
"bn": ..., "losses2": ...}: the parameter gradients of one forward + backward
(update=False), then the weights, Adam moments, BatchNorm statistics and losses after two
optimiser steps of a fresh model.
"""
import argparse
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_NAME = "mid-attribute-speaker-generation_amd"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--poison", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--path", default="c", choices=["c", "kernel"])
    ap.add_argument("--fuse", type=int, default=-1, help="FUSE_LN_MIN_ROWS (-1: default)")
    ap.add_argument("--batch", default="8x32")
    ap.add_argument("--seed", type=int, default=25)
    ap.add_argument("--no-side", action="store_true", help="weight gradients on the main stream")
    ap.add_argument("--drop-keep", action="store_true",
                    help="detector self-check: StepCtx.keep forgets what it is given, so the "
                         "side stream's operands may be freed before it reads them")
    ap.add_argument("--race-mode", type=int, default=0,
                    help="0: side streams trail the main stream; 1: the main stream trails")
    ap.add_argument("--race", type=int, default=0,
                    help="hold every non-main stream back this many us after each cross-stream "
                         "wait (fs2_debug_race): a side-stream read of a buffer the main stream "
                         "freed before it then reads the poison")
    ap.add_argument("--plain", action="store_true",
                    help="no poisoning and torch's caching allocator (a repeat-run baseline)")
    a = ap.parse_args(argv)

    if not a.plain:
        os.environ["FS2_POISON"] = str(a.poison)
    import torch
    sys.path.insert(0, REPO)
    lib_mod = importlib.import_module(PKG_NAME + "._lib")
    if not a.plain:
        alloc = torch.cuda.memory.CUDAPluggableAllocator(lib_mod.LIB_PATH, "fs2_debug_alloc",
                                                          "fs2_debug_free")
        torch.cuda.memory.change_current_allocator(alloc)
        lib_mod.lib.fs2_debug_poison(a.poison)
    if a.race:
        lib_mod.lib.fs2_debug_race(a.race, torch.cuda.current_stream().cuda_stream, a.race_mode, 0)

    if a.drop_keep:
        M = importlib.import_module(PKG_NAME + ".model")

        class _Forget(list):
            def append(self, x):
                pass

            def extend(self, x):
                pass

        init = M.StepCtx.__init__

        def _init(self, *args, **kw):
            init(self, *args, **kw)
            self.keep = _Forget()
        M.StepCtx.__init__ = _init
    out = run_config(dtype=a.dtype, path=a.path, fuse=a.fuse, batch=a.batch, seed=a.seed,
                     side=not a.no_side)
    torch.save(out, a.out)
    print(f"stale_probe poison={a.poison} dtype={a.dtype} path={a.path}: "
          f"losses2 {out['losses2'][-1].tolist()}")


def run_config(dtype="bf16", path="c", fuse=-1, batch="8x32", seed=25, side=True):
    """The probe's training runs in this process (whatever allocator is installed): one
    forward + backward without update (parameter gradients), then two optimiser steps of a
    fresh model.  Returns the dict described in the module docstring."""
    import torch
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    pkg = importlib.import_module(PKG_NAME)
    M = importlib.import_module(PKG_NAME + ".model")
    T = importlib.import_module(PKG_NAME + ".train")
    saved = M.C_BLOCKS, M.FUSE_LN_MIN_ROWS
    M.C_BLOCKS = path == "c"
    if fuse >= 0:
        M.FUSE_LN_MIN_ROWS = fuse
    try:
        dev = torch.device("cuda", 0)
        dt = torch.bfloat16 if dtype == "bf16" else torch.float32
        B, Ts = (int(v) for v in batch.split("x"))
        pp, mc, tc, cpath = pkg.config.load_configs("JVS-VCTK")
        b = pkg.data.to_device(pkg.data.syn_batch(B, Ts, seed=8), dev)

        def fresh():
            model = M.FastSpeech2(pp, mc, cpath, device=dev, compute_dtype=dt)
            pkg.seeded.load_seeded_(model)
            model.train()
            model.seed(seed)
            model.overlap_wgrad = side
            return model, T.Trainer(model, pp, mc, tc)

        out = {}
        model, tr = fresh()
        losses = T.train_step(model, tr.opt, tr.Loss, tr.eLoss, b, update=False)[0]
        torch.cuda.synchronize()
        out["losses1"] = torch.stack(list(losses)).detach().cpu()
        out["grads"] = {n: M._g(p).detach().cpu().clone() for n, p in model.named_parameters()
                        if hasattr(p, "_fs2_grad")}
        del model, tr, losses
        model, tr = fresh()
        steps_g, steps_w = [], []
        clip = tr.opt.clip_grad_norm_

        def capture(max_norm):  # each step's gradients as the clip sees them
            model.join_side()
            steps_g.append(model.arena().grad.detach().clone())
            return clip(max_norm)
        tr.opt.clip_grad_norm_ = capture
        l2 = []
        for _ in range(2):
            l2.append(torch.stack(list(tr.step(b)[0])).detach().clone())
            steps_w.append(model.arena().flat.detach().clone())
        torch.cuda.synchronize()
        out["step_grads"] = [g.cpu() for g in steps_g]
        out["step_flat"] = [w.cpu() for w in steps_w]
        out["losses2"] = torch.stack(l2).cpu()
        out["flat"] = model.arena().flat.cpu()
        out["m"] = tr.opt.m.cpu()
        out["v"] = tr.opt.v.cpu()
        out["bn"] = torch.cat([torch.cat([l[1].running_mean, l[1].running_var])
                               for l in model.postnet.convolutions]).cpu()
        names = names_of(model)
        out["names"] = [(names[id(p)], o, p.numel()) for p, o in
                        zip(model.arena().params, model.arena().offsets)]
        return out
    finally:
        M.C_BLOCKS, M.FUSE_LN_MIN_ROWS = saved


def names_of(model):
    return {id(p): n for n, p in model.named_parameters()}


def diff(a, b):
    """Human-readable differences between two probe outputs (empty list: bitwise equal)."""
    import torch
    msgs = []
    for n in a["grads"]:
        x, y = a["grads"][n], b["grads"][n]
        if not torch.equal(x, y):
            d = (x - y).abs()
            msgs.append(f"grad {n}: max|diff| {float(d.max()):.3e} at {int(d.argmax())} "
                        f"({int((d > 0).sum())} of {d.numel()} differ; scale {float(y.abs().max()):.3e})")
    if not torch.equal(a["losses1"], b["losses1"]):
        msgs.append(f"losses1 {a['losses1'].tolist()} vs {b['losses1'].tolist()}")
    if not torch.equal(a["losses2"], b["losses2"]):
        msgs.append(f"losses2 {a['losses2'].tolist()} vs {b['losses2'].tolist()}")
    for i, (ga, gb) in enumerate(zip(a.get("step_grads", []), b.get("step_grads", []))):
        if not torch.equal(ga, gb):
            bad = [n for n, o, c in a["names"] if not torch.equal(ga[o:o + c], gb[o:o + c])]
            first = [n for n, o, c in a["names"] if n in bad]
            worst = max(((float((ga[o:o + c] - gb[o:o + c]).abs().max()), n) for n, o, c in a["names"]
                         if n in bad), default=(0.0, ""))
            msgs.append(f"step {i + 1} gradients: {len(bad)} parameters differ (max |diff| {worst[0]:.3e} "
                        f"in {worst[1]}): {', '.join(first)}")
    for i, (wa, wb) in enumerate(zip(a.get("step_flat", []), b.get("step_flat", []))):
        if not torch.equal(wa, wb):
            bad = [n for n, o, c in a["names"] if not torch.equal(wa[o:o + c], wb[o:o + c])]
            msgs.append(f"weights after step {i + 1}: {len(bad)} parameters differ: {', '.join(bad[:12])}")
    for k in ("flat", "m", "v"):
        if not torch.equal(a[k], b[k]):
            bad = [n for n, o, c in a["names"] if not torch.equal(a[k][o:o + c], b[k][o:o + c])]
            msgs.append(f"{k}: {len(bad)} parameters differ: {', '.join(bad[:8])}")
    if not torch.equal(a["bn"], b["bn"]):
        msgs.append("BatchNorm running statistics differ")
    return msgs


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--compare":  # --compare a.pt b.pt
        import torch
        x, y = (torch.load(p, weights_only=True) for p in sys.argv[2:4])
        d = diff(x, y)
        print("\n".join(d) if d else "bitwise equal")
        sys.exit(1 if d else 0)
    main()
