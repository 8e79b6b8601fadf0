"""Determinism probe: the C-ABI step against the per-kernel step (test_c_blocks_step_bitwise's
setup, fuse threshold 0), repeated, with the pitch predictor's forward on the side stream on /
off: prints the max abs difference of (weights, Adam m, Adam v, losses) per repetition."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
T = importlib.import_module("mid-attribute-speaker-generation_amd.train")


def run(c_blocks, va_side, batch_seed=8):
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    M.C_BLOCKS, M.FUSE_LN_MIN_ROWS, M.VA_SIDE = c_blocks, 0, va_side
    model = M.FastSpeech2(pp, mc, path, device="cuda", compute_dtype=torch.bfloat16)
    PKG.seeded.load_seeded_(model)
    model.train()
    model.seed(25)
    tr = T.Trainer(model, pp, mc, tc)
    batch = PKG.data.to_device(PKG.data.syn_batch(8, 32, seed=batch_seed), "cuda")
    losses = [torch.stack(list(tr.step(batch)[0])).clone() for _ in range(2)]
    torch.cuda.synchronize()
    return (model.arena().flat.clone(), tr.opt.m.clone(), tr.opt.v.clone(), torch.stack(losses))


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for va_side in (True, False):
    ref = run(False, va_side)
    bad = 0
    for r in range(reps):
        got = run(True, va_side)
        d = [float((a - b).abs().max()) for a, b in zip(got, ref)]
        bad += any(x != 0 for x in d)
        print(f"VA_SIDE={va_side} rep {r}: {d}", flush=True)
        py = run(False, va_side)
        d = [float((a - b).abs().max()) for a, b in zip(py, ref)]
        bad += any(x != 0 for x in d)
        print(f"VA_SIDE={va_side} py rep {r}: {d}", flush=True)
    print(f"VA_SIDE={va_side}: {bad} mismatching runs of {2 * reps}", flush=True)
