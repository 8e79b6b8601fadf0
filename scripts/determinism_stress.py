"""Repeat one fixed training configuration in ONE process, interleaved with the workloads the
GPU test suite runs before the round-5 intermittent failures (use_clf steps, collective-model
steps with and without a communication stream, graph replays, a SYN-48 step), and compare every
repetition with the first bitwise (tests/stale_probe.run_config: step-1 gradients, then weights,
Adam moments, BatchNorm statistics and losses after two optimiser steps).

    python scripts/determinism_stress.py [--iters 6] [--dtype bf16] [--path c]
"""
import argparse
import importlib
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import stale_probe  # noqa: E402

PKG_NAME = "mid-attribute-speaker-generation_amd"
pkg = importlib.import_module(PKG_NAME)
M = importlib.import_module(PKG_NAME + ".model")
T = importlib.import_module(PKG_NAME + ".train")
G = importlib.import_module(PKG_NAME + ".ge2e")
DEV = torch.device("cuda", 0)


def _model(dt=torch.bfloat16, seed=None, dropout=True):
    pp, mc, tc, path = pkg.config.load_configs("JVS-VCTK")
    if seed is not None:
        torch.manual_seed(seed)
    model = M.FastSpeech2(pp, mc, path, device=DEV, compute_dtype=dt)
    if seed is None:
        pkg.seeded.load_seeded_(model)
    model.train()
    model.dropout = dropout
    return model, (pp, mc, tc)


def w_clf():
    model, (pp, mc, tc) = _model(torch.float32, dropout=False)
    tr = T.Trainer(model, pp, mc, tc)
    d = G.SpeechEmbedder(device=DEV)
    pkg.seeded.load_seeded_(d)
    d.da_dropout = 0.0
    batch = pkg.data.to_device(pkg.data.syn_batch(3, 48, seed=3), DEV)
    for step in (4, 5):
        T.train_step(model, tr.opt, tr.Loss, tr.eLoss, batch, tr.clip, clf=(d, G.GE2ELoss(DEV)),
                     clf_args=([2, 0, 1], step, 10, 1.0))


def w_collective(comm):
    def f():
        model, (pp, mc, tc) = _model(seed=0, dropout=False)
        t = T.Trainer(model, pp, mc, tc, collective_model=T.CollectiveModel(
            ranks=8, busbw_gbs=300.0, blocks=8, latency_us=5.0), bucket_bytes=16 << 20,
            comm_stream=comm)
        for s in range(2):
            t.step(pkg.data.to_device(pkg.data.syn_batch(8, 32, seed=10 + s), DEV))
    return f


def w_graph():
    model, (pp, mc, tc) = _model()
    model.seed(11)
    tr = T.Trainer(model, pp, mc, tc, graph=True)
    batch = pkg.data.to_device(pkg.data.syn_batch(8, 32, seed=4), DEV)
    for _ in range(4):
        tr.step(batch)


def w_big():
    model, (pp, mc, tc) = _model(seed=1)
    tr = T.Trainer(model, pp, mc, tc)
    batch = pkg.data.to_device(pkg.data.syn_batch(48, 128, seed=0), DEV)
    for _ in range(2):
        tr.step(batch)


WORK = {"clf": w_clf, "coll0": w_collective(False), "coll1": w_collective(True),
        "graph": w_graph, "big": w_big}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--path", default="c")
    ap.add_argument("--fuse", type=int, default=-1)
    a = ap.parse_args()
    cfg = dict(dtype=a.dtype, path=a.path, fuse=a.fuse)
    t0 = time.time()
    ref = stale_probe.run_config(**cfg)
    print(f"reference: losses2 {ref['losses2'][-1].tolist()} ({time.time() - t0:.1f} s)", flush=True)
    bad = 0
    for it in range(a.iters):
        for name, fn in WORK.items():
            fn()
            torch.cuda.synchronize()
            got = stale_probe.run_config(**cfg)
            d = stale_probe.diff(ref, got)
            print(f"iter {it} after {name}: {'equal' if not d else 'DIFFERS'} "
                  f"({time.time() - t0:.0f} s)", flush=True)
            for line in d[:30]:
                print("   ", line, flush=True)
            bad += bool(d)
    print(f"{bad} differing repetitions of {a.iters * len(WORK)}")


if __name__ == "__main__":
    main()
