"""Explore stream interleavings of one training configuration in ONE process: a baseline run
(no delays), then runs under seeded random schedules (fs2_debug_race mode 2: at every
cross-stream wait the waiter and the signaler are each held back, with probability 1/2, by a
random 0..max_us), each compared bitwise with the baseline (tests/stale_probe.run_config:
step-1 gradients, then weights / Adam moments / BatchNorm statistics / losses after two
optimiser steps).  A seed that differs replays its interleaving: rerun with --seeds S.

    python scripts/schedule_explorer.py [--seeds 1-40] [--max-us 400] [--path c] [--fuse -1]
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

lib = importlib.import_module("mid-attribute-speaker-generation_amd._lib").lib


def seeds_of(spec):
    out = []
    for part in spec.split(","):
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="1-40")
    ap.add_argument("--max-us", type=int, default=400)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--path", default="c")
    ap.add_argument("--fuse", type=int, default=-1)
    ap.add_argument("--batch", default="8x32")
    a = ap.parse_args()
    cfg = dict(dtype=a.dtype, path=a.path, fuse=a.fuse, batch=a.batch)
    main_st = torch.cuda.current_stream().cuda_stream
    t0 = time.time()
    base = stale_probe.run_config(**cfg)
    again = stale_probe.run_config(**cfg)
    print(f"baseline: losses2 {base['losses2'][-1].tolist()}; repeat "
          f"{'equal' if not stale_probe.diff(base, again) else 'DIFFERS'} ({time.time() - t0:.1f} s)",
          flush=True)
    bad = []
    for s in seeds_of(a.seeds):
        lib.fs2_debug_race(a.max_us, main_st, 2, s)
        got = stale_probe.run_config(**cfg)
        torch.cuda.synchronize()
        lib.fs2_debug_race(0, main_st, 0, 0)
        d = stale_probe.diff(base, got)
        print(f"seed {s}: {'equal' if not d else 'DIFFERS'} ({time.time() - t0:.0f} s)", flush=True)
        for line in d[:40]:
            print("   ", line[:400], flush=True)
        if d:
            bad.append(s)
    print(f"differing seeds: {bad}")


if __name__ == "__main__":
    main()
