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
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")


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
    ap.add_argument("--mode", type=int, default=2,
                    help="fs2_debug_race mode: 2 seeded random; 0 side trails / 1 main trails by "
                         "--max-us after every wait (the seed is then ignored)")
    ap.add_argument("--guard", action="store_true",
                    help="guard tails on every C-path region; report out-of-bounds writes")
    ap.add_argument("--save-snaps", default="")
    a = ap.parse_args()
    M._GUARD["on"] = a.guard
    snapbuf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda") if a.guard else None
    if a.guard:
        lib.fs2_debug_snap(snapbuf.data_ptr(), snapbuf.numel())
    snapdata = {}
    saved = {}

    snaps = {}

    def guards(tag):
        if a.guard:
            torch.cuda.synchronize()
            used = lib.fs2_debug_snap_used()
            snapdata[tag] = snapbuf[:min(used, snapbuf.numel())].cpu()
            lib.fs2_debug_snap(snapbuf.data_ptr(), snapbuf.numel())
            if tag != "baseline":
                x, y = snapdata["baseline"], snapdata[tag]
                if x.numel() != y.numel():
                    print(f"  snapshots: {x.numel()} vs {y.numel()} bytes", flush=True)
                else:
                    ne = (x != y).nonzero()
                    if ne.numel():
                        print(f"  snapshots differ from byte {int(ne[0])} of {x.numel()} "
                              f"({ne.numel()} bytes differ)", flush=True)

            snaps[tag] = [(site, [t.cpu() for t in ts]) for site, ts in M._GUARD.pop("snap", [])]
            if tag != "baseline" and "baseline" in snaps:
                names = ("lin_w", "lin_b", "ln2_g", "ln2_b", "dpred", "act", "x_t")
                for i, ((s0, ta), (s1, tb)) in enumerate(zip(snaps["baseline"], snaps[tag])):
                    bad = [n for n, x, y in zip(names, ta, tb) if not torch.equal(x, y)]
                    if bad:
                        print(f"  predictor backward #{i} (site {s0}) inputs differ: {bad}", flush=True)
            bad = M.check_guards()
            print(f"  guards after {tag}: {'intact' if not bad else 'WRITTEN: ' + ', '.join(bad)}",
                  flush=True)
            M._GUARD["regions"].clear()
    cfg = dict(dtype=a.dtype, path=a.path, fuse=a.fuse, batch=a.batch)
    main_st = torch.cuda.current_stream().cuda_stream
    t0 = time.time()
    base = stale_probe.run_config(**cfg)
    guards("baseline")
    again = stale_probe.run_config(**cfg)
    guards("repeat")
    print(f"baseline: losses2 {base['losses2'][-1].tolist()}; repeat "
          f"{'equal' if not stale_probe.diff(base, again) else 'DIFFERS'} ({time.time() - t0:.1f} s)",
          flush=True)
    bad = []
    for s in seeds_of(a.seeds):
        lib.fs2_debug_race(a.max_us, main_st, a.mode, s)
        got = stale_probe.run_config(**cfg)
        torch.cuda.synchronize()
        lib.fs2_debug_race(0, main_st, 0, 0)
        guards(f"seed {s}")
        d = stale_probe.diff(base, got)
        if d and a.save_snaps and len(saved) < 4:  # the intermediates of a differing run
            saved[f"seed {s}"] = snapdata[f"seed {s}"]
            torch.save({"baseline": snapdata["baseline"], **saved}, a.save_snaps)
        print(f"seed {s}: {'equal' if not d else 'DIFFERS'} ({time.time() - t0:.0f} s)", flush=True)
        for line in d[:40]:
            print("   ", line[:3000], flush=True)
        if d:
            bad.append(s)
    print(f"differing seeds: {bad}")


if __name__ == "__main__":
    main()
