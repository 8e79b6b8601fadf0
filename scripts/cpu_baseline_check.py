"""Validate the on-box CPU baseline proxy (BASELINE.md / SURVEY.md §8d): the oracle's CPU
train step (oracle/fs2_cpu.py, what bench.py's cpu_baseline times on the GPU box) against
the reference's own step (imported from /root/reference, build container only), same
SYN-48 batch, same thread count, dropout on, 1 warm-up + 3 timed steps each, median.

    python scripts/cpu_baseline_check.py [--threads 8] [--out profiles/r2_cpu_baseline_validation.json]
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timed_steps(step, n=3):
    step()  # warm-up
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r2_cpu_baseline_validation.json"))
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    spec = importlib.util.spec_from_file_location("mg", os.path.join(REPO, "oracle", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    fs2, loss_mod, _, _ = mg.import_reference()  # dropout stays ON (no mg.no_dropout())
    from model.optimizer import ScheduledOptim
    from oracle import fs2_cpu
    PKG = mg.PKG
    batch_np = PKG.data.syn_batch(48, 128, seed=0)
    b = PKG.data.to_device(batch_np, "cpu")
    frames = int(np.sum(batch_np[7]))

    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    ref = fs2.FastSpeech2(pp, mc, path)
    mg.seeded(ref)
    ref.train()
    opt = ScheduledOptim(ref, tc, mc, 0)
    Loss, eLoss = loss_mod.FastSpeech2Loss(pp, mc), loss_mod.SpeakerMetaEncLoss(pp, mc)

    def ref_step():  # train.py:145-206 with grad_acc_step 1, use_clf off
        out = ref(*(b[2:12]), accents=b[13], speaker_meta=b[12])
        losses = Loss(b[:12], out[:-2])
        losses[0].backward()
        (-eLoss(out[-1], out[-2])).backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        opt.step_and_update_lr()
        opt.zero_grad()

    orc, _ = fs2_cpu.build("JVS-VCTK")
    orc.train()
    oopt = fs2_cpu.make_opt(orc)
    t_ref = timed_steps(ref_step)
    t_orc = timed_steps(lambda: fs2_cpu.train_step(orc, oopt, b))
    mr, mo = float(np.median(t_ref)), float(np.median(t_orc))
    cpu = "unknown"
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
    res = {"workload": "SYN-48 train step (dropout on), seed 0, 18,044 valid frames",
           "threads": torch.get_num_threads(), "cpu_model": cpu,
           "reference_s": [round(t, 3) for t in t_ref], "oracle_s": [round(t, 3) for t in t_orc],
           "reference_median_s": round(mr, 3), "oracle_median_s": round(mo, 3),
           "reference_mel_frames_per_s": round(frames / mr, 1),
           "oracle_mel_frames_per_s": round(frames / mo, 1),
           "oracle_over_reference": round(mo / mr, 4),
           "within_10pct": bool(abs(mo / mr - 1.0) <= 0.10)}
    print(json.dumps(res, indent=1))
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
