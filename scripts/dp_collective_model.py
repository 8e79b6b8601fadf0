"""Price the data-parallel step at N ranks on ONE GPU: the SYN-48 bf16 step
with every bucket's all-reduce replaced by a stand-in on the stream the real collective is
issued from (train.CollectiveModel -> fs2_collective_standin: RCCL-like CU occupancy, HBM
traffic 2 (n-1)/n S read + written, paced to 2 (n-1)/n S / busbw + latency).  Schedules:
  side      the default: each bucket issued from the weight-gradient stream, event-gated on
            the main stream, as soon as its parameters are final; the collective then runs on
            a stream of its own gated on the issuing stream (as ProcessGroupNCCL does)
  comm      issued from a stream of its own, event-gated on the main + weight-gradient streams
  inline    what if the collective ran ON the issuing (weight-gradient) stream: every later
            weight gradient queues behind it
  bucket=B  bucket size B MB (default 32; 139 = one bucket after the backward: no overlap)
Interleaved rounds in one process; prints ms/step per variant and the predicted N-rank
throughput (N x valid frames / step).

    python scripts/dp_collective_model.py [--ranks 8] [--busbw 150,300,450] [--steps 20]
"""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--busbw", default="150,300,450")
    ap.add_argument("--blocks", type=int, default=32)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=torch.bfloat16)
    model.train()
    syn = PKG.data.syn_batch(48, 128, seed=0)
    valid = int(np.sum(syn[7]))
    batch = PKG.data.to_device(syn, dev)
    arena_mb = model.arena().grad.numel() * 4 / 2**20

    variants = [("plain", None)]
    for bw in (float(b) for b in args.busbw.split(",")):
        variants.append((f"side   bucket=32  busbw={bw:.0f}", dict(bw=bw, bucket=32, comm=False)))
    bw0 = float(args.busbw.split(",")[1 if "," in args.busbw else 0])
    for bk in (16, 64, 160):
        variants.append((f"side   bucket={bk:<3d} busbw={bw0:.0f}", dict(bw=bw0, bucket=bk, comm=False)))
    variants.append((f"comm   bucket=32  busbw={bw0:.0f}", dict(bw=bw0, bucket=32, comm=True)))
    variants.append((f"inline bucket=32  busbw={bw0:.0f}", dict(bw=bw0, bucket=32, comm=False, inline=True)))

    def trainer(cfg):
        model._hooks["grad"] = None
        if cfg is None:
            return TR.Trainer(model, pp, mc, tc)
        cm = TR.CollectiveModel(ranks=args.ranks, busbw_gbs=cfg["bw"], blocks=args.blocks,
                                inline=cfg.get("inline", False))
        return TR.Trainer(model, pp, mc, tc, collective_model=cm,
                          bucket_bytes=cfg["bucket"] << 20, comm_stream=cfg["comm"])

    res = {name: [] for name, _ in variants}
    for rnd in range(args.rounds):
        for name, cfg in variants:
            tr = trainer(cfg)
            for _ in range(5):
                tr.step(batch)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.steps):
                tr.step(batch)
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / args.steps)
            print(f"round {rnd} {name:32s} {res[name][-1]:.3f} ms/step", flush=True)
    model._hooks["grad"] = None
    cm = TR.CollectiveModel(ranks=args.ranks)
    wire = cm.wire_bytes(arena_mb * 2**20) / 2**20
    print(f"\nranks {args.ranks}, gradient buffer {arena_mb:.1f} MB fp32, per-rank ring traffic "
          f"{wire:.1f} MB/step, stand-in blocks {args.blocks}, latency {cm.lat:.0f} us per collective")
    base = min(res["plain"])
    for name, _ in variants:
        t = min(res[name])
        print(f"{name:32s} {t:7.3f} ms/step (min of {args.rounds})  x{t / base:5.3f} of plain  "
              f"predicted {args.ranks}-rank {args.ranks * valid / t * 1e3 / 1e6:6.2f} M mel-frames/s "
              f"(scaling eff {base / t:5.3f})", flush=True)


if __name__ == "__main__":
    main()
