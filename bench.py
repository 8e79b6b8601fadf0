"""Throughput of the FastSpeech2 + TacoSpawn training step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

A step is one full optimiser step of train.py:138-206 (forward, FastSpeech2Loss + GMM
backward, clip_grad_norm_, Adam + LR schedule, zero_grad) on a synthetic SYN-48 batch per
rank (B = 48, 128 phonemes x 512 frames padded) with inputs resident in HBM.
value = valid mel frames of all ranks per second (max-over-ranks time, weak scaling).

The JSON line also carries
  roofline     the decoder FFN Conv1d(256->1024, k=9) forward implicit GEMM (the dominant
               kernel: the k=9 convs are 75% of the FFT-block FLOPs), achieved FLOP/s from HIP
               events around its launches inside the timed region, against the dense MFMA
               peak of the compute dtype;
  cpu_baseline the CPU oracle (oracle/fs2_cpu.py, a restatement of the reference step) timed
               on this host's cores on a bounded sample (rank 0, N = 1 only).
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")

PEAK = {"f32": (157.3, "TFLOP/s"), "bf16": (2500.0, "TFLOP/s")}
# the dominant kernel as rocprofv3 names it (bf16 path: the channel-block-major halo kernel,
# 1,536 workgroups of 128 x 128 at SYN-48; scripts/kshape.py isolates the same launches)
ROOF_KERNEL = "conv_gemm_halo<256, 128, 2, 16, false, 8>"
_SYN = PKG.data.syn_batch(48, 128, seed=0)
_N, _VALID = 48 * int(_SYN[8]), int(np.sum(_SYN[7]))
# compulsory bytes of one decoder FFN Conv1d(256 -> 1024, k=9) forward launch at SYN-48 (rank
# 0's batch), bf16 operands: read the valid rows of x (V x 256) and the re-laid-out weight
# (1024 x 9*256) once, write every row of h (N x 1024; padded rows are written as zeros)
ALG_BYTES = _VALID * 256 * 2 + 1024 * 2304 * 2 + _N * 1024 * 2


class ConvTimer:
    """HIP events around every decoder FFN Conv1d(256 -> 1024, k=9) forward launch (the
    dominant kernel; 6 launches per step at SYN-48, each a 24,576 x 1,024 x 2,304 implicit
    GEMM, grid 1,536 tiles of 128 x 128 -- the only launch of that grid in the step, so the
    rocprofv3 trace isolates the same launches: scripts/kshape.py).

    Eager steps: events are recorded around the launches of the timed steps.  Graph replay:
    the event records are captured into the step graph next to the kernels (``capture``
    mode), so every replay re-records them and the durations read after the timed loop are
    those of the last timed replay."""

    def __init__(self):
        self.on = False
        self.capture = False
        self.events, self.flops = [], []
        self.rows = 0  # padded mel frames of the batch (the decoder's rows)
        self.valid = 0  # valid mel frames of the batch (algorithmic rows)
        self._orig = K.conv_gemm

    def install(self):
        orig = self._orig

        def timed(x, wk, rows, seq_len, c_in, c_out, taps, pad, **kw):
            rec = (taps == 9 and c_out > c_in and rows == self.rows and
                   (self.on or (self.capture and torch.cuda.is_current_stream_capturing())))
            if not rec:
                return orig(x, wk, rows, seq_len, c_in, c_out, taps, pad, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            y = orig(x, wk, rows, seq_len, c_in, c_out, taps, pad, **kw)
            e.record()
            self.events.append((s, e))
            # algorithmic FLOP: valid frames only (the kernel also computes the padded rows
            # of tiles that hold a valid frame, and skips all-padding tiles)
            self.flops.append(2.0 * self.valid * c_out * c_in * taps)
            return y

        K.conv_gemm = timed

    def result(self):
        if not self.events:
            return None, None, 0
        torch.cuda.synchronize()
        try:
            ms = [s.elapsed_time(e) for s, e in self.events]
        except RuntimeError:
            return None, None, 0
        if not all(np.isfinite(ms)) or min(ms) <= 0:
            return None, None, 0
        return float(np.sum(self.flops)), float(np.sum(ms)) / 1e3, len(ms)


PROBE_SHAPES = [  # the decoder's FFN k=9 forward launch (h = relu(conv(x1) + b))
    (24576, 512, 256, 1024, 9, "fwd")]


def probe_conv(reps=10):
    """The dominant kernel's launches alone (same shapes / epilogues as the step), for the
    PMC passes of ``hbm_traffic``."""
    dev = torch.device("cuda", 0)
    lens = torch.tensor(_SYN[7], device=dev)  # the step passes the mel lengths (tile skip)
    for M_, T_, cin, cout, k, kind in PROBE_SHAPES:
        x = torch.randn(M_, cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(cout * cin * k, device=dev) * 0.02).to(torch.bfloat16)
        if kind == "fwd":
            b = torch.randn(cout, device=dev)
            run = lambda: K.conv_gemm(x, w, M_, T_, cin, cout, k, 4, bias=b, flags=K.EPI_RELU,
                                      out_dtype=torch.bfloat16, lens=lens)
        else:
            aux = torch.randn(M_, cout, device=dev)
            run = lambda: K.conv_gemm(x, w, M_, T_, cin, cout, k, 4, flags=K.EPI_ADD_AUX,
                                      aux=aux, out=aux, lens=lens)
        for _ in range(reps):
            run()
    torch.cuda.synchronize()


def hbm_traffic(timeout=300):
    """Per-launch memory-side bytes of the k=9 conv GEMM from rocprofv3 PMC counters:
    FETCH_SIZE and WRITE_SIZE (KiB) in separate passes (they do not fit one TCC pass),
    FETCH_SIZE doubled (gfx950 reports half the bytes of 16-B-per-lane streaming reads;
    MI355X_MICROARCH.md, HBM).  These count L2 misses, Infinity-Cache hits included."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    per = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = [prof, "--pmc", ctr, "-d", d, "-o", "probe", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--probe-conv"]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
            except subprocess.TimeoutExpired:
                return None, f"{ctr} pass timed out"
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None, f"{ctr} pass failed (rc {r.returncode})"
            vals = []
            for row in csv.DictReader(open(files[0])):
                if ROOF_KERNEL in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                    vals.append(float(row["Counter_Value"]))
            if not vals:
                return None, f"{ctr}: no {ROOF_KERNEL} dispatches"
            per[ctr] = float(np.mean(vals))
    # both counters are in KiB
    return (per["FETCH_SIZE"] * 2.0 + per["WRITE_SIZE"]) * 1024.0, per


def cpu_baseline(batch_np, steps=2):
    from oracle import fs2_cpu
    n_thr = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(n_thr)
    ref, _ = fs2_cpu.build("JVS-VCTK")
    ref.train()
    opt = fs2_cpu.make_opt(ref)
    b = PKG.data.to_device(batch_np, "cpu")
    fs2_cpu.train_step(ref, opt, b)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        fs2_cpu.train_step(ref, opt, b)
    dt = time.perf_counter() - t0
    frames = int(np.sum(batch_np[7]))
    return {"value": round(frames * steps / dt, 1), "unit": "mel-frames/s",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/fs2_cpu.py train step (dropout on), SYN-{len(batch_np[4])} "
                      f"seed 0, {steps} timed steps after 1 warm-up, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=48)
    ap.add_argument("--src-len", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["f32", "bf16"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--graph", action="store_true",
                    help="N=1: capture the step once into a HIP graph and replay it (measured "
                         "slower than eager here: replay serialises the weight-gradient stream)")
    ap.add_argument("--use-clf", action="store_true",
                    help="BASELINE config 3: the --use_clf step (second forward with shuffled "
                         "speakers + GE2E language discriminator on 150-frame chunks)")
    ap.add_argument("--probe-conv", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.probe_conv:
        probe_conv()
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    cdt = {"f32": torch.float32, "bf16": torch.bfloat16}[args.dtype]
    model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=cdt)
    model.train()
    model.seed(1234 + rank)
    use_graph = world == 1 and args.graph
    trainer = TR.Trainer(model, pp, mc, tc, graph=use_graph and not args.use_clf)
    if args.use_clf:
        import random
        G = importlib.import_module("mid-attribute-speaker-generation_amd.ge2e")
        disc = G.SpeechEmbedder(device=dev)
        PKG.seeded.load_seeded_(disc)
        clf = (disc, G.GE2ELoss(dev))
        rnd = random.Random(1234 + rank)
        counter = [0]

        def clf_kw():  # train.py:171 draws the shuffle with random.sample each step
            counter[0] += 1
            return {"clf": clf, "clf_args": (rnd.sample(range(args.batch), args.batch),
                                             counter[0], tc["step"]["total_step"],
                                             float(tc.get("lambda", 1)))}
    batch_np = PKG.data.syn_batch(args.batch, args.src_len, seed=rank)
    batch = PKG.data.to_device(batch_np, dev)
    frames_local = int(np.sum(batch_np[7]))
    padded_local = int(args.batch * batch_np[8])

    timer = ConvTimer()
    timer.rows = padded_local
    timer.valid = frames_local
    if not args.no_roofline:
        timer.install()
        timer.capture = use_graph
    for _ in range(max(args.warmup, 2 if use_graph else 0)):  # graph: step 1 captures
        trainer.step(batch, **(clf_kw() if args.use_clf else {}))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer.on = not use_graph
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses, eloss, gnorm = trainer.step(batch, **(clf_kw() if args.use_clf else {}))[:3]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    timer.on = False
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    fr = torch.tensor([frames_local], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(fr)
    dt, frames = float(t.item()), float(fr.item())
    loss_now = float(losses[0])

    if rank == 0:
        flops, secs, n = timer.result()
        if not flops and use_graph and not args.no_roofline:
            # event timing inside the graph unavailable: time the same launches in one
            # eager step after the timed region (same kernels, same shapes)
            timer.events, timer.flops, timer.capture, timer.on = [], [], False, True
            trainer.graph_mode = False
            trainer.step(batch)
            timer.on = False
            flops, secs, n = timer.result()
        roof = None
        if flops:
            peak, unit = PEAK[args.dtype]
            ach = flops / secs / 1e12
            roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": unit,
                    "frac": round(ach / peak, 4), "traffic": None,
                    "kernel": (f"{ROOF_KERNEL if args.dtype == 'bf16' else 'conv_gemm_nt_f32'} "
                               "(decoder FFN Conv1d 256->1024 k=9, forward)"),
                    "flop_basis": "2 * valid frames * 1024 * 256 * 9 per launch",
                    "per_launch_flop": round(flops / n), "avg_launch_ms": round(secs / n * 1e3, 4)}
            if world == 1 and args.dtype == "bf16" and not args.no_traffic:
                traffic, detail = hbm_traffic()
                if traffic is not None:
                    roof["traffic"] = round(traffic)
                    roof["traffic_unit"] = "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, PMC)"
                    roof["traffic_algorithmic"] = ALG_BYTES
                else:
                    roof["traffic_note"] = detail
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(batch_np)
        out = {"metric": "mel-frames/sec (node) FastSpeech2 train step, JVS-VCTK bs=48, 1/2/4/8 MI355X",
               "value": round(frames * args.steps / dt, 1), "unit": "mel-frames/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic SYN-B (seeded, rank r uses seed r), random-init weights",
               "config": {"workload": f"SYN-{args.batch}: FastSpeech2+TacoSpawn train step, "
                                      f"B={args.batch}/GPU, {args.src_len} phonemes x "
                                      f"{int(batch_np[8])} frames padded",
                          "global_batch": args.batch * world, "seq_len": int(batch_np[8]),
                          "valid_frames_per_rank_step": frames_local,
                          "padded_frames_per_rank_step": padded_local,
                          "parallelism": f"dp{world}",
                          "use_clf": bool(args.use_clf),
                          "execution": "hip-graph replay" if use_graph else "eager"},
               "roofline": roof, "cpu_baseline": cpu, "final_loss": round(loss_now, 5)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
