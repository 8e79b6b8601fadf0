"""Throughput of the FastSpeech2 + TacoSpawn training step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype bf16|f32]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

``--gpus N`` without a launcher (no WORLD_SIZE in the environment) starts N fresh child
processes itself, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1),
before anything touches the GPU; under a launcher WORLD_SIZE must equal ``--gpus``.

A step is one full optimiser step of train.py:138-206 (forward, FastSpeech2Loss + GMM
backward, clip_grad_norm_, Adam + LR schedule, zero_grad) on a synthetic SYN-48 batch per
rank (B = 48, 128 phonemes x 512 frames padded) with inputs resident in HBM.
value = valid mel frames of all ranks per second (max-over-ranks time, weak scaling).

The JSON line also carries
  roofline      the DOMINANT launch set of the step by in-step time: HIP events (on the
                stream each launch runs on, the weight-gradient side stream included) around
                every GEMM / conv / attention launch of the last 3 warm-up steps, grouped by
                op class (``classes``); the class with the most time is then timed alone over
                the timed steps: achieved = its algorithmic FLOP (valid frames) per step / its
                launches' summed duration per step; ``traffic``: PMC bytes per launch of the
                class's decoder-shaped launches;
  fft_block     one decoder FFT block fwd+bwd (north_star's target): HIP events around the
                decoder's forward and backward (its weight-gradient stream joined) in extra
                steps after the timed region, / 6 layers, against SURVEY §8d's 463.9 GFLOP
                (padded shapes) and the valid-frame FLOP;
  step_roofline the whole step: 3,904.7 GFLOP (§8d, padded) / ms_per_step;
  f32           (bf16 runs, N = 1) the same step at the reference's precision (fp32);
  cpu_baseline  the CPU oracle (oracle/fs2_cpu.py, a restatement of the reference step) timed
                on this host's cores: median of 3 steps after 1 warm-up (rank 0, N = 1 only).
"""
import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")

PEAK = {"f32": (157.3, "TFLOP/s"), "bf16": (2500.0, "TFLOP/s")}
METRIC = "mel-frames/sec (node) FastSpeech2 train step, JVS-VCTK bs=48, 1/2/4/8 MI355X"
STEP_GFLOP_PADDED = 3904.7  # SURVEY.md §8d, SYN-48 fwd+bwd at padded shapes
DEC_BLOCK_GFLOP_PADDED = 463.9  # SURVEY.md §8d, one decoder FFT block fwd+bwd at 48 x 512
D, F, KW = 256, 1024, 9


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """Start ``n`` ranks of this script (one process per GPU) and wait for them.  Called
    before anything initialises the GPU; returns the first non-zero exit code (and stops the
    remaining ranks, by PID) or 0."""
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:  # a failed rank leaves the others waiting in a collective
                    q.kill()
        time.sleep(0.05)
    return rc


# ----------------------------------------------------------------------------- timing
class ClassTimer:
    """HIP events around every GEMM / conv / attention launch, on the stream it runs on.

    Launch classes (the k=9 class is the FFN Conv1d of all 10 FFT blocks, forward and data
    gradient, encoder and decoder):
      conv_k9 / conv_k5 / conv_k3 / linear_k1   fwd + data-gradient implicit GEMMs
      wgrad_k9 / wgrad_k5 / wgrad_k3 / wgrad_k1 weight(+bias)-gradient GEMMs incl. reduce
      attention_fwd / attention_bwd             flash attention
    FLOP per launch = 2 * algorithmic rows * C_out * C_in * taps (attention: 4 * d * sum L^2
    forward, 2.5x that backward), algorithmic rows = valid frames of launches given the
    utterance lengths (the kernels skip all-padding tiles), all rows otherwise."""

    def __init__(self, K, valid_by_T, sq_by_T):
        self.K = K
        self.valid_by_T = valid_by_T  # seq_len -> valid rows of the batch
        self.sq_by_T = sq_by_T        # seq_len -> sum of squared lengths (attention)
        self.mode = None               # None: off; "all": every class; else one class name
        self.rec = []                  # (class, start, end, flop)
        self._streams = {}
        self._pool, self._next = [], 0  # events created up front (creation is host-expensive)
        self._orig = {n: getattr(K, n) for n in ("conv_gemm", "conv_wgrad", "conv_wgrad_k1_multi",
                                                 "attn_fwd", "attn_bwd")}

    def reset(self, mode, n_events):
        self.mode, self.rec, self._next = mode, [], 0
        while len(self._pool) < n_events:
            self._pool.append(torch.cuda.Event(enable_timing=True))

    def _stream(self, handle):
        if handle is None:
            return torch.cuda.current_stream()
        s = self._streams.get(handle)
        if s is None:
            s = self._streams[handle] = torch.cuda.ExternalStream(handle)
        return s

    def _timed(self, cls, flop, stream_handle, fn, *a, **kw):
        if self.mode is None or (self.mode != "all" and self.mode != cls) or \
                self._next + 2 > len(self._pool):
            return fn(*a, **kw)
        st = self._stream(stream_handle)
        s, e = self._pool[self._next], self._pool[self._next + 1]
        self._next += 2
        s.record(st)
        y = fn(*a, **kw)
        e.record(st)
        self.rec.append((cls, s, e, flop))
        return y

    def _rows(self, rows, seq_len, lens):
        return self.valid_by_T.get(seq_len, rows) if lens is not None else rows

    def install(self):
        o = self._orig
        T = self

        def conv_gemm(x, wk, rows, seq_len, c_in, c_out, taps, pad, **kw):
            r = T._rows(rows, seq_len, kw.get("lens"))
            cls = f"conv_k{taps}" if taps > 1 else "linear_k1"
            return T._timed(cls, 2.0 * r * c_out * c_in * taps, None, o["conv_gemm"],
                            x, wk, rows, seq_len, c_in, c_out, taps, pad, **kw)

        def conv_wgrad(dy, x, dw, rows, seq_len, c_in, c_out, taps, pad, **kw):
            r = T._rows(rows, seq_len, kw.get("lens"))
            return T._timed(f"wgrad_k{taps}", 2.0 * r * c_out * c_in * taps, kw.get("on_stream"),
                            o["conv_wgrad"], dy, x, dw, rows, seq_len, c_in, c_out, taps, pad, **kw)

        def conv_wgrad_k1_multi(jobs, rows, seq_len, **kw):  # grouped k = 1 weight gradients
            r = T._rows(rows, seq_len, kw.get("lens"))
            fl = sum(2.0 * r * j[4] * j[5] for j in jobs)
            return T._timed("wgrad_k1", fl, kw.get("on_stream"), o["conv_wgrad_k1_multi"], jobs,
                            rows, seq_len, **kw)

        def attn_fwd(qkv, lens, batch, seq_len, heads, d_head, scale):
            fl = 4.0 * heads * d_head * T.sq_by_T.get(seq_len, batch * seq_len * seq_len)
            return T._timed("attention_fwd", fl, None, o["attn_fwd"], qkv, lens, batch, seq_len,
                            heads, d_head, scale)

        def attn_bwd(qkv, o_, d_o, lse, lens, batch, seq_len, heads, d_head, scale):
            fl = 10.0 * heads * d_head * T.sq_by_T.get(seq_len, batch * seq_len * seq_len)
            return T._timed("attention_bwd", fl, None, o["attn_bwd"], qkv, o_, d_o, lse, lens,
                            batch, seq_len, heads, d_head, scale)

        self.K.conv_gemm, self.K.conv_wgrad = conv_gemm, conv_wgrad
        self.K.conv_wgrad_k1_multi = conv_wgrad_k1_multi
        self.K.attn_fwd, self.K.attn_bwd = attn_fwd, attn_bwd

    def table(self, steps, peak):
        torch.cuda.synchronize()
        agg = {}
        for cls, s, e, fl in self.rec:
            ms = s.elapsed_time(e)
            a = agg.setdefault(cls, [0.0, 0.0, 0])
            a[0] += ms
            a[1] += fl
            a[2] += 1
        out = {}
        for cls, (ms, fl, n) in agg.items():
            tf = fl / (ms / 1e3) / 1e12 if ms > 0 else 0.0
            out[cls] = {"ms_per_step": round(ms / steps, 4), "launches_per_step": round(n / steps, 2),
                        "avg_launch_ms": round(ms / n, 4), "gflop_per_step": round(fl / steps / 1e9, 2),
                        "tflops": round(tf, 1), "frac": round(tf / peak, 4)}
        return out


class BlockTimer:
    """Decoder forward / backward timing with the side stream joined at the decoder's end."""

    def __init__(self, M, model):
        self.M, self.model = M, model
        self.on = False
        self.ev = []
        Fn = M.DecoderFn
        self._f, self._b = Fn.forward, Fn.backward
        me = self

        self.ops = None  # OpTimer: per-op spans (this pass puts the GPU behind the host first)

        def spin():
            if me.ops is not None:
                try:
                    torch.cuda._sleep(8_000_000)  # a few ms: the host enqueues the pass meanwhile
                except Exception:
                    pass

        def fwd(fctx, *a):
            if not me.on:
                return me._f(fctx, *a)
            spin()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            if me.ops is not None:
                me.ops.phase = "fwd"
            r = me._f(fctx, *a)
            if me.ops is not None:
                me.ops.phase = None
            e.record()
            me.ev.append(("fwd", s, e))
            return r

        def bwd(fctx, *a):
            if not me.on:
                return me._b(fctx, *a)
            spin()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            if me.ops is not None:
                me.ops.phase = "bwd"
            r = me._b(fctx, *a)
            if me.ops is not None:
                me.ops.phase = None
            me.model.join_side()  # the decoder's weight gradients belong to its backward
            e.record()
            me.ev.append(("bwd", s, e))
            return r

        Fn.forward, Fn.backward = staticmethod(fwd), staticmethod(bwd)

    def result(self):
        torch.cuda.synchronize()
        f = [s.elapsed_time(e) for k, s, e in self.ev if k == "fwd"]
        b = [s.elapsed_time(e) for k, s, e in self.ev if k == "bwd"]
        return (float(np.median(f)), float(np.median(b))) if f and b else (None, None)


class OpTimer:
    """Per-op spans of the decoder's FFT blocks inside the training step (the north star's
    fft_block broken down): every kernel call made while ``phase`` is "fwd" / "bwd" (set by
    BlockTimer around DecoderFn) is bracketed by HIP events on the stream it runs on (the
    weight gradients on the side stream) and labelled by its role in the block.  Before each
    decoder pass a spin kernel (torch.cuda._sleep) puts the GPU behind the host, so the spans
    carry no host launch gaps; the side-stream weight gradients still share the CUs with the
    main-stream chain as in every step."""

    FNS = ("conv_gemm", "conv_gemm_ln", "conv_gemm_ln_bwd", "attn_fwd", "attn_bwd", "ln_fwd",
           "ln_bwd", "conv_wgrad", "conv_wgrad_k1_multi")
    FWD = {(256, 768, 1): "qkv", (256, 256, 1): "fc", (256, 1024, 9): "w1_k9",
           (1024, 256, 1): "w2"}
    BWD = {(256, 1024, 1): "w2_dgrad", (1024, 256, 9): "w1_k9_dgrad", (256, 256, 1): "fc_dgrad",
           (768, 256, 1): "qkv_dgrad"}
    WGRAD = {(1024, 256, 1): "w2_wgrad", (256, 1024, 9): "w1_k9_wgrad", (256, 256, 1): "fc_wgrad",
             (256, 768, 1): "qkv_wgrad"}

    def __init__(self, K, valid_by_T, sq_by_T):
        self.K, self.valid_by_T, self.sq_by_T = K, valid_by_T, sq_by_T
        self.phase = None
        self.rec = []  # (op, start event, end event, flop)
        self._streams = {}
        self._orig = {n: getattr(K, n) for n in self.FNS}

    def _stream(self, handle):
        if handle is None:
            return torch.cuda.current_stream()
        s = self._streams.get(handle)
        if s is None:
            s = self._streams[handle] = torch.cuda.ExternalStream(handle)
        return s

    def _label(self, name, a, kw):
        if name == "attn_fwd":  # (qkv, lens, batch, seq_len, heads, d_head, scale)
            return "attention", 4.0 * a[4] * a[5] * self.sq_by_T.get(a[3], a[2] * a[3] * a[3])
        if name == "attn_bwd":  # (qkv, o, d_o, lse, lens, batch, seq_len, heads, d_head, scale)
            return "attention_bwd", 10.0 * a[7] * a[8] * self.sq_by_T.get(a[6], a[5] * a[6] * a[6])
        if name in ("ln_fwd", "ln_bwd"):
            return name, 0.0
        if name == "conv_wgrad_k1_multi":  # (jobs, rows, seq_len): w_2 + fc + QKV, one launch
            jobs, rows, T = a[0], a[1], a[2]
            r = self.valid_by_T.get(T, rows) if kw.get("lens") is not None else rows
            names = "+".join(self.WGRAD.get((j[4], j[5], 1), "k1").replace("_wgrad", "") for j in jobs)
            return f"{names}_wgrad(grouped)", sum(2.0 * r * j[4] * j[5] for j in jobs)
        rows, T, c_in, c_out, taps = a[2], a[3], a[4], a[5], a[6]
        if name == "conv_wgrad":
            rows, T, c_in, c_out, taps = a[3], a[4], a[5], a[6], a[7]
        r = self.valid_by_T.get(T, rows) if kw.get("lens") is not None else rows
        fl = 2.0 * r * c_in * c_out * taps
        key = (c_in, c_out, taps)
        if name == "conv_wgrad":
            return self.WGRAD.get(key, f"wgrad{key}"), fl
        if name == "conv_gemm_ln":
            return self.FWD.get(key, f"gemm{key}") + "+ln", fl
        if name == "conv_gemm_ln_bwd":
            return "qkv_dgrad+ln2_bwd", fl
        tab = self.FWD if self.phase == "fwd" else self.BWD
        return tab.get(key, f"gemm{key}"), fl

    def install(self):
        me = self

        def wrap(name, fn):
            def f(*a, **kw):
                if me.phase is None:
                    return fn(*a, **kw)
                op, fl = me._label(name, a, kw)
                st = me._stream(kw.get("on_stream"))
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(st)
                y = fn(*a, **kw)
                e.record(st)
                me.rec.append((("fwd:" if me.phase == "fwd" else "bwd:") + op, s, e, fl))
                return y
            return f
        for n, fn in self._orig.items():
            setattr(self.K, n, wrap(n, fn))

    def table(self, blocks, peak, wall_ms):
        torch.cuda.synchronize()
        agg = {}
        for op, s, e, fl in self.rec:
            a = agg.setdefault(op, [0.0, 0.0, 0])
            a[0] += s.elapsed_time(e)
            a[1] += fl
            a[2] += 1
        out, tot = {}, 0.0
        for op, (ms, fl, n) in agg.items():
            per = ms / blocks
            tot += per
            d = {"ms_per_block": round(per, 4), "calls_per_block": round(n / blocks, 2),
                 "share_of_block": round(per / wall_ms, 3) if wall_ms else None}
            if fl > 0:
                d["gflop"] = round(fl / blocks / 1e9, 2)
                d["frac"] = round(fl / (ms / 1e3) / 1e12 / peak, 4)
            out[op] = d
        return out, round(tot, 4)


# ----------------------------------------------------------------------------- PMC traffic
def probe_conv(reps=10):
    """The decoder-shaped launches of the k=9 class alone (forward h = relu(conv(x1) + b) and
    the data gradient dx1 += conv^T(dh), same shapes / epilogues / lens as the step), for
    the PMC passes of ``hbm_traffic``."""
    K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
    syn = PKG.data.syn_batch(48, 128, seed=0)
    M_, T_ = 48 * int(syn[8]), int(syn[8])
    dev = torch.device("cuda", 0)
    lens = torch.tensor(syn[7], device=dev)
    x = torch.randn(M_, D, device=dev).to(torch.bfloat16)
    w = (torch.randn(F * D * KW, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(F, device=dev)
    dh = torch.randn(M_, F, device=dev).to(torch.bfloat16)
    dx = torch.randn(M_, D, device=dev)
    for _ in range(reps):
        K.conv_gemm(x, w, M_, T_, D, F, KW, 4, bias=b, flags=K.EPI_RELU, out_dtype=torch.bfloat16,
                    lens=lens)
        K.conv_gemm(dh, w, M_, T_, F, D, KW, 4, flags=K.EPI_ADD_AUX, aux=dx, out=dx, lens=lens)
    torch.cuda.synchronize()


def probe_wgrad(reps=10):
    """The decoder-shaped launches of the k=9 weight-gradient class alone (dW1 += dh^T x1~ with
    the fused bias gradient, lens as in the step), for the PMC passes of ``hbm_traffic``."""
    K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
    syn = PKG.data.syn_batch(48, 128, seed=0)
    M_, T_ = 48 * int(syn[8]), int(syn[8])
    dev = torch.device("cuda", 0)
    lens = torch.tensor(syn[7], device=dev)
    valid = (torch.arange(T_, device=dev)[None] < lens[:, None]).reshape(-1, 1)
    x = (torch.randn(M_, D, device=dev) * valid).to(torch.bfloat16)
    dh = (torch.randn(M_, F, device=dev) * valid).to(torch.bfloat16)
    dw = torch.zeros(F, D, KW, device=dev)
    db = torch.zeros(F, device=dev)
    for _ in range(reps):
        K.conv_wgrad(dh, x, dw, M_, T_, D, F, KW, 4, db=db, lens=lens)
    torch.cuda.synchronize()


def probe_wgrad_alg_bytes(syn):
    """Compulsory bytes of one k=9 weight-gradient launch: the valid rows of dh (V x 1024 bf16)
    and of x (V x 256 bf16) read once, dW (1024 x 2304 fp32) read and written (accumulated)."""
    V = int(np.sum(syn[7]))
    return V * F * 2 + V * D * 2 + 2 * F * D * KW * 4


def probe_alg_bytes(syn):
    """Compulsory bytes of the probe's two launches (mean per launch): forward reads the
    valid rows of x (V x 256 bf16) and the weight (1024 x 2304 bf16) once and writes every
    row of h (N x 1024 bf16); the data gradient reads the valid rows of dh (V x 1024 bf16),
    the weight, and reads + writes dx (N x 256 fp32)."""
    V, N = int(np.sum(syn[7])), 48 * int(syn[8])
    wb = F * D * KW * 2
    fwd = V * D * 2 + wb + N * F * 2
    dgr = V * F * 2 + wb + 2 * N * D * 4
    return (fwd + dgr) // 2


def hbm_traffic(timeout=300, kind="conv"):
    """Per-launch memory-side bytes of the probe's k=9 conv (kind "conv") or weight-gradient
    (kind "wgrad") launches from rocprofv3 PMC
    counters: FETCH_SIZE and WRITE_SIZE (KiB) in separate passes (they do not fit one TCC
    pass), FETCH_SIZE doubled (gfx950 reports half the bytes of 16-B-per-lane streaming
    reads; MI355X_MICROARCH.md, HBM).  These count L2 misses, Infinity-Cache hits included."""
    import csv
    import glob
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    per = {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as tmp:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", ctr, "-d", d, "-o",
                   "probe", "--output-format", "csv", "--", sys.executable,
                   os.path.abspath(__file__), "--probe-" + kind]
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 30)
            except subprocess.TimeoutExpired:
                return None, f"{ctr} pass timed out"
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None, f"{ctr} pass failed (rc {r.returncode})"
            # per kernel kind: a split-K weight gradient is two launches (partials + the
            # in-order reduce), so its bytes per call are the sum of the two kinds' means
            kinds = ({"main": ("conv_gemm_halo", "conv_gemm_tapreg")} if kind == "conv" else
                     {"main": ("conv_wgrad_band", "conv_wgrad_halo", "conv_wgrad_wide"),
                      "reduce": ("wgrad_reduce", "wgrad_k1_multi_reduce")})
            vals = {k: [] for k in kinds}
            for row in csv.DictReader(open(files[0])):
                kn = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != ctr:
                    continue
                for k, names in kinds.items():
                    if any(n in kn for n in names):
                        vals[k].append(float(row["Counter_Value"]))
                        break
            if not vals["main"]:
                return None, f"{ctr}: no {kind} dispatches"
            per[ctr] = float(sum(np.mean(v) for v in vals.values() if v))
    return (per["FETCH_SIZE"] * 2.0 + per["WRITE_SIZE"]) * 1024.0, per


# ----------------------------------------------------------------------------- CPU baseline
def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(batch_np, steps=3):
    from oracle import fs2_cpu
    n_thr = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    torch.set_num_threads(n_thr)
    ref, _ = fs2_cpu.build("JVS-VCTK")
    ref.train()
    opt = fs2_cpu.make_opt(ref)
    b = PKG.data.to_device(batch_np, "cpu")
    fs2_cpu.train_step(ref, opt, b)  # warm-up
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fs2_cpu.train_step(ref, opt, b)
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    frames = int(np.sum(batch_np[7]))
    return {"value": round(frames / med, 1), "unit": "mel-frames/s",
            "cores": torch.get_num_threads(), "kind": "port", "cpu_model": _cpu_model(),
            "sample": f"oracle/fs2_cpu.py train step (dropout on), SYN-{len(batch_np[4])} seed 0: "
                      f"median of {steps} timed steps after 1 warm-up "
                      f"({', '.join(f'{t:.2f}' for t in ts)} s)"}


# ----------------------------------------------------------------------------- main
def build_trainer(M, TR, dtype, dev, rank, graph=False, data_parallel=None):
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    cdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dtype]
    # the random init draws from torch's global generator: seed it so final_loss reproduces
    # across runs (data parallel: rank 0's weights are broadcast at the first step anyway)
    torch.manual_seed(1234)
    model = M.FastSpeech2(pp, mc, path, device=dev, compute_dtype=cdt)
    model.train()
    model.seed(1234 + rank)
    return model, TR.Trainer(model, pp, mc, tc, graph=graph, data_parallel=data_parallel), tc


def launch_check(world, rank):
    """--launch-check: the rank set the launcher produced (gloo, CPU only)."""
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.ones(1)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world": world, "ranks_seen": int(t.item()), "parallelism": f"dp{world}"}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


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
    ap.add_argument("--no-f32", action="store_true", help="skip the fp32 companion measurement")
    ap.add_argument("--per-kernel-issue", action="store_true",
                    help="A/B: issue the FFT blocks kernel by kernel from Python (model.C_BLOCKS off)")
    ap.add_argument("--graph", action="store_true",
                    help="N=1: capture the step once into a HIP graph and replay it (measured "
                         "slower than eager here: replay serialises the weight-gradient stream)")
    ap.add_argument("--use-clf", action="store_true",
                    help="BASELINE config 3: the --use_clf step (second forward with shuffled "
                         "speakers + GE2E language discriminator on 150-frame chunks)")
    ap.add_argument("--probe-conv", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--probe-wgrad", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.probe_wgrad:
        probe_wgrad()
        return
    if args.probe_conv:
        probe_conv()
        return 0

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:  # no launcher: start one process per GPU (nothing touched the GPU yet)
            return launch_ranks(args.gpus, sys.argv[1:])
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}",
              file=sys.stderr)
        return 2
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        launch_check(world, rank)
        return 0

    if torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but {torch.cuda.device_count()} GPUs", file=sys.stderr)
        return 2
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
    TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    if args.per_kernel_issue:
        M.C_BLOCKS = False
    # FS2_TUNE="knob=value,...": kernel-selection knobs (include/fs2hip.h) for A/B runs
    for kv in filter(None, os.environ.get("FS2_TUNE", "").split(",")):
        knob, val = kv.split("=")
        K.lib.fs2_set_tuning(int(knob), int(val))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # FS2_DP1=1 (A/B): at N = 1, run the step through the data-parallel path on a one-rank
    # RCCL group (global denominators, bucketed all-reduce from the weight-gradient stream) to
    # price that machinery without the interconnect
    dp1 = world == 1 and os.environ.get("FS2_DP1") == "1"
    if world > 1 or dp1:
        if dp1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            TR.init_data_parallel(dev, rank=0, world_size=1)
        else:
            TR.init_data_parallel(dev)

    use_graph = world == 1 and args.graph and not dp1
    model, trainer, tc = build_trainer(M, TR, args.dtype, dev, rank,
                                       graph=use_graph and not args.use_clf,
                                       data_parallel=True if dp1 else None)
    if args.use_clf:
        import random
        G = importlib.import_module("mid-attribute-speaker-generation_amd.ge2e")
        disc = G.SpeechEmbedder(device=dev)
        PKG.seeded.load_seeded_(disc)
        clf = (disc, G.GE2ELoss(dev))
        # under data parallelism the shuffle is one permutation of the global batch, drawn with
        # the same seed on every rank (train.clf_backward gathers the speakers it indexes)
        rnd = random.Random(1234)
        counter = [0]
        n_perm = world * args.batch

        def clf_kw():  # train.py:171 draws the shuffle with random.sample each step
            counter[0] += 1
            return {"clf": clf, "clf_args": (rnd.sample(range(n_perm), n_perm),
                                             counter[0], tc["step"]["total_step"],
                                             float(tc.get("lambda", 1)))}
    batch_np = PKG.data.syn_batch(args.batch, args.src_len, seed=rank)
    batch = PKG.data.to_device(batch_np, dev)
    frames_local = int(np.sum(batch_np[7]))
    T_m, T_s = int(batch_np[8]), int(batch_np[5])
    padded_local = int(args.batch * T_m)
    mel = np.asarray(batch_np[7], np.float64)
    src = np.asarray(batch_np[4], np.float64)
    timer = ClassTimer(K, {T_m: frames_local, T_s: int(src.sum())},
                       {T_m: float((mel ** 2).sum()), T_s: float((src ** 2).sum())})
    if not args.no_roofline and not use_graph:
        timer.install()

    kw = (lambda: clf_kw()) if args.use_clf else (lambda: {})
    n_warm = max(args.warmup, 2 if use_graph else 0)  # graph: step 1 captures
    survey = 3 if (not args.no_roofline and not use_graph and n_warm >= 4) else 0
    # The FFT blocks are issued from C (model.C_BLOCKS) in the measured steps; the per-class and
    # per-op attributions need a Python-side event around every kernel, so their steps run the
    # per-kernel host path: the same kernels in the same order (bitwise the same step,
    # tests/test_gpu_parity.py::test_c_blocks_step_bitwise), only the host issue differs.
    c_blocks = M.C_BLOCKS
    for i in range(n_warm):
        if survey and i == n_warm - survey:
            M.C_BLOCKS = False
            timer.reset("all", 600 * survey)  # class survey: the last warm-up steps
        trainer.step(batch, **kw())
    M.C_BLOCKS = c_blocks
    torch.cuda.synchronize()
    classes, dom = None, None
    if survey:
        classes = timer.table(survey, PEAK[args.dtype][0])
        dom = max(classes, key=lambda c: classes[c]["ms_per_step"])
        timer.mode = None
        for _ in range(2):  # settle after the instrumented steps
            trainer.step(batch, **kw())
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = trainer.step(batch, **kw())[0]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    timed = None
    if dom:
        # the dominant class alone, its launches between HIP events, over as many further steps
        # on the per-kernel host path
        n_dom = min(args.steps, 10)
        M.C_BLOCKS = False
        timer.reset(dom, 200 * n_dom)
        for _ in range(n_dom):
            trainer.step(batch, **kw())
        torch.cuda.synchronize()
        timed = timer.table(n_dom, PEAK[args.dtype][0])
        M.C_BLOCKS = c_blocks
    timer.mode = None
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    fr = torch.tensor([frames_local], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(fr)
    dt, frames = float(t.item()), float(fr.item())
    loss_now = float(losses[0].detach())
    ms_step = dt / args.steps * 1e3
    peak, unit = PEAK[args.dtype]

    out = None
    if rank == 0:
        roof = None
        if timed and dom in timed:
            c = timed[dom]
            roof = {"bound": "mfma", "achieved": c["tflops"], "peak": peak, "unit": unit,
                    "frac": c["frac"], "traffic": None,
                    "kernel": f"{dom}: the step's dominant launch set by in-step time "
                              f"({c['launches_per_step']} launches/step, {c['ms_per_step']} ms/step "
                              "in steps after the timed region, per-kernel host path)",
                    "flop_basis": "2 * valid frames * C_out * C_in * taps per launch (kernels "
                                  "skip all-padding row tiles)",
                    "per_launch_flop": round(c["gflop_per_step"] * 1e9 / c["launches_per_step"]),
                    "avg_launch_ms": c["avg_launch_ms"]}
            if dom in ("conv_k9", "wgrad_k9") and world == 1 and args.dtype == "bf16" and \
                    not args.no_traffic:
                kind = "conv" if dom == "conv_k9" else "wgrad"
                traffic, detail = hbm_traffic(kind=kind)
                if traffic is not None:
                    syn0 = PKG.data.syn_batch(48, 128, seed=0)
                    roof["traffic"] = round(traffic)
                    roof["traffic_unit"] = (
                        "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, PMC) of the class's decoder-shaped "
                        + ("fwd + data-gradient launches" if kind == "conv" else "weight-gradient launches"))
                    roof["traffic_algorithmic"] = (probe_alg_bytes(syn0) if kind == "conv"
                                                   else probe_wgrad_alg_bytes(syn0))
                else:
                    roof["traffic_note"] = detail
            roof["classes"] = classes
            roof["classes_basis"] = ("every class timed in the last 3 warm-up steps (events on "
                                     "~170 launches make those steps host-bound); the dominant "
                                     "class alone over up to 10 steps after the timed region; "
                                     "both on the per-kernel host path (model.C_BLOCKS off: the "
                                     "same kernels, issued one by one from Python)")
        step_roof = {"gflop_padded": STEP_GFLOP_PADDED, "achieved": None, "frac": None}
        if args.batch == 48 and args.src_len == 128 and not args.use_clf:
            ach = STEP_GFLOP_PADDED / (ms_step / 1e3) / 1e3
            step_roof = {"gflop_padded": STEP_GFLOP_PADDED, "achieved": round(ach, 1),
                         "unit": unit, "peak": peak, "frac": round(ach / peak, 4)}
        out = {"metric": METRIC, "value": round(frames * args.steps / dt, 1), "unit": "mel-frames/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(ms_step, 3), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic SYN-B (seeded, rank r uses seed r), random-init weights",
               "config": {"workload": f"SYN-{args.batch}: FastSpeech2+TacoSpawn train step, "
                                      f"B={args.batch}/GPU, {args.src_len} phonemes x "
                                      f"{T_m} frames padded",
                          "global_batch": args.batch * world, "seq_len": T_m,
                          "valid_frames_per_rank_step": frames_local,
                          "padded_frames_per_rank_step": padded_local,
                          "parallelism": f"dp{world}",
                          "use_clf": bool(args.use_clf),
                          "execution": "hip-graph replay" if use_graph else "eager",
                          "host_issue": ("one C-ABI call per FFT block, mel head and variance "
                                         "predictor (fs2_fft_block_* / fs2_mel_head_* / "
                                         "fs2_variance_predictor_*)"
                                         if M.C_BLOCKS else "one C-ABI call per kernel"),
                          **({"data_parallel": "one-rank RCCL group (FS2_DP1)"} if dp1 else {})},
               "roofline": roof, "step_roofline": step_roof}

    # decoder FFT block fwd + bwd, 3 extra steps (rank 0's figures; every rank runs them so
    # collectives stay matched)
    if not args.no_roofline and not use_graph and not args.use_clf:
        bt = BlockTimer(M, model)
        bt.on = True
        for _ in range(3):
            trainer.step(batch)
        bt.on = False
        f_ms, b_ms = bt.result()
        if rank == 0 and f_ms is not None:
            L = len(model.decoder.layer_stack)
            blk_ms = (f_ms + b_ms) / L
            per_block_fwd_valid = frames_local * (8 * D * D + 2 * KW * D * F + 2 * F * D) + \
                4 * D * float((mel ** 2).sum())
            gf_valid = 3 * per_block_fwd_valid / 1e9
            gf_pad = DEC_BLOCK_GFLOP_PADDED if (args.batch == 48 and T_m == 512) else None
            fb = {"fwd_ms_per_block": round(f_ms / L, 4), "bwd_ms_per_block": round(b_ms / L, 4),
                  "gflop_valid": round(gf_valid, 1), "unit": unit, "peak": peak,
                  "achieved_valid": round(gf_valid / blk_ms, 1),
                  "frac_valid": round(gf_valid / blk_ms / peak, 4),
                  "basis": "HIP events around DecoderFn forward / backward (+ its side-stream "
                           "weight gradients joined) in 3 steps after the timed region, median, "
                           "/ 6 layers"}
            if gf_pad:
                fb.update(gflop_padded=gf_pad, achieved_padded=round(gf_pad / blk_ms, 1),
                          frac_padded=round(gf_pad / blk_ms / peak, 4))
            out["fft_block"] = fb
        # per-op attribution of the block: 3 more steps with every decoder kernel call timed
        ot = OpTimer(K, {T_m: frames_local, T_s: int(src.sum())},
                     {T_m: float((mel ** 2).sum()), T_s: float((src ** 2).sum())})
        ot.install()
        bt.ops, bt.ev, bt.on = ot, [], True
        M.C_BLOCKS = False  # every kernel call between events: the per-kernel host path
        for _ in range(3):
            trainer.step(batch)
        M.C_BLOCKS = c_blocks
        bt.on, bt.ops = False, None
        for n, fn in ot._orig.items():
            setattr(K, n, fn)
        f2, b2 = bt.result()
        if rank == 0 and f_ms is not None and f2 is not None:
            L = len(model.decoder.layer_stack)
            wall = (f2 + b2) / L
            ops, tot = ot.table(3 * L, peak, wall)
            out["fft_block"]["ops"] = ops
            out["fft_block"]["ops_basis"] = (
                "3 further steps, every kernel call inside DecoderFn forward / backward between HIP "
                "events on its own stream (weight gradients: the side stream, concurrent with the "
                "main-stream chain), after a spin kernel that puts the GPU behind the host; "
                "ms per block = total / (3 steps x 6 layers); frac on valid-frame FLOP")
            out["fft_block"]["ops_wall_ms_per_block"] = round(wall, 4)
            out["fft_block"]["ops_sum_ms_per_block"] = tot

    # the reference's precision (fp32), N = 1, a short companion measurement
    if world == 1 and args.dtype == "bf16" and not args.no_f32 and not args.use_clf:
        del trainer, model
        torch.cuda.empty_cache()
        m32, tr32, _ = build_trainer(M, TR, "f32", dev, rank)
        for _ in range(2):
            tr32.step(batch)
        torch.cuda.synchronize()
        n32 = 5
        t0 = time.perf_counter()
        for _ in range(n32):
            tr32.step(batch)
        torch.cuda.synchronize()
        d32 = time.perf_counter() - t0
        ach = STEP_GFLOP_PADDED / (d32 / n32) / 1e3
        out["f32"] = {"value": round(frames_local * n32 / d32, 1), "unit": "mel-frames/s",
                      "ms_per_step": round(d32 / n32 * 1e3, 3), "steps": n32, "warmup": 2,
                      "step_frac_of_f32_peak": round(ach / PEAK["f32"][0], 4)}

    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(batch_np)
        else:
            out["cpu_baseline"] = None
        out["final_loss"] = round(loss_now, 5)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
