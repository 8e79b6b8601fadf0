"""Time the k >= 3 Conv1d kernels of the step alone at their step shapes (SYN-48 lengths):
forward, data gradient and weight gradient (+ its split reduce), then the data gradient and
the weight gradient together on two streams as the step runs them (the weight gradients ride
a side stream), to show what the overlap costs each.

    python scripts/conv_bench.py [--reps 20] [--only dec] [--ab KNOB=V0/V1] [--abw KNOB=V0/V1]

--ab: forward and data gradient under fs2_set_tuning(KNOB, V0) and (KNOB, V1), alternating
three times, with a bitwise comparison of the two outputs.
"""
import importlib
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
dev = "cuda:0"
_b = PKG.data.syn_batch(48, 128, seed=0)
LENS = {512: torch.tensor(_b[7], device=dev), 128: torch.tensor(_b[4], device=dev)}
VALID = {512: int(np.sum(_b[7])), 128: int(np.sum(_b[4]))}
bf = torch.bfloat16

# name, T, cin, cout, taps, count per step
SHAPES = [
    ("dec w1 k9", 512, 256, 1024, 9, 6),
    ("enc w1 k9", 128, 256, 1024, 9, 4),
    ("postnet 512 k5", 512, 512, 512, 5, 3),
    ("postnet in k5", 512, 80, 512, 5, 1),
    ("postnet out k5", 512, 512, 80, 5, 1),
    ("vp k3 T128", 128, 256, 256, 3, 4),
    ("vp k3 T512", 512, 256, 256, 3, 2),
    # k = 1 projections (their weight gradients: long-K split GEMMs)
    ("dec qkv k1", 512, 256, 768, 1, 6),
    ("dec fc k1", 512, 256, 256, 1, 6),
    ("dec w2 k1", 512, 1024, 256, 1, 6),
]


def timeit(fn, reps, streams=None):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    if streams:
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def ab(spec, reps, only):
    knob, vals = spec.split("=")
    v0, v1 = (int(v) for v in vals.split("/"))
    knob = int(knob)
    for name, T, cin, cout, k, cnt in SHAPES:
        if only and not name.startswith(only):
            continue
        M, pad = 48 * T, (k - 1) // 2
        lens = LENS[T]
        valid = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
        x = (torch.randn(M, cin, device=dev) * valid[:, None]).to(bf)
        dy = (torch.randn(M, cout, device=dev) * valid[:, None]).to(bf)
        if os.environ.get("NOLENS"):  # every row valid (no padding skips)
            lens = None
        w = torch.randn(cout, cin, k, device=dev) / math.sqrt(cin * k)
        wf = torch.empty(cout * cin * k, device=dev, dtype=bf)
        wb = torch.empty_like(wf)
        K.weight_prep(w, cout, cin, k, wf, wb)
        bias = torch.randn(cout, device=dev)
        aux = torch.randn(M, cin, device=dev)
        ys = {v: torch.empty(M, cout, device=dev, dtype=bf) for v in (v0, v1)}
        dxs = {v: torch.empty(M, cin, device=dev) for v in (v0, v1)}
        res = {}
        for v in (v0, v1, v0, v1, v0, v1):
            K.lib.fs2_set_tuning(knob, v)
            fwd = lambda: K.conv_gemm(x, wf, M, T, cin, cout, k, pad, bias=bias,
                                      flags=K.EPI_RELU, out=ys[v], lens=lens)
            dgr = lambda: K.conv_gemm(dy, wb, M, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX,
                                      aux=aux, out=dxs[v], lens=lens)
            for _ in range(20):
                fwd()
                dgr()
            res.setdefault(v, []).append((timeit(fwd, reps), timeit(dgr, reps)))
        K.lib.fs2_set_tuning(knob, 0)
        eq_f = torch.equal(ys[v0], ys[v1])
        eq_d = torch.equal(dxs[v0], dxs[v1])
        fl = 2.0 * VALID[T] * cin * cout * k / 1e6
        line = f"{name:15s}"
        for v in (v0, v1):
            tf = min(r[0] for r in res[v])
            td = min(r[1] for r in res[v])
            line += f"  [{knob}={v}] fwd {tf:6.1f} us ({fl / tf:4.0f} TF/s) dgrad {td:6.1f} ({fl / td:4.0f})"
        print(line + f"  bitwise fwd {eq_f} dgrad {eq_d}", flush=True)


def abw(spec, reps, only):
    """weight gradient (+ reduce) under two knob values, alternating; dW compared bitwise"""
    knob, vals = spec.split("=")
    v0, v1 = (int(v) for v in vals.split("/"))
    knob = int(knob)
    for name, T, cin, cout, k, cnt in SHAPES:
        if only and not name.startswith(only):
            continue
        M, pad = 48 * T, (k - 1) // 2
        lens = LENS[T]
        valid = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
        x = (torch.randn(M, cin, device=dev) * valid[:, None]).to(bf)
        dy = (torch.randn(M, cout, device=dev) * valid[:, None]).to(bf)
        dws = {v: torch.zeros(cout, cin, k, device=dev) for v in (v0, v1)}
        dbs = {v: torch.zeros(cout, device=dev) for v in (v0, v1)}
        res = {}
        for v in (v0, v1, v0, v1, v0, v1):
            K.lib.fs2_set_tuning(knob, v)
            wsb = K.ws(K.lib.fs2_conv_wgrad_ws_bytes(M, cin, cout, k), dev)
            wgr = lambda: K.conv_wgrad(dy, x, dws[v], M, T, cin, cout, k, pad, db=dbs[v],
                                       ws_buf=wsb, lens=lens)
            dws[v].zero_()
            dbs[v].zero_()
            wgr()
            torch.cuda.synchronize()
            snap = (dws[v].clone(), dbs[v].clone())
            for _ in range(20):
                wgr()
            res.setdefault(v, []).append(timeit(wgr, reps))
            dws[v].copy_(snap[0])
            dbs[v].copy_(snap[1])
        K.lib.fs2_set_tuning(knob, 0)
        eq = torch.equal(dws[v0], dws[v1]) and torch.equal(dbs[v0], dbs[v1])
        fl = 2.0 * VALID[T] * cin * cout * k / 1e6
        line = f"{name:15s}"
        for v in (v0, v1):
            t = min(res[v])
            line += f"  [{knob}={v}] wgrad+reduce {t:6.1f} us ({fl / t:4.0f} TF/s)"
        print(line + f"  bitwise {eq}", flush=True)


def probe(kind, only):
    """10 launches of one kernel (PMC passes): --probe fwd|dgrad|wgrad --only <shape>"""
    name, T, cin, cout, k, _ = [s_ for s_ in SHAPES if s_[0].startswith(only or "dec")][0]
    M, pad = 48 * T, (k - 1) // 2
    lens = LENS[T]
    valid = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
    x = (torch.randn(M, cin, device=dev) * valid[:, None]).to(bf)
    dy = (torch.randn(M, cout, device=dev) * valid[:, None]).to(bf)
    w = torch.randn(cout, cin, k, device=dev) / math.sqrt(cin * k)
    wf = torch.empty(cout * cin * k, device=dev, dtype=bf)
    wb = torch.empty_like(wf)
    K.weight_prep(w, cout, cin, k, wf, wb)
    if kind == "fwd":
        y = torch.empty(M, cout, device=dev, dtype=bf)
        bias = torch.randn(cout, device=dev)
        run = lambda: K.conv_gemm(x, wf, M, T, cin, cout, k, pad, bias=bias, flags=K.EPI_RELU,
                                  out=y, lens=lens)
    elif kind == "dgrad":
        dx = torch.empty(M, cin, device=dev)
        run = lambda: K.conv_gemm(dy, wb, M, T, cout, cin, k, pad, out=dx, lens=lens)
    else:
        dw = torch.zeros(cout, cin, k, device=dev)
        wsb = K.ws(K.lib.fs2_conv_wgrad_ws_bytes(M, cin, cout, k), dev)
        run = lambda: K.conv_wgrad(dy, x, dw, M, T, cin, cout, k, pad, ws_buf=wsb, lens=lens)
    for _ in range(10):
        run()
    torch.cuda.synchronize()


def main():
    for kv in filter(None, os.environ.get("FS2_TUNE", "").split(",")):  # "knob=value,..."
        kn, v = kv.split("=")
        K.lib.fs2_set_tuning(int(kn), int(v))
    if "--probe" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
        probe(sys.argv[sys.argv.index("--probe") + 1], only)
        return
    if "--ab" in sys.argv:
        reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 20
        only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
        ab(sys.argv[sys.argv.index("--ab") + 1], reps, only)
        return
    if "--abw" in sys.argv:
        reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 20
        only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
        abw(sys.argv[sys.argv.index("--abw") + 1], reps, only)
        return
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 20
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    side = torch.cuda.Stream()
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "pair": 0.0}
    for name, T, cin, cout, k, cnt in SHAPES:
        if only and not name.startswith(only):
            continue
        M, pad = 48 * T, (k - 1) // 2
        lens = LENS[T]
        valid = (torch.arange(T, device=dev)[None] < lens[:, None]).reshape(-1)
        x = (torch.randn(M, cin, device=dev) * valid[:, None]).to(bf)
        dy = (torch.randn(M, cout, device=dev) * valid[:, None]).to(bf)
        w = torch.randn(cout, cin, k, device=dev) / math.sqrt(cin * k)
        wf = torch.empty(cout * cin * k, device=dev, dtype=bf)
        wb = torch.empty_like(wf)
        K.weight_prep(w, cout, cin, k, wf, wb)
        y = torch.empty(M, cout, device=dev, dtype=bf)
        dx = torch.empty(M, cin, device=dev)
        dw = torch.zeros(cout, cin, k, device=dev)
        db = torch.zeros(cout, device=dev)
        bias = torch.randn(cout, device=dev)
        wsb = K.ws(K.lib.fs2_conv_wgrad_ws_bytes(M, cin, cout, k), dev)
        fwd = lambda: K.conv_gemm(x, wf, M, T, cin, cout, k, pad, bias=bias, flags=K.EPI_RELU,
                                  out=y, lens=lens)
        dgr = lambda: K.conv_gemm(dy, wb, M, T, cout, cin, k, pad, out=dx, lens=lens)
        wgr = lambda: K.conv_wgrad(dy, x, dw, M, T, cin, cout, k, pad, db=db, ws_buf=wsb,
                                   lens=lens)

        def wgr_side():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                wgr()

        def pair():
            wgr_side()
            dgr()

        # parity of the weight gradient on valid rows (fp32 reference of the bf16 operands)
        dw.zero_()
        db.zero_()
        wgr()
        xp = torch.nn.functional.pad(x.float().view(48, T, cin), (0, 0, pad, pad))
        cols = torch.stack([xp[:, j:j + T] for j in range(k)], -1).reshape(M, cin, k)
        ref = torch.einsum("mo,mck->ock", dy.float(), cols)
        err = ((dw - ref).abs().max() / ref.abs().max()).item()
        for _ in range(50):  # clocks settle
            pair()
        t_f = timeit(fwd, reps)
        t_d = timeit(dgr, reps)
        t_w = timeit(wgr, reps)
        t_p = timeit(pair, reps, [side])
        fl = 2.0 * VALID[T] * cin * cout * k / 1e6
        print(f"{name:15s} fwd {t_f:7.1f} us ({fl / t_f:4.0f} TF/s)  dgrad {t_d:7.1f} "
              f"({fl / t_d:4.0f})  wgrad+reduce {t_w:7.1f} ({fl / t_w:4.0f})  dgrad||wgrad "
              f"{t_p:7.1f} (sum {t_d + t_w:7.1f})  x{cnt}  wgrad err {err:.1e}", flush=True)
        for key, v in (("fwd", t_f), ("dgrad", t_d), ("wgrad", t_w), ("pair", t_p)):
            tot[key] += v * cnt
    print("per step (us): " + "  ".join(f"{k_} {v:.0f}" for k_, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
