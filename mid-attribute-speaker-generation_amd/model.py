"""FastSpeech2 + TacoSpawn GMM, host side: the reference's module API on HIP kernels.

Drop-in for ``model.fastspeech2.FastSpeech2`` (``model/fastspeech2.py:15-341``): same
constructor ``(preprocess_config, model_config, config_path)``, same ``forward`` signature
and 12-tuple, same 242 state-dict keys and shapes, same ``model.parameters()`` order (so a
reference checkpoint and its Adam state load unchanged).  Every tensor op of the training
path runs in ``csrc/libfs2hip.so``; the submodules here are parameter containers plus a
hand-written forward/backward per block, wired to autograd at block granularity:

  EncoderFn        embed + 4 FFT blocks               (transformer/Models.py:77-112)
  VarianceAdaptorFn speaker add, 3 predictors, bucketized pitch/energy embeddings,
                   LengthRegulator + decoder position encoding
                                                      (fastspeech2.py:80-85, modules.py:102-194,
                                                       Models.py:165-174)
  DecoderFn        6 FFT blocks                       (transformer/Models.py:151-183)
  MelHeadFn        mel_linear + PostNet + residual    (fastspeech2.py:109-111, Layers.py:67-137)
  (loss.py)        FastSpeech2Loss, GMM log-likelihood

Parameters live in one flat fp32 buffer (``ParamArena``), laid out in reverse backward
order so gradient buckets complete front-to-back; kernels accumulate weight gradients
straight into the flat gradient buffer (``param.grad`` are views of it).
"""
import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import config as cfg
from . import kernels as K

D_HEAD = 128

# ----------------------------------------------------------------------------- containers


class Linear(nn.Module):
    def __init__(self, d_in, d_out, bias=True):
        super().__init__()
        self.in_features, self.out_features = d_in, d_out
        self.weight = nn.Parameter(torch.empty(d_out, d_in))
        self.bias = nn.Parameter(torch.empty(d_out)) if bias else None
        bound = 1.0 / math.sqrt(d_in)  # nn.Linear default init
        with torch.no_grad():
            nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
            if self.bias is not None:
                self.bias.uniform_(-bound, bound)


class Conv1d(nn.Module):
    def __init__(self, c_in, c_out, k, padding):
        super().__init__()
        self.c_in, self.c_out, self.k, self.padding = c_in, c_out, k, padding
        self.weight = nn.Parameter(torch.empty(c_out, c_in, k))
        self.bias = nn.Parameter(torch.empty(c_out))
        bound = 1.0 / math.sqrt(c_in * k)
        with torch.no_grad():
            nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
            self.bias.uniform_(-bound, bound)


class LayerNorm(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.bias = nn.Parameter(torch.zeros(d))


class Embedding(nn.Module):
    def __init__(self, n, d, padding_idx=None):
        super().__init__()
        self.padding_idx = -1 if padding_idx is None else padding_idx
        self.weight = nn.Parameter(torch.randn(n, d))
        if padding_idx is not None:
            with torch.no_grad():
                self.weight[padding_idx].zero_()


class BatchNorm1d(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


class _ConvWrap(nn.Module):
    """``.conv`` holder: the reference's ``Conv`` (modules.py:253) / ``ConvNorm`` (Layers.py:33)."""

    def __init__(self, c_in, c_out, k, padding):
        super().__init__()
        self.conv = Conv1d(c_in, c_out, k, padding)


def sinusoid_table(n_position, d_hid):
    """``transformer/Models.py:10-30`` (float64 angles, stored float32)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    denom = np.array([np.power(10000, 2 * (j // 2) / d_hid) for j in range(d_hid)])
    ang = pos / denom[None, :]
    tab = np.empty_like(ang)
    tab[:, 0::2] = np.sin(ang[:, 0::2])
    tab[:, 1::2] = np.cos(ang[:, 1::2])
    return torch.from_numpy(tab.astype(np.float32))




# ----------------------------------------------------------------------------- runtime state




# Debug (tests/stale_probe.py --guard): every region handed to a C entry point (activations,
# temporaries, the side-stream workspace) gets a guard tail filled with a pattern and is kept;
# check_guards() names each region whose tail a kernel wrote (an out-of-bounds write).
_GUARD = {"on": False, "regions": []}
_GUARD_BYTES = 1 << 16


def _region(nbytes, device, label):
    nbytes = int(nbytes)
    if not _GUARD["on"]:
        return torch.empty(nbytes, dtype=torch.uint8, device=device)
    t = torch.empty(nbytes + _GUARD_BYTES, dtype=torch.uint8, device=device)
    t[nbytes:].fill_(0x5A)
    _GUARD["regions"].append((t, nbytes, label))
    return t[:nbytes]


def check_guards():
    """Labels of the guarded regions whose guard tail was overwritten (synchronises)."""
    torch.cuda.synchronize()
    return [f"{label} ({n} B)" for t, n, label in _GUARD["regions"] if bool((t[n:] != 0x5A).any())]


class StepCtx:
    """Per-forward state: compute dtype of the GEMM operands, one Philox seed per step (one
    site id per dropout call, assigned at construction)."""

    def __init__(self, seed, training, dropout, cdt=torch.float32):
        self.seed = seed  # device int64[1] tensor (or a host int when no dropout runs)
        self.drop = bool(training and dropout)
        self.cdt = cdt
        self.copy = None if cdt == torch.float32 else cdt  # bf16 compute copies wanted?
        self.hook = None  # gradient-ready callback (data-parallel bucketed all-reduce)
        self.side = None  # stream for the weight-gradient GEMMs (off the critical path)
        self.ws_cache = None  # dict holding the side stream's shared split-K workspace
        self.keep = []  # operands read by side-stream work, released at the next join
        self.k1 = None  # held-back grouped k = 1 weight gradients: (key, jobs, lens)
        self.after_first = None  # issued after the encoder's first block (prep_weights)

    def p(self, p):
        return float(p) if self.drop else 0.0

    def _side_ws(self, need, device):
        # one workspace for every side-stream weight gradient (they run in stream order);
        # allocated on the main stream and only grown outside graph capture, so nothing is
        # allocated on the side stream (a captured graph owns only main-stream allocations)
        need = need // 4 + 1
        ws = self.ws_cache.get("wgrad")
        if ws is None or ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("weight-gradient workspace must be sized before capture")
            K.lib.fs2_stream_wait(K.stream(), self.side.cuda_stream)  # old buffer drained
            ws = self.ws_cache["wgrad"] = _region(need * 4, device, "side_ws").view(torch.float32)
        return ws

    def wgrad(self, dy, x, dw, rows, seq_len, c_in, c_out, taps, pad, db=None, lens=None,
              group=False):
        """Weight (+bias) gradient GEMM.  Nothing in the backward waits for it, so with a
        side stream it runs concurrently with the data-gradient chain on the main stream
        (the small GEMMs of a block fill the GPU together); ``join`` orders it back.
        ``group`` (k = 1 only): held back and issued with the other grouped k = 1 weight
        gradients of the same rows as ONE grouped launch at ``flush`` (fs2_conv_wgrad_k1_multi)."""
        if group and taps == 1:
            key = (rows, seq_len, None if lens is None else lens.data_ptr())
            if self.k1 and (self.k1[0] != key or len(self.k1[1]) == 4):
                self.flush()
            if not self.k1:
                self.k1 = (key, [], lens)
            self.k1[1].append((dy, x, dw, db, c_in, c_out))
            return
        if self.side is None:
            return K.conv_wgrad(dy, x, dw, rows, seq_len, c_in, c_out, taps, pad, db=db,
                                lens=lens)
        ws = self._side_ws(K.lib.fs2_conv_wgrad_ws_bytes(rows, c_in, c_out, taps), dy.device)
        side = self.side.cuda_stream
        K.lib.fs2_stream_wait(side, K.stream())
        K.conv_wgrad(dy, x, dw, rows, seq_len, c_in, c_out, taps, pad, db=db, ws_buf=ws,
                     on_stream=side, lens=lens)
        self.keep.append((dy, x))  # not freed (reusable by the main stream) before the join

    def flush(self):
        """Issue the held-back grouped k = 1 weight gradients (one launch + one reduce)."""
        if not self.k1:
            return
        (rows, seq_len, _), jobs, lens = self.k1
        self.k1 = None
        if self.side is None:
            return K.conv_wgrad_k1_multi(jobs, rows, seq_len, lens=lens)
        ws = self._side_ws(K.conv_wgrad_k1_multi_ws_bytes(jobs, rows), jobs[0][0].device)
        side = self.side.cuda_stream
        K.lib.fs2_stream_wait(side, K.stream())
        K.conv_wgrad_k1_multi(jobs, rows, seq_len, lens=lens, ws_buf=ws, on_stream=side)
        self.keep.extend((j[0], j[1]) for j in jobs)

    def join(self):
        """Make the current stream wait for every weight-gradient GEMM issued so far."""
        self.flush()
        if self.side is not None:
            K.lib.fs2_stream_wait(K.stream(), self.side.cuda_stream)
            self.keep.clear()

    def notify(self, params):
        """Tell the gradient hook that these parameters' gradients are final (``params``: a
        list, or a callable returning it -- built only when a hook is installed)."""
        if self.hook is not None:
            self.hook(params() if callable(params) else params)


# bf16 path: FFT-block post-LayerNorms fused into the fc / w_2 GEMM epilogues (fs2_conv_gemm_ln)
# on decoder-sized grids; the bitwise tests compare against the two-launch form by clearing it
FUSE_LN = True
FUSE_LN_MIN_ROWS = 16384
# ... and each block's QKV data gradient carries the previous block's LN2 backward
FUSE_LN_BWD = True
# bf16 path: each FFT block's forward / backward is ONE call into the library
# (fs2_fft_block_fwd / _bwd issue its kernels and stream waits from C, in the order of
# FFTBlock.fwd / .bwd below: bitwise the same results, a fifth of the host time); the tests
# compare it against the per-kernel path by clearing it
C_BLOCKS = True
# pitch and duration predictor forwards on the side stream beside the energy predictor (A/B)
VA_SIDE = True
# fs2_mel_head_* descriptor geometry (include/fs2hip.h: FS2_MH_LAYER0 + FS2_MH_MAX_LAYERS x
# FS2_MHL_WORDS words)
MH_MAX_LAYERS = 8
MH_WORDS = 12 + MH_MAX_LAYERS * 12


def _t(f, t):
    """Compute-dtype view of an activation: the bf16 copy if one was made, else the fp32."""
    return f if t is None else t


def _g(p):
    """Flat-buffer gradient view of parameter ``p`` (set up by ParamArena)."""
    return p._fs2_grad


# Bumped whenever a compute-weight buffer or the parameter arena is (re)allocated: the C-entry
# descriptors (FFTBlock.cdesc, ...) hold raw pointers and are rebuilt when it moves
_GEN = [0]


def _buf(holder, name, n, dtype, device):
    t = getattr(holder, name, None)
    if t is None or t.numel() != n or t.dtype != dtype:
        t = torch.empty(n, dtype=dtype, device=device)
        setattr(holder, name, t)
        _GEN[0] += 1
    return t


class _WeightHolder:
    """Compute-layout weights of a fused projection that has no module of its own (QKV)."""

    def __init__(self, d_in, d_out):
        self.in_features, self.out_features = d_in, d_out


def _prep(w, c_out, c_in, taps, wf, wb, jobs):
    """Launch the re-layout now, or (jobs given) record it for the one-launch batch."""
    if jobs is None:
        K.weight_prep(w, c_out, c_in, taps, wf, wb)
    else:
        jobs.append((w.data_ptr(), c_out, c_in, taps, 0 if wf is None else wf.data_ptr(),
                     0 if wb is None else wb.data_ptr()))


def _linear_prep(lin, cdt, w=None, c_out=None, c_in=None, jobs=None):
    """Compute-layout weights of a Linear: w_fwd (out, in) and its transpose w_bwd (in, out).
    fp32 forward uses the master weight itself."""
    w = lin.weight.detach() if w is None else w
    c_out = lin.out_features if c_out is None else c_out
    c_in = lin.in_features if c_in is None else c_in
    wb = _buf(lin, "_w_bwd", c_in * c_out, cdt, w.device).view(c_in, c_out)
    if cdt == torch.float32:
        lin._w_fwd = w.reshape(c_out, c_in)
        _prep(w, c_out, c_in, 1, None, wb, jobs)
    else:
        wf = _buf(lin, "_w_fwd_b", c_out * c_in, cdt, w.device).view(c_out, c_in)
        lin._w_fwd = wf
        _prep(w, c_out, c_in, 1, wf, wb, jobs)
    lin._w_bwd = wb


def _conv_prep(conv, cdt, jobs=None):
    n = conv.c_out * conv.c_in * conv.k
    wf = _buf(conv, "_w_fwd", n, cdt, conv.weight.device)
    wb = _buf(conv, "_w_bwd", n, cdt, conv.weight.device)
    _prep(conv.weight.detach(), conv.c_out, conv.c_in, conv.k, wf, wb, jobs)


# ----------------------------------------------------------------------------- FFT block


class MultiHeadAttention(nn.Module):
    """Parameters of ``transformer/SubLayers.py:8-57``."""

    def __init__(self, n_head, d_model, d_k, dropout):
        super().__init__()
        self.n_head, self.d_k, self.p = n_head, d_k, dropout
        self.w_qs = Linear(d_model, n_head * d_k)
        self.w_ks = Linear(d_model, n_head * d_k)
        self.w_vs = Linear(d_model, n_head * d_k)
        self.layer_norm = LayerNorm(d_model)
        self.fc = Linear(n_head * d_k, d_model)


class PositionwiseFeedForward(nn.Module):
    """Parameters of ``transformer/SubLayers.py:60-93``."""

    def __init__(self, d_in, d_hid, kernel_size, dropout):
        super().__init__()
        self.p = dropout
        self.w_1 = Conv1d(d_in, d_hid, kernel_size[0], (kernel_size[0] - 1) // 2)
        self.w_2 = Conv1d(d_hid, d_in, kernel_size[1], (kernel_size[1] - 1) // 2)
        self.layer_norm = LayerNorm(d_in)


# Weight-gradient streams created ahead of the communicator, per device index: see
# reserve_streams.  _RESERVED_BEFORE_PG[index]: no process group existed at the reservation.
_RESERVED_SIDE = {}
_RESERVED_BEFORE_PG = {}


def reserve_streams(device):
    """Give the step's two compute streams hardware queues of their own; call it before
    anything else creates streams on ``device`` -- in particular before
    ``dist.init_process_group(..., device_id=...)``, whose RCCL communicator creates streams.

    HIP maps streams onto at most ``GPU_MAX_HW_QUEUES`` hardware queues per priority (4 on
    the MI355X boxes): the first streams created get fresh queues, later ones share the
    least-used queue, ties broken arbitrarily.  Two streams on one queue run in order, so the
    weight-gradient stream sharing the legacy stream's queue serialises the step: the data-
    parallel step on a one-rank group lost 1.9 ms/step (9.3 vs 7.4 ms) in 3 of 4 runs that
    way (profiles/r3_ab_experiments.txt).  This launches on the legacy stream (its queue is
    created on first use) and creates the weight-gradient stream next, so both get fresh
    queues; FastSpeech2.side_stream() then hands out the reserved stream.  It mitigates the
    collision rather than removing it: HIP exposes no way to pin a stream to a queue, and a
    one-rank DP run still measured 8.16 ms once against 7.53 plain (r3_ab_experiments.txt).
    Trainer(data_parallel=True) warns when the reservation did not precede the process group
    (stream_reservation_problem).
    """
    dev = torch.device(device)
    idx = torch.cuda.current_device() if dev.index is None else dev.index
    if idx not in _RESERVED_SIDE:
        import torch.distributed as dist
        _RESERVED_BEFORE_PG[idx] = not (dist.is_available() and dist.is_initialized())
        torch.zeros(1, device=dev).add_(1)  # first use of the legacy stream: its queue
        _RESERVED_SIDE[idx] = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize(dev)
    return _RESERVED_SIDE[idx]


def stream_reservation_problem(device):
    """None if ``device``'s compute streams were reserved (reserve_streams) before any process
    group existed, else what went wrong -- the data-parallel step then risks sharing one hardware
    queue between the two compute streams (+25 % step time, silently; profiles/r3_ab_experiments.txt).
    The reservation mitigates the collision (fresh queues for the first streams); it cannot
    prove which queue a stream landed on."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return None
    idx = torch.cuda.current_device() if dev.index is None else dev.index
    if idx not in _RESERVED_SIDE:
        return (f"cuda:{idx}: the weight-gradient stream was not reserved; call "
                "train.init_data_parallel(device, ...) (or model.reserve_streams(device) before "
                "dist.init_process_group) so the RCCL communicator's streams do not take the "
                "compute streams' hardware queues")
    if not _RESERVED_BEFORE_PG.get(idx, False):
        return (f"cuda:{idx}: the weight-gradient stream was reserved after the process group "
                "was created; the communicator's streams may already share its hardware queue")
    return None


def _flat_view(t, n):
    """A 1-D view of ``n`` elements starting at ``t``'s first element (same storage)."""
    return t.detach().as_strided((n,), (1,), t.storage_offset())


class FFTBlock(nn.Module):
    """``transformer/Layers.py:11-30``: post-LN MHA + Conv1d FFN, padded rows zeroed.

    fwd/bwd take and return activations as (fp32, compute copy) pairs; the fp32 tensor is
    the residual stream, the copy (bf16 on the bf16 path) feeds the next GEMM."""

    def __init__(self, d_model, n_head, d_inner, kernel_size, dropout):
        super().__init__()
        self.d = d_model
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_model // n_head, dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout)
        self.site = 0  # assigned by FastSpeech2

    def prep(self, cdt, jobs=None):
        a, f = self.slf_attn, self.pos_ffn
        n3 = 3 * a.n_head * a.d_k
        wq, bq = a.w_qs.weight, a.w_qs.bias
        # fused [Wq; Wk; Wv] (3hd, d) and [bq; bk; bv]: adjacent in the arena (fft_param_order)
        q = self.__dict__.get("_qkv_holder")
        if q is None:
            q = self._qkv_holder = _WeightHolder(self.d, n3)
        self._qkv_b = _flat_view(bq, n3)
        self._qkv_gw = _flat_view(_g(wq), n3 * self.d).view(n3, self.d)
        self._qkv_gb = _flat_view(_g(bq), n3)
        _linear_prep(q, cdt, w=_flat_view(wq, n3 * self.d).view(n3, self.d), jobs=jobs)
        _linear_prep(a.fc, cdt, jobs=jobs)
        _conv_prep(f.w_1, cdt, jobs)
        _conv_prep(f.w_2, cdt, jobs)

    def cdesc(self):
        """The block's fs2_fft_block_* descriptor (include/fs2hip.h, FS2_FB_*): geometry, the
        compute-layout weights, biases, LayerNorm affines and gradient views, as a host int64
        table (cached: the compute-layout buffers and the gradient arena persist)."""
        key = (_GEN[0], self.site)
        d = self.__dict__.get("_cdesc")
        if d is not None and d[0] == key:
            return d[1]
        a, f = self.slf_attn, self.pos_ffn
        q = self._qkv_holder
        P = lambda t: t.data_ptr()
        w = [self.d, a.n_head, a.d_k, f.w_1.c_out, f.w_1.k, f.w_1.padding, self.site,
             P(q._w_fwd), P(q._w_bwd), P(self._qkv_b), P(a.fc._w_fwd), P(a.fc._w_bwd), P(a.fc.bias),
             P(f.w_1._w_fwd), P(f.w_1._w_bwd), P(f.w_1.bias), P(f.w_2._w_fwd), P(f.w_2._w_bwd),
             P(f.w_2.bias), P(a.layer_norm.weight), P(a.layer_norm.bias), P(f.layer_norm.weight),
             P(f.layer_norm.bias), P(self._qkv_gw), P(self._qkv_gb), P(_g(a.fc.weight)),
             P(_g(a.fc.bias)), P(_g(f.w_1.weight)), P(_g(f.w_1.bias)), P(_g(f.w_2.weight)),
             P(_g(f.w_2.bias)), P(_g(a.layer_norm.weight)), P(_g(a.layer_norm.bias)),
             P(_g(f.layer_norm.weight)), P(_g(f.layer_norm.bias))]
        if f.w_2.k != 1:
            raise RuntimeError("fs2_fft_block_*: w_2 must be a 1x1 conv (SubLayers.py:78-83)")
        arr = (ctypes.c_int64 * len(w))(*w)
        self._cdesc = (key, arr)
        return arr

    def fwd(self, x, x_t, lens, B, T, ctx):
        a, f = self.slf_attn, self.pos_ffn
        M, d = x.shape
        q = self._qkv_holder
        n3 = q.out_features
        p = ctx.p(a.p)
        x_c = _t(x, x_t)
        qkv = K.conv_gemm(x_c, q._w_fwd, M, T, d, n3, 1, 0, bias=self._qkv_b, out_dtype=ctx.cdt,
                          lens=lens)
        o, lse = K.attn_fwd(qkv, lens, B, T, a.n_head, a.d_k, 1.0 / math.sqrt(a.d_k))
        hd = a.n_head * a.d_k
        # bf16: the post-LNs run in the epilogues of fc and w_2 (fs2_conv_gemm_ln, bitwise
        # equal to the two-launch form below, without the fp32 y round trip).  Decoder-sized
        # grids only: at 6,144 rows (the encoder) its 96 64-row tiles under-fill the chip
        # (scripts/ln_fuse_bench.py: decoder fc 31.7 -> 26.8 us, w_2 42.3 -> 37.4 us; encoder
        # w_2 22.7 -> 29.5 us)
        fuse = FUSE_LN and ctx.copy is not None and d == 256 and M >= FUSE_LN_MIN_ROWS
        if fuse:
            x1, x1_t, xh1, rs1 = K.conv_gemm_ln(
                o, a.fc._w_fwd, M, T, hd, d, 1, 0, a.layer_norm.weight, a.layer_norm.bias,
                bias=a.fc.bias, res=x, lens=lens, p_in=p, seed=ctx.seed, site_in=self.site,
                copy=ctx.copy)
        else:
            y1 = K.conv_gemm(o, a.fc._w_fwd, M, T, hd, d, 1, 0, bias=a.fc.bias, lens=lens)
            x1, x1_t, xh1, rs1, _ = K.ln_fwd(y1, a.layer_norm.weight, a.layer_norm.bias, res=x,
                                             lens=lens, seq_len=T, p_in=p, seed=ctx.seed,
                                             site_in=self.site, copy=ctx.copy)
        w1, w2 = f.w_1, f.w_2
        x1_c = _t(x1, x1_t)
        h = K.conv_gemm(x1_c, w1._w_fwd, M, T, d, w1.c_out, w1.k, w1.padding, bias=w1.bias,
                        flags=K.EPI_RELU, out_dtype=ctx.cdt, lens=lens)
        if fuse:
            x2, x2_t, xh2, rs2 = K.conv_gemm_ln(
                h, w2._w_fwd, M, T, w2.c_in, d, w2.k, w2.padding, f.layer_norm.weight,
                f.layer_norm.bias, bias=w2.bias, res=x1, lens=lens, p_in=p, seed=ctx.seed,
                site_in=self.site + 1, copy=ctx.copy)
        else:
            y2 = K.conv_gemm(h, w2._w_fwd, M, T, w2.c_in, d, w2.k, w2.padding, bias=w2.bias,
                             lens=lens)
            x2, x2_t, xh2, rs2, _ = K.ln_fwd(y2, f.layer_norm.weight, f.layer_norm.bias, res=x1,
                                             lens=lens, seq_len=T, p_in=p, seed=ctx.seed,
                                             site_in=self.site + 1, copy=ctx.copy)
        saved = (x_c, qkv, o, lse, x1_c, h, xh1, rs1, xh2, rs2, p, ctx, lens, B, T)
        return x2, x2_t, saved

    def bwd(self, dx2, saved, ln2_done=None, prev=None):
        """Block backward from the gradient of its output.  ``ln2_done`` = (dy2 copy, dx1):
        this block's LN2 backward already ran in the epilogue of the following block's QKV data
        gradient.  ``prev`` = (previous block, its saved tensors): run the previous block's LN2
        backward in this block's QKV data-gradient epilogue (fs2_conv_gemm_ln_bwd) and return
        its (dy2 copy, dx1) instead of dx."""
        a, f = self.slf_attn, self.pos_ffn
        x_c, qkv, o, lse, x1_c, h, xh1, rs1, xh2, rs2, p, ctx, lens, B, T = saved
        M, d = x_c.shape
        q = self._qkv_holder
        n3 = q.out_features
        seed, cdt = ctx.seed, ctx.cdt
        w1, w2 = f.w_1, f.w_2
        ln2, ln1 = f.layer_norm, a.layer_norm
        if ln2_done is not None:
            dy2, dy2_t, dx1 = None, ln2_done[0], ln2_done[1]
        else:
            # LN2 (masked; dropout before the residual add): dx1 starts as dz2
            dx1 = torch.empty((M, d), dtype=torch.float32, device=x_c.device)
            dy2, dy2_t = K.ln_bwd(xh2, rs2, ln2.weight, ln2.bias, _g(ln2.weight), _g(ln2.bias),
                                  dout=dx2, lens=lens, seq_len=T, p_in=p, seed=seed,
                                  site_in=self.site + 1, dres=dx1, dres_add=False, copy=ctx.copy,
                                  dbias_in=_g(w2.bias))
        dy2_c = _t(dy2, dy2_t)
        ctx.wgrad(dy2_c, h, _g(w2.weight), M, T, w2.c_in, d, w2.k, w2.padding, lens=lens,
                  group=True)
        dh = K.conv_gemm(dy2_c, w2._w_bwd, M, T, d, w2.c_in, w2.k, w2.padding,
                         flags=K.EPI_RELU_MASK_AUX, aux=h, out_dtype=cdt, lens=lens)
        ctx.wgrad(dh, x1_c, _g(w1.weight), M, T, d, w1.c_out, w1.k, w1.padding,
                  db=_g(w1.bias), lens=lens)
        K.conv_gemm(dh, w1._w_bwd, M, T, w1.c_out, d, w1.k, w1.padding, flags=K.EPI_ADD_AUX,
                    aux=dx1, out=dx1, lens=lens)
        # LN1 -> fc -> attention -> QKV
        dx = torch.empty((M, d), dtype=torch.float32, device=x_c.device)
        dy1, dy1_t = K.ln_bwd(xh1, rs1, ln1.weight, ln1.bias, _g(ln1.weight), _g(ln1.bias),
                              dout=dx1, lens=lens, seq_len=T, p_in=p, seed=seed,
                              site_in=self.site, dres=dx, dres_add=False, copy=ctx.copy,
                              dbias_in=_g(a.fc.bias))
        dy1_c = _t(dy1, dy1_t)
        hd = a.n_head * a.d_k
        ctx.wgrad(dy1_c, o, _g(a.fc.weight), M, T, hd, d, 1, 0, lens=lens, group=True)
        do = K.conv_gemm(dy1_c, a.fc._w_bwd, M, T, d, hd, 1, 0, out_dtype=cdt, lens=lens)
        dqkv = K.attn_bwd(qkv, o, do, lse, lens, B, T, a.n_head, a.d_k, 1.0 / math.sqrt(a.d_k))
        ctx.wgrad(dqkv, x_c, self._qkv_gw, M, T, d, n3, 1, 0, db=self._qkv_gb, lens=lens,
                  group=True)
        ctx.flush()
        if prev is not None:
            pb, ps = prev
            pf = pb.pos_ffn
            pl2 = pf.layer_norm
            return K.conv_gemm_ln_bwd(
                dqkv, q._w_bwd, M, T, n3, d, 1, 0, ps[8], ps[9], pl2.weight, _g(pl2.weight),
                _g(pl2.bias), aux=dx, lens=lens, p_in=ps[10], seed=seed, site_in=pb.site + 1,
                dbias_in=_g(pf.w_2.bias), copy=ctx.copy)
        K.conv_gemm(dqkv, q._w_bwd, M, T, n3, d, 1, 0, flags=K.EPI_ADD_AUX, aux=dx, out=dx,
                    lens=lens)
        return dx


_SIZE_MEMO = {}


def _csize(name, desc, ngeo, *args):
    """Memoised size / offset query of a per-module C entry (``fs2_*_bytes`` / ``_offset``):
    they depend only on the descriptor's leading geometry words and the call's sizes, and a
    ctypes call costs microseconds of host time per block and step."""
    key = (name, tuple(desc[:ngeo]), args)
    v = _SIZE_MEMO.get(key)
    if v is None:
        v = _SIZE_MEMO[key] = getattr(K.lib, name)(desc, *args)
    return v


def _c_blocks(ctx, d):
    return C_BLOCKS and ctx.copy is not None and ctx.cdt == torch.bfloat16 and d == 256


def _stack_fwd_c(layers, x, x_t, lens, B, T, ctx, after_first=None):
    """Forward through a stack of FFT blocks, one fs2_fft_block_fwd call per block; each block's
    activations live in one region (saved for the backward); ``after_first`` is called once the
    first block is issued.  Returns the last block's output, its bf16 copy and the per-block
    saved tuples."""
    M, d = x.shape
    fuse = FUSE_LN and M >= FUSE_LN_MIN_ROWS
    saved = []
    xp, xtp, x_keep = x.data_ptr(), x_t.data_ptr(), x_t
    lp = 0 if lens is None else lens.data_ptr()
    stream = K.stream()
    acts = []
    for layer in layers:
        desc = layer.cdesc()
        p = ctx.p(layer.slf_attn.p)
        act = _region(_csize('fs2_fft_block_act_bytes', desc, 7, M, B, T, int(fuse)), x.device,
                      "fft_block act")
        K.lib.fs2_fft_block_fwd(desc, xp, xtp, act.data_ptr(), M, B, T, lp, p,
                                ctx.seed.data_ptr() if p > 0 else None, int(fuse), stream)
        if after_first is not None:
            after_first()
            after_first = None
        saved.append(("C", act, xtp, x_keep, fuse, p))
        o2 = _csize('fs2_fft_block_act_offset', desc, 7, M, B, T, int(fuse), 0)
        o2t = _csize('fs2_fft_block_act_offset', desc, 7, M, B, T, int(fuse), 1)
        xp, xtp, x_keep = act.data_ptr() + o2, act.data_ptr() + o2t, act
        acts.append((act, o2, o2t))
    act, o2, o2t = acts[-1]
    out = act[o2:o2 + M * d * 4].view(torch.float32).view(M, d)
    out_t = act[o2t:o2t + M * d * 2].view(torch.bfloat16).view(M, d)
    return out, out_t, saved


def _stack_bwd_c(layers, saved, dx, ctx, lens, B, T):
    """Backward through a stack of FFT blocks, one fs2_fft_block_bwd call per block (the
    previous block's LN2 backward in each QKV data-gradient epilogue on decoder-sized grids, as
    _stack_bwd)."""
    layers, saved = list(reversed(layers)), list(reversed(saved))
    M, d = dx.shape
    ctx.flush()
    lp = 0 if lens is None else lens.data_ptr()
    side = ctx.side.cuda_stream if ctx.side is not None else None
    stream = K.stream()
    carry = None
    dev = dx.device
    for i, (layer, s) in enumerate(zip(layers, saved)):
        _, act, xtp, x_keep, fuse, p = s
        desc = layer.cdesc()
        fuse_bwd = FUSE_LN_BWD and M >= FUSE_LN_MIN_ROWS and i + 1 < len(layers)
        tmp = _region(_csize('fs2_fft_block_tmp_bytes', desc, 7, M, B, T), dev, "fft_block tmp")
        ws = ctx._side_ws(_csize('fs2_fft_block_side_ws_bytes', desc, 7, M), dev) if side is not None else \
            K.ws(_csize('fs2_fft_block_side_ws_bytes', desc, 7, M), dev)
        dxo = torch.empty((M, d), dtype=torch.float32, device=dev)
        pdesc = pact = pdy2 = pdx1 = None
        pfuse, pp = 0, 0.0
        if fuse_bwd:
            ps = saved[i + 1]
            pdesc, pact, pfuse, pp = layers[i + 1].cdesc(), ps[1].data_ptr(), int(ps[4]), ps[5]
            pdy2 = torch.empty((M, d), dtype=torch.bfloat16, device=dev)
            pdx1 = torch.empty((M, d), dtype=torch.float32, device=dev)
        need_seed = p > 0 or (fuse_bwd and pp > 0)
        K.lib.fs2_fft_block_bwd(
            desc, act.data_ptr(), xtp, int(fuse), p,
            dx.data_ptr() if carry is None else None,
            carry[0].data_ptr() if carry is not None else None,
            carry[1].data_ptr() if carry is not None else None,
            pdesc, pact, pfuse, pp, tmp.data_ptr(), dxo.data_ptr(),
            None if pdy2 is None else pdy2.data_ptr(), None if pdx1 is None else pdx1.data_ptr(),
            M, B, T, lp, ctx.seed.data_ptr() if need_seed else None, ws.data_ptr(), ws.numel() * 4,
            stream, side)
        # read by the side stream's weight gradients after this call: kept until the join
        ctx.keep.append((tmp, act, x_keep, carry))
        ctx.notify(lambda: fft_param_order(layer))
        if fuse_bwd:
            carry, dx = (pdy2, pdx1), None
        else:
            carry, dx = None, dxo
    return dx


def _stack_bwd(layers, saved, dx, ctx):
    """Backward through a stack of FFT blocks.  bf16, decoder-sized grids: each block's QKV data
    gradient carries the previous block's LN2 backward in its epilogue (fs2_conv_gemm_ln_bwd),
    and that block then starts from the (dy2 copy, dx1) it left."""
    layers, saved = list(reversed(layers)), list(reversed(saved))
    carry = None
    for i, (layer, s) in enumerate(zip(layers, saved)):
        M, d = s[0].shape
        fuse = (FUSE_LN_BWD and ctx.copy is not None and d == 256 and M >= FUSE_LN_MIN_ROWS and
                i + 1 < len(layers))
        out = layer.bwd(dx, s, ln2_done=carry, prev=(layers[i + 1], saved[i + 1]) if fuse else None)
        ctx.notify(lambda: fft_param_order(layer))
        if fuse:
            carry, dx = out, None
        else:
            carry, dx = None, out
    return dx


def _ffn_stack(config, side):
    t = config["transformer"]
    d = t[f"{side}_hidden"]
    return [FFTBlock(d, t[f"{side}_head"], t["conv_filter_size"], t["conv_kernel_size"],
                     t[f"{side}_dropout"]) for _ in range(t[f"{side}_layer"])]


class Encoder(nn.Module):
    """``transformer/Models.py:33-112``."""

    def __init__(self, config):
        super().__init__()
        d = config["transformer"]["encoder_hidden"]
        self.d = d
        self.max_seq_len = config["max_seq_len"]
        self.src_word_emb = Embedding(429, d, padding_idx=0)
        self.src_accent_emb = Embedding(5, d, padding_idx=0)
        self.position_enc = nn.Parameter(sinusoid_table(config["max_seq_len"] + 1, d)[None],
                                         requires_grad=False)
        self.layer_stack = nn.ModuleList(_ffn_stack(config, "encoder"))


class Decoder(nn.Module):
    """``transformer/Models.py:115-183``."""

    def __init__(self, config):
        super().__init__()
        d = config["transformer"]["decoder_hidden"]
        self.d = d
        self.max_seq_len = config["max_seq_len"]
        self.position_enc = nn.Parameter(sinusoid_table(config["max_seq_len"] + 1, d)[None],
                                         requires_grad=False)
        self.layer_stack = nn.ModuleList(_ffn_stack(config, "decoder"))


# ----------------------------------------------------------------------------- adaptor


class VariancePredictor(nn.Module):
    """``model/modules.py:197-250``: 2 x (Conv1d k=3 -> ReLU -> LN -> Dropout) -> Linear."""

    def __init__(self, config):
        super().__init__()
        d = config["transformer"]["encoder_hidden"]
        fs = config["variance_predictor"]["filter_size"]
        k = config["variance_predictor"]["kernel_size"]
        self.p = config["variance_predictor"]["dropout"]
        self.conv_layer = nn.Module()
        self.conv_layer.conv1d_1 = _ConvWrap(d, fs, k, (k - 1) // 2)
        self.conv_layer.layer_norm_1 = LayerNorm(fs)
        self.conv_layer.conv1d_2 = _ConvWrap(fs, fs, k, 1)  # padding hard-coded (modules.py:230)
        self.conv_layer.layer_norm_2 = LayerNorm(fs)
        self.linear_layer = Linear(fs, 1)
        self.site = 0

    def prep(self, cdt, jobs=None):
        _conv_prep(self.conv_layer.conv1d_1.conv, cdt, jobs)
        _conv_prep(self.conv_layer.conv1d_2.conv, cdt, jobs)

    def cdesc(self):
        """fs2_variance_predictor_* descriptor (include/fs2hip.h, FS2_VP_*), cached as
        FFTBlock.cdesc."""
        key = (_GEN[0], self.site)
        d = self.__dict__.get("_cdesc")
        if d is not None and d[0] == key:
            return d[1]
        c = self.conv_layer
        c1, c2 = c.conv1d_1.conv, c.conv1d_2.conv
        ln1, ln2, lin = c.layer_norm_1, c.layer_norm_2, self.linear_layer
        P = lambda t: t.data_ptr()
        w = [c1.c_in, c1.c_out, c1.k, c1.padding, c2.padding, self.site,
             P(c1._w_fwd), P(c1._w_bwd), P(c1.bias), P(ln1.weight), P(ln1.bias),
             P(c2._w_fwd), P(c2._w_bwd), P(c2.bias), P(ln2.weight), P(ln2.bias), P(lin.weight),
             P(lin.bias), P(_g(c1.weight)), P(_g(c1.bias)), P(_g(ln1.weight)), P(_g(ln1.bias)),
             P(_g(c2.weight)), P(_g(c2.bias)), P(_g(ln2.weight)), P(_g(ln2.bias)),
             P(_g(lin.weight)), P(_g(lin.bias))]
        if c2.c_in != c1.c_out or c2.k != c1.k or lin.out_features != 1:
            raise RuntimeError("fs2_variance_predictor_*: unexpected geometry (modules.py:197-250)")
        arr = (ctypes.c_int64 * len(w))(*w)
        self._cdesc = (key, arr)
        return arr

    def fwd(self, x, x_t, lens, B, T, ctx, stream=None):
        """``stream`` (raw handle): the C-ABI path issues on it instead of the current stream
        (the caller orders it); the per-kernel path always runs on the current stream."""
        if _c_blocks(ctx, x.shape[1]) and x_t is not None:
            return self._fwd_c(x_t, lens, B, T, ctx, stream)
        c = self.conv_layer
        c1, c2 = c.conv1d_1.conv, c.conv1d_2.conv
        M = x.shape[0]
        p = ctx.p(self.p)
        x_c = _t(x, x_t)
        h1 = K.conv_gemm(x_c, c1._w_fwd, M, T, c1.c_in, c1.c_out, c1.k, c1.padding, bias=c1.bias,
                         flags=K.EPI_RELU)
        u1, u1_t, xh1, rs1, _ = K.ln_fwd(h1, c.layer_norm_1.weight, c.layer_norm_1.bias, p_out=p,
                                         seed=ctx.seed, site_out=self.site, copy=ctx.copy)
        u1_c = _t(u1, u1_t)
        h2 = K.conv_gemm(u1_c, c2._w_fwd, M, T, c2.c_in, c2.c_out, c2.k, c2.padding, bias=c2.bias,
                         flags=K.EPI_RELU)
        _, _, xh2, rs2, pred = K.ln_fwd(h2, c.layer_norm_2.weight, c.layer_norm_2.bias, lens=lens,
                                        seq_len=T, p_out=p, seed=ctx.seed, site_out=self.site + 1,
                                        dot_w=self.linear_layer.weight,
                                        dot_b=self.linear_layer.bias)
        saved = (x_c, h1, u1_c, h2, xh1, rs1, xh2, rs2, p, ctx, lens, T)
        return pred.view(B, T), saved

    def _fwd_c(self, x_t, lens, B, T, ctx, stream=None):
        """One fs2_variance_predictor_fwd call (bitwise the per-kernel path below); its
        activations are allocated on the current stream whatever stream computes them."""
        desc = self.cdesc()
        M = x_t.shape[0]
        p = ctx.p(self.p)
        act = _region(_csize('fs2_variance_predictor_act_bytes', desc, 6, M), x_t.device,
                      f"predictor {self.site} act")
        K.lib.fs2_variance_predictor_fwd(desc, x_t.data_ptr(), act.data_ptr(), M, T,
                                         0 if lens is None else lens.data_ptr(), p,
                                         ctx.seed.data_ptr() if p > 0 else None,
                                         K.stream() if stream is None else stream)
        o = _csize('fs2_variance_predictor_act_offset', desc, 6, M, 0)
        pred = act[o:o + M * 4].view(torch.float32)
        return pred.view(B, T), ("C", act, x_t, lens, T, p, ctx)

    def _bwd_c(self, dpred, saved, dx_acc):
        _, act, x_t, lens, T, p, ctx = saved
        desc = self.cdesc()
        if _GUARD["on"]:  # debug: the inputs this backward reads, in stream order
            c = self.conv_layer
            _GUARD.setdefault("snap", []).append(
                (self.site, [t.detach().clone() for t in (self.linear_layer.weight, self.linear_layer.bias,
                                                          c.layer_norm_2.weight, c.layer_norm_2.bias,
                                                          dpred, act, x_t)]))
        M = x_t.shape[0]
        dev = x_t.device
        dpred = dpred.contiguous()
        tmp = _region(_csize('fs2_variance_predictor_tmp_bytes', desc, 6, M), dev,
                      f"predictor {self.site} tmp")
        need = _csize('fs2_variance_predictor_side_ws_bytes', desc, 6, M)
        side = ctx.side.cuda_stream if ctx.side is not None else None
        ws = ctx._side_ws(need, dev) if side is not None else K.ws(need, dev)
        K.lib.fs2_variance_predictor_bwd(desc, act.data_ptr(), x_t.data_ptr(), dpred.data_ptr(),
                                         tmp.data_ptr(), dx_acc.data_ptr(), M, T,
                                         0 if lens is None else lens.data_ptr(), p,
                                         ctx.seed.data_ptr() if p > 0 else None, ws.data_ptr(),
                                         ws.numel() * 4, K.stream(), side)
        ctx.keep.append((tmp, act, x_t))  # read by the side stream until the join

    def bwd(self, dpred, saved, dx_acc):
        """Backward; the input gradient is *added* into ``dx_acc`` (fp32, in place)."""
        if isinstance(saved[0], str):
            return self._bwd_c(dpred, saved, dx_acc)
        x_c, h1, u1_c, h2, xh1, rs1, xh2, rs2, p, ctx, lens, T = saved
        c = self.conv_layer
        c1, c2 = c.conv1d_1.conv, c.conv1d_2.conv
        ln1, ln2, lin = c.layer_norm_1, c.layer_norm_2, self.linear_layer
        M = x_c.shape[0]
        seed = ctx.seed
        dh2, dh2_t = K.ln_bwd(xh2, rs2, ln2.weight, ln2.bias, _g(ln2.weight), _g(ln2.bias),
                              ddot=dpred.contiguous().view(-1), dot_w=lin.weight,
                              dw_dot=_g(lin.weight), db_dot=_g(lin.bias), lens=lens, seq_len=T,
                              p_out=p, seed=seed, site_out=self.site + 1, relu_y=h2,
                              copy=ctx.copy, dbias_in=_g(c2.bias))
        dh2_c = _t(dh2, dh2_t)
        ctx.wgrad(dh2_c, u1_c, _g(c2.weight), M, T, c2.c_in, c2.c_out, c2.k, c2.padding)
        du1 = K.conv_gemm(dh2_c, c2._w_bwd, M, T, c2.c_out, c2.c_in, c2.k, c2.padding)
        dh1, dh1_t = K.ln_bwd(xh1, rs1, ln1.weight, ln1.bias, _g(ln1.weight), _g(ln1.bias),
                              dout=du1, p_out=p, seed=seed, site_out=self.site, relu_y=h1,
                              copy=ctx.copy, dbias_in=_g(c1.bias))
        dh1_c = _t(dh1, dh1_t)
        ctx.wgrad(dh1_c, x_c, _g(c1.weight), M, T, c1.c_in, c1.c_out, c1.k, c1.padding)
        K.conv_gemm(dh1_c, c1._w_bwd, M, T, c1.c_out, c1.c_in, c1.k, c1.padding,
                    flags=K.EPI_ADD_AUX, aux=dx_acc, out=dx_acc)


class VarianceAdaptor(nn.Module):
    """``model/modules.py:17-158`` (phoneme-level pitch and energy, linear bins)."""

    def __init__(self, preprocess_config, model_config, config_path):
        super().__init__()
        d = model_config["transformer"]["encoder_hidden"]
        n_bins = model_config["variance_embedding"]["n_bins"]
        for key in ("pitch", "energy"):
            assert preprocess_config[key]["feature"] == "phoneme_level", \
                "frame-level variance features are not built (SURVEY.md §8a row 10)"
            assert model_config["variance_embedding"][f"{key}_quantization"] == "linear", \
                "log quantisation is not built"
        p_min, p_max, e_min, e_max = cfg.pitch_energy_range(config_path)
        self.duration_predictor = VariancePredictor(model_config)
        self.pitch_predictor = VariancePredictor(model_config)
        self.energy_predictor = VariancePredictor(model_config)
        self.pitch_bins = nn.Parameter(torch.linspace(p_min, p_max, n_bins - 1), requires_grad=False)
        self.energy_bins = nn.Parameter(torch.linspace(e_min, e_max, n_bins - 1), requires_grad=False)
        self.pitch_embedding = Embedding(n_bins, d)
        self.energy_embedding = Embedding(n_bins, d)


# ----------------------------------------------------------------------------- PostNet


class PostNet(nn.Module):
    """``transformer/Layers.py:67-137``: 5 x (Conv1d k=5 + BatchNorm1d), tanh on 0-3,
    dropout 0.5 on all (hard-coded, active in training)."""

    def __init__(self, n_mel=80, dim=512, k=5, n=5):
        super().__init__()
        chans = [n_mel] + [dim] * (n - 1) + [n_mel]
        self.convolutions = nn.ModuleList(
            nn.Sequential(_ConvWrap(chans[i], chans[i + 1], k, (k - 1) // 2),
                          BatchNorm1d(chans[i + 1])) for i in range(n))
        self.site = 0

    def prep(self, cdt, jobs=None):
        for layer in self.convolutions:
            _conv_prep(layer[0].conv, cdt, jobs)

    def mel_head_desc(self, lin):
        """fs2_mel_head_* descriptor (include/fs2hip.h, FS2_MH_* / FS2_MHL_*) of mel_linear
        ``lin`` followed by this PostNet, cached as FFTBlock.cdesc."""
        key = (_GEN[0], self.site, id(lin))
        d = self.__dict__.get("_cdesc")
        if d is not None and d[0] == key:
            return d[1]
        c0 = self.convolutions[0][0].conv
        P = lambda t: t.data_ptr()
        n = len(self.convolutions)
        if n > MH_MAX_LAYERS:
            raise RuntimeError(f"fs2_mel_head_*: at most {MH_MAX_LAYERS} PostNet layers")
        w = [lin.out_features, lin.in_features, c0.c_out, c0.k, c0.padding, n, self.site,
             P(lin._w_fwd), P(lin._w_bwd), P(lin.bias), P(_g(lin.weight)), P(_g(lin.bias))]
        for conv, bn in ((layer[0].conv, layer[1]) for layer in self.convolutions):
            if conv.k != c0.k or conv.padding != c0.padding:
                raise RuntimeError("fs2_mel_head_*: PostNet convs of one kernel size")
            w += [P(conv._w_fwd), P(conv._w_bwd), P(conv.bias), P(bn.weight), P(bn.bias),
                  P(bn.running_mean), P(bn.running_var), P(bn.num_batches_tracked),
                  P(_g(conv.weight)), P(_g(conv.bias)), P(_g(bn.weight)), P(_g(bn.bias))]
        w += [0] * (MH_WORDS - len(w))
        arr = (ctypes.c_int64 * len(w))(*w)
        self._cdesc = (key, arr)
        return arr

    def fwd(self, x, x_t, B, T, ctx):
        """x: (M, n_mel) mel_linear output; returns postnet(x) + x."""
        if not self.training:
            return self.fwd_eval(x, x_t, T, ctx.copy), None
        M = x.shape[0]
        a_c = _t(x, x_t)
        saved = []
        n = len(self.convolutions)
        p = ctx.p(0.5)
        out = None
        for i, layer in enumerate(self.convolutions):
            conv, bn = layer[0].conv, layer[1]
            z = K.conv_gemm(a_c, conv._w_fwd, M, T, conv.c_in, conv.c_out, conv.k, conv.padding,
                            bias=conv.bias)
            rm, rv = (bn.running_mean, bn.running_var) if self.training else (None, None)
            last = i == n - 1
            out, out_t, mean, rstd = K.bn_fwd(z, bn.weight, bn.bias, rm, rv, not last, p, ctx.seed,
                                              self.site + i, res=x if last else None,
                                              copy=None if last else ctx.copy, want_out=last,
                                              num_batches_tracked=bn.num_batches_tracked
                                              if self.training else None)
            saved.append((a_c, z, mean, rstd))
            a_c = _t(out, out_t)
        return out, (saved, p, ctx, T)

    def fwd_eval(self, x, x_t, T, copy):
        """Eval mode: BatchNorm on the running statistics, no dropout, no stat update."""
        M = x.shape[0]
        a_c = _t(x, x_t)
        n = len(self.convolutions)
        out = None
        for i, layer in enumerate(self.convolutions):
            conv, bn = layer[0].conv, layer[1]
            z = K.conv_gemm(a_c, conv._w_fwd, M, T, conv.c_in, conv.c_out, conv.k, conv.padding,
                            bias=conv.bias)
            last = i == n - 1
            out, out_t = K.bn_eval_fwd(z, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                       not last, res=x if last else None,
                                       copy=None if last else copy, want_out=last)
            a_c = _t(out, out_t)
        return out

    def bwd(self, dout, saved, dx_acc):
        """dout: grad of postnet(x) + x; adds the postnet input grad into ``dx_acc``."""
        layers, p, ctx, T = saved
        n = len(self.convolutions)
        d = dout
        for i in range(n - 1, -1, -1):
            conv, bn = self.convolutions[i][0].conv, self.convolutions[i][1]
            a_c, z, mean, rstd = layers[i]
            M = z.shape[0]
            dz, dz_t = K.bn_bwd(d, z, mean, rstd, bn.weight, bn.bias, _g(bn.weight), _g(bn.bias),
                                i < n - 1, p, ctx.seed, self.site + i, copy=ctx.copy)
            dz_c = _t(dz, dz_t)
            ctx.wgrad(dz_c, a_c, _g(conv.weight), M, T, conv.c_in, conv.c_out, conv.k,
                      conv.padding, db=_g(conv.bias))
            if i > 0:
                d = K.conv_gemm(dz_c, conv._w_bwd, M, T, conv.c_out, conv.c_in, conv.k, conv.padding)
            else:
                K.conv_gemm(dz_c, conv._w_bwd, M, T, conv.c_out, conv.c_in, conv.k, conv.padding,
                            flags=K.EPI_ADD_AUX, aux=dx_acc, out=dx_acc)


# ----------------------------------------------------------------------------- GMM head


class SpeakerMetaEncoder(nn.Module):
    """TacoSpawn head, ``model/fastspeech2.py:306-341``."""

    def __init__(self, preprocess_config, model_config):
        super().__init__()
        self.metadata_list = preprocess_config["speaker_generation"]["metadata"]
        self.input_dim = cfg.meta_dim(preprocess_config)
        self.K = model_config["speaker_generation"]["GMM_mixtures"]
        self.D = model_config["transformer"]["encoder_hidden"]
        self.pi_linear = nn.Sequential(Linear(self.input_dim, self.K), nn.Softmax(dim=1))
        self.sigma_linear = nn.Sequential(Linear(self.input_dim, self.K * self.D), nn.Softplus())
        self.mu_linear = Linear(self.input_dim, self.K * self.D)

    def forward(self, meta):
        from .loss import GMMPrior
        meta = meta.contiguous().float()
        pi, mu, sigma, sigma_pre = K.gmm_head_fwd(
            meta, self.pi_linear[0].weight, self.pi_linear[0].bias, self.sigma_linear[0].weight,
            self.sigma_linear[0].bias, self.mu_linear.weight, self.mu_linear.bias, self.K, self.D)
        return GMMPrior(pi, mu, sigma, sigma_pre=sigma_pre, meta=meta, head=self)

    def params(self):
        return [self.pi_linear[0].weight, self.pi_linear[0].bias, self.sigma_linear[0].weight,
                self.sigma_linear[0].bias, self.mu_linear.weight, self.mu_linear.bias]

    def grads(self):
        return [_g(p) for p in self.params()]


# ----------------------------------------------------------------------------- arena


class ParamArena:
    """One flat fp32 buffer for all trainable parameters and one for their gradients.

    ``order`` is the flat layout (reverse backward order); each parameter's ``.data`` and
    ``.grad`` become views, so the module API (state_dict, parameters(), .grad) is unchanged
    while kernels, the optimiser and the gradient all-reduce see contiguous buffers."""

    def __init__(self, params, device):
        self.params = list(params)
        offs, n = [], 0
        for p in self.params:
            offs.append(n)
            n += (p.numel() + 3) // 4 * 4  # 16-B aligned sections
        self.numel = n
        self.flat = torch.zeros(n, dtype=torch.float32, device=device)
        self.grad = torch.zeros(n, dtype=torch.float32, device=device)
        self.offsets = offs
        _GEN[0] += 1
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                v = self.flat[o:o + p.numel()]
                v.copy_(p.data.reshape(-1).to(device))
                p.data = v.view(p.shape)
                p._fs2_grad = self.grad[o:o + p.numel()].view(p.shape)
                p.grad = p._fs2_grad
        self.version = 0

    def zero_grad(self):
        K.fill_(self.grad, 0.0)
        for p in self.params:
            if p.grad is not p._fs2_grad:  # (setting .grad costs microseconds per parameter)
                p.grad = p._fs2_grad


def fft_param_order(b):
    """Flat layout of one FFT block: q/k/v weights (then biases) adjacent for the fused GEMM."""
    f, a = b.pos_ffn, b.slf_attn
    return [f.layer_norm.weight, f.layer_norm.bias, f.w_2.weight, f.w_2.bias, f.w_1.weight,
            f.w_1.bias, a.layer_norm.weight, a.layer_norm.bias, a.fc.weight, a.fc.bias,
            a.w_qs.weight, a.w_ks.weight, a.w_vs.weight, a.w_qs.bias, a.w_ks.bias, a.w_vs.bias]


def vp_param_order(v):
    c = v.conv_layer
    return [v.linear_layer.weight, v.linear_layer.bias, c.layer_norm_2.weight, c.layer_norm_2.bias,
            c.conv1d_2.conv.weight, c.conv1d_2.conv.bias, c.layer_norm_1.weight,
            c.layer_norm_1.bias, c.conv1d_1.conv.weight, c.conv1d_1.conv.bias]


def postnet_param_order(pn):
    out = []
    for layer in reversed(pn.convolutions):
        out += [layer[1].weight, layer[1].bias, layer[0].conv.weight, layer[0].conv.bias]
    return out


def _flat_order(m):
    """Reverse-backward layout of the whole model (see ParamArena)."""
    out = []

    def add(*ps):
        out.extend(ps)

    def fft(b):
        add(*fft_param_order(b))

    def vp(v):
        add(*vp_param_order(v))

    add(*postnet_param_order(m.postnet))
    add(m.mel_linear.weight, m.mel_linear.bias)
    for b in reversed(m.decoder.layer_stack):
        fft(b)
    va = m.variance_adaptor
    add(va.energy_embedding.weight)
    vp(va.energy_predictor)
    add(va.pitch_embedding.weight)
    vp(va.pitch_predictor)
    vp(va.duration_predictor)
    add(m.speaker_emb.weight)
    for b in reversed(m.encoder.layer_stack):
        fft(b)
    add(m.encoder.src_accent_emb.weight, m.encoder.src_word_emb.weight)
    e = m.speaker_enc
    add(e.pi_linear[0].weight, e.pi_linear[0].bias, e.sigma_linear[0].weight,
        e.sigma_linear[0].bias, e.mu_linear.weight, e.mu_linear.bias)
    train = [p for p in m.parameters() if p.requires_grad]
    assert len(out) == len(train) and {id(p) for p in out} == {id(p) for p in train}, \
        "flat layout must cover every trainable parameter exactly once"
    return out




# ----------------------------------------------------------------------------- autograd
# Block-granular autograd nodes.  Differentiable tensors crossing them are the fp32
# activations; the compute copies (bf16 path) travel as non-differentiable side outputs.


class EncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, token, enc, texts, accents, lens, B, T, ctx):
        x, x_t = K.encoder_embed(texts, accents, enc.src_word_emb.weight, enc.src_accent_emb.weight,
                                 enc.position_enc, B, T, enc.d, copy=ctx.copy)
        after_first, ctx.after_first = ctx.after_first, None
        if _c_blocks(ctx, enc.d) and x_t is not None:
            x, x_t, saved = _stack_fwd_c(enc.layer_stack, x, x_t, lens, B, T, ctx, after_first)
        else:
            saved = []
            for layer in enc.layer_stack:
                x, x_t, s = layer.fwd(x, x_t, lens, B, T, ctx)
                saved.append(s)
                if after_first is not None:
                    after_first()
                    after_first = None
        if not enc.layer_stack and after_first is not None:
            after_first()
        fctx.enc, fctx.saved, fctx.ids, fctx.ctx = enc, saved, (texts, accents), ctx
        fctx.geom = (lens, B, T)
        return x

    @staticmethod
    def backward(fctx, dx):
        enc = fctx.enc
        dx = dx.contiguous()
        if fctx.saved and isinstance(fctx.saved[0][0], str):
            dx = _stack_bwd_c(enc.layer_stack, fctx.saved, dx, fctx.ctx, *fctx.geom)
        else:
            dx = _stack_bwd(enc.layer_stack, fctx.saved, dx, fctx.ctx)
        texts, accents = fctx.ids
        K.embedding_bwd(dx, texts, _g(enc.src_word_emb.weight), 0)
        K.embedding_bwd(dx, accents, _g(enc.src_accent_emb.weight), 0)
        fctx.ctx.join()  # last block of the backward: every weight gradient is final after this
        fctx.ctx.notify(lambda: [enc.src_accent_emb.weight, enc.src_word_emb.weight])
        fctx.saved = None
        return (None,) * 8


class VarianceAdaptorFn(torch.autograd.Function):
    """Speaker add + variance adaptor (training branch) + decoder position encoding."""

    @staticmethod
    def forward(fctx, token, enc_out, m, speakers, src_lens, p_t, e_t, d_t, B, Ts, T_dec, ctx):
        fctx.set_materialize_grads(False)  # unused outputs' gradients stay None (no zero fills)
        va = m.variance_adaptor
        x0, x0_t = K.rowvec_add(enc_out, speakers, m.speaker_emb.weight, B, Ts, copy=ctx.copy)
        # the three predictors are independent under teacher forcing (the energy predictor's
        # input adds the pitch *target*'s embedding, the LengthRegulator uses the duration
        # *targets*): the pitch and duration predictors run on the side stream -- idle in the
        # forward once the weights are prepared -- beside the energy predictor, the embeddings
        # and the LengthRegulator, joined after them (C-ABI path; same results)
        side = ctx.side.cuda_stream if ctx.side is not None and VA_SIDE else None
        if side is not None:
            K.lib.fs2_stream_wait(side, K.stream())
        p, s_p = va.pitch_predictor.fwd(x0, x0_t, src_lens, B, Ts, ctx, stream=side)
        log_d, s_d = va.duration_predictor.fwd(x0, x0_t, src_lens, B, Ts, ctx, stream=side)
        x1, x1_t, idx_p = K.bucket_embed(x0, p_t.contiguous().view(-1), va.pitch_bins,
                                         va.pitch_embedding.weight, copy=ctx.copy)
        e, s_e = va.energy_predictor.fwd(x1, x1_t, src_lens, B, Ts, ctx)
        x2, _, idx_e = K.bucket_embed(x1, e_t.contiguous().view(-1), va.energy_bins,
                                      va.energy_embedding.weight)
        cum, mel_len = K.lr_index(d_t.contiguous())
        x_lr, x_lr_t = K.lr_expand(x2, cum, T_dec, posenc=m.decoder.position_enc, copy=ctx.copy)
        if side is not None:
            K.lib.fs2_stream_wait(K.stream(), side)
        fctx.m, fctx.saved = m, (s_d, s_p, s_e, idx_p, idx_e, cum, speakers, B, Ts, T_dec, ctx)
        side = x_lr_t if x_lr_t is not None else torch.empty(0, device=x_lr.device)
        fctx.mark_non_differentiable(mel_len, side)
        return x_lr, log_d, p, e, mel_len, side

    @staticmethod
    def backward(fctx, d_xlr, d_logd, d_p, d_e, _a, _b):
        m = fctx.m
        va = m.variance_adaptor
        s_d, s_p, s_e, idx_p, idx_e, cum, speakers, B, Ts, T_dec, ctx = fctx.saved
        d = m.encoder.d
        if d_xlr is None:
            dx = K.zeros((B * Ts, d), m._token.device)
        else:
            dx = K.lr_expand_bwd(d_xlr.contiguous(), cum, T_dec, d)
        K.bucket_embed_bwd(dx, idx_e, _g(va.energy_embedding.weight))
        if d_e is not None:
            va.energy_predictor.bwd(d_e, s_e, dx)
        ctx.notify(lambda: [va.energy_embedding.weight] + vp_param_order(va.energy_predictor))
        K.bucket_embed_bwd(dx, idx_p, _g(va.pitch_embedding.weight))
        if d_p is not None:
            va.pitch_predictor.bwd(d_p, s_p, dx)
        ctx.notify(lambda: [va.pitch_embedding.weight] + vp_param_order(va.pitch_predictor))
        if d_logd is not None:
            va.duration_predictor.bwd(d_logd, s_d, dx)
        ctx.notify(lambda: vp_param_order(va.duration_predictor))
        K.rowvec_add_bwd(dx, speakers, _g(m.speaker_emb.weight), B, Ts)
        ctx.notify(lambda: [m.speaker_emb.weight])
        fctx.saved = None
        return (None, dx) + (None,) * 10


class DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, token, x, x_t, dec, lens, B, T, ctx):
        fctx.set_materialize_grads(False)  # the compute-copy side output gets no zero gradient
        x_t = x_t if x_t.numel() else None
        if _c_blocks(ctx, x.shape[1]) and x_t is not None:
            x, x_t, saved = _stack_fwd_c(dec.layer_stack, x, x_t, lens, B, T, ctx)
        else:
            saved = []
            for layer in dec.layer_stack:
                x, x_t, s = layer.fwd(x, x_t, lens, B, T, ctx)
                saved.append(s)
        fctx.dec, fctx.saved, fctx.ctx = dec, saved, ctx
        fctx.geom, fctx.xshape, fctx.xdev = (lens, B, T), tuple(x.shape), x.device
        side = x_t if x_t is not None else torch.empty(0, device=x.device)
        fctx.mark_non_differentiable(side)
        return x, side

    @staticmethod
    def backward(fctx, dx, _):
        if dx is None:
            dx = K.zeros(fctx.xshape, fctx.xdev)
        dx = dx.contiguous()
        if fctx.saved and isinstance(fctx.saved[0][0], str):
            dx = _stack_bwd_c(fctx.dec.layer_stack, fctx.saved, dx, fctx.ctx, *fctx.geom)
        else:
            dx = _stack_bwd(fctx.dec.layer_stack, fctx.saved, dx, fctx.ctx)
        fctx.saved = None
        return None, dx, None, None, None, None, None, None


class MelHeadFn(torch.autograd.Function):
    """mel_linear + (postnet(out) + out)."""

    @staticmethod
    def forward(fctx, token, x, x_t, m, B, T, ctx):
        lin = m.mel_linear
        M = x.shape[0]
        x_c = x_t if x_t.numel() else x
        if _c_blocks(ctx, x.shape[1]) and x_t.numel() and m.postnet.training:
            # one fs2_mel_head_fwd call: mel_linear + PostNet (bitwise the path below)
            desc = m.postnet.mel_head_desc(lin)
            p = ctx.p(0.5)
            act = _region(_csize('fs2_mel_head_act_bytes', desc, 7, M), x.device, "mel_head act")
            K.lib.fs2_mel_head_fwd(desc, x_c.data_ptr(), act.data_ptr(), M, T, p,
                                   ctx.seed.data_ptr() if p > 0 else None, K.stream())
            n_mel = lin.out_features
            o = _csize('fs2_mel_head_act_offset', desc, 7, M, 0)
            po = _csize('fs2_mel_head_act_offset', desc, 7, M, 1)
            out = act[o:o + M * n_mel * 4].view(torch.float32)
            post = act[po:po + M * n_mel * 4].view(torch.float32)
            fctx.m, fctx.saved = m, ("C", act, x_c, p, B, T, ctx)
            return out.view(B, T, -1), post.view(B, T, -1)
        out = K.conv_gemm(x_c, lin._w_fwd, M, T, lin.in_features, lin.out_features, 1, 0,
                          bias=lin.bias)
        out_t = K.cast_bf16(out) if ctx.copy is not None else None
        post, s = m.postnet.fwd(out, out_t, B, T, ctx)
        fctx.m, fctx.saved = m, (x_c, s, B, T, ctx)
        return out.view(B, T, -1), post.view(B, T, -1)

    @staticmethod
    def backward(fctx, d_out, d_post):
        m = fctx.m
        if isinstance(fctx.saved[0], str):
            return MelHeadFn._backward_c(fctx, d_out, d_post)
        x_c, s, B, T, ctx = fctx.saved
        lin = m.mel_linear
        M = x_c.shape[0]
        n_mel = lin.out_features
        d_out = d_out.contiguous().view(M, n_mel) if d_out is not None else None
        if d_post is not None:
            d_post = d_post.contiguous().view(M, n_mel)
            dm = K.add(d_out, d_post) if d_out is not None else d_post.clone()
            m.postnet.bwd(d_post, s, dm)
        else:
            dm = d_out
        ctx.notify(lambda: postnet_param_order(m.postnet))
        dm_c = K.cast_bf16(dm) if ctx.copy is not None else dm
        ctx.wgrad(dm_c, x_c, _g(lin.weight), M, T, lin.in_features, n_mel, 1, 0, db=_g(lin.bias))
        dx = K.conv_gemm(dm_c, lin._w_bwd, M, T, n_mel, lin.in_features, 1, 0)
        ctx.notify(lambda: [lin.weight, lin.bias])
        fctx.saved = None
        return None, dx, None, None, None, None, None

    @staticmethod
    def _backward_c(fctx, d_out, d_post):
        m = fctx.m
        _, act, x_c, p, B, T, ctx = fctx.saved
        lin = m.mel_linear
        M = x_c.shape[0]
        n_mel = lin.out_features
        dev = x_c.device
        d_out = d_out.contiguous().view(M, n_mel) if d_out is not None else None
        d_post = d_post.contiguous().view(M, n_mel) if d_post is not None else None
        if d_out is None and d_post is None:
            d_out = K.zeros((M, n_mel), dev)
        desc = m.postnet.mel_head_desc(lin)
        tmp = _region(_csize('fs2_mel_head_tmp_bytes', desc, 7, M), dev, "mel_head tmp")
        need = _csize('fs2_mel_head_side_ws_bytes', desc, 7, M)
        side = ctx.side.cuda_stream if ctx.side is not None else None
        ws = ctx._side_ws(need, dev) if side is not None else K.ws(need, dev)
        dx = torch.empty((M, lin.in_features), dtype=torch.float32, device=dev)
        P = lambda t: None if t is None else t.data_ptr()
        K.lib.fs2_mel_head_bwd(desc, act.data_ptr(), x_c.data_ptr(), P(d_out), P(d_post),
                               tmp.data_ptr(), dx.data_ptr(), M, T, p,
                               ctx.seed.data_ptr() if p > 0 else None,
                               ws.data_ptr(), ws.numel() * 4, K.stream(), side)
        ctx.keep.append((tmp, act, x_c))  # read by the side stream until the join
        ctx.notify(lambda: postnet_param_order(m.postnet))
        ctx.notify(lambda: [lin.weight, lin.bias])
        fctx.saved = None
        return None, dx, None, None, None, None, None


# ----------------------------------------------------------------------------- top level


class FastSpeech2(nn.Module):
    """``model/fastspeech2.py:15-303`` on the HIP kernels (multi_speaker, no JDIT).

    ``compute_dtype``: ``torch.float32`` (exact f32 MFMA; the parity path) or
    ``torch.bfloat16`` (bf16 MFMA operands with fp32 accumulation, fp32 master weights,
    fp32 residual stream, norms, softmax statistics, losses and optimiser)."""

    def __init__(self, preprocess_config, model_config, config_path, device="cuda",
                 compute_dtype=torch.float32):
        super().__init__()
        self.model_config = model_config
        assert not model_config["jdit"]["use_jdit"], "JDIT aligner is out of scope (SURVEY.md §2.1)"
        assert model_config["multi_speaker"], "single-speaker FastSpeech2 is not built"
        self.encoder = Encoder(model_config)
        self.variance_adaptor = VarianceAdaptor(preprocess_config, model_config, config_path)
        self.decoder = Decoder(model_config)
        self.mel_linear = Linear(model_config["transformer"]["decoder_hidden"],
                                 preprocess_config["mel"]["n_mel_channels"])
        self.postnet = PostNet()
        self.speaker_emb = Embedding(cfg.n_speakers(config_path),
                                     model_config["transformer"]["encoder_hidden"])
        self.speaker_enc = SpeakerMetaEncoder(preprocess_config, model_config)
        # dropout site ids (2 per FFT block / variance predictor, 5 for the PostNet)
        site = 16
        for b in list(self.encoder.layer_stack) + list(self.decoder.layer_stack):
            b.site, site = site, site + 2
        va = self.variance_adaptor
        for v in (va.duration_predictor, va.pitch_predictor, va.energy_predictor):
            v.site, site = site, site + 2
        self.postnet.site = site
        self.dropout = True
        self.compute_dtype = compute_dtype
        self._seed_base = 0
        self._seed_state = None  # device int64[3] {base, counter, current}, fs2_seed_next
        self._arena = None
        self._prep = None
        self._hooks = {"grad": None}  # gradient-ready callback, see StepCtx.notify
        self.overlap_wgrad = True  # weight-gradient GEMMs on a side stream (StepCtx.wgrad)
        self._side = None
        self._ws_cache = {}
        self.to(device)

    # -- plumbing ---------------------------------------------------------------------
    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        _GEN[0] += 1
        self._arena = None  # parameters were re-materialised: rebuild the flat views lazily
        self._prep = None
        return r

    def arena(self):
        if self._arena is None:
            dev = self.encoder.position_enc.device
            if dev.type != "cuda":
                raise RuntimeError("FastSpeech2 (fs2-mi355x) runs on the GPU only; move it with .cuda()")
            self._arena = ParamArena(_flat_order(self), dev)
            self._token = torch.zeros((), device=dev, requires_grad=True)
            self.speaker_enc._tok = self._token
            self.speaker_enc._model_hooks = self._hooks
        return self._arena

    def side_stream(self):
        """The weight-gradient stream (None when overlap is off)."""
        if not self.overlap_wgrad:
            return None
        if self._side is None:
            dev = self.encoder.position_enc.device
            self._side = _RESERVED_SIDE.get(dev.index) or torch.cuda.Stream(device=dev)
        return self._side

    def join_side(self):
        """Make the current stream wait for all weight-gradient work issued so far."""
        if self._side is not None:
            K.lib.fs2_stream_wait(K.stream(), self._side.cuda_stream)

    def seed(self, s):
        """Seed the per-step dropout stream: step i's Philox key is splitmix64(s, i), drawn on
        the device (fs2_seed_next) so a captured step graph draws a fresh key per replay."""
        self._seed_base = int(s) & (2 ** 63 - 1)
        self._seed_state = None

    def _step_seed(self):
        if self._seed_state is None:
            self._seed_state = torch.tensor([self._seed_base, 0, 0], dtype=torch.int64,
                                            device=self.encoder.position_enc.device)
        K.seed_next(self._seed_state)
        return self._seed_state[2:3].clone()  # this forward's key (backward re-reads it)

    def prep_weights(self, side=None):
        """Re-lay out (and cast) every weight for the GEMMs, batched launches; the job tables
        (pointers into the arena and the compute-weight buffers) are built once.  Without a side
        stream everything is prepared on the current stream.  With one, only the first encoder
        block's weights are prepared on the current stream; the other encoder blocks' follow on
        ``side`` under the first block's forward, and everything after them (variance predictors,
        decoder, PostNet, mel head) under the rest of the encoder.  Returns None, or (with
        ``side``) the callable the encoder calls once its first block is issued: the current
        stream waits for the other encoder blocks' weights there, and the rest is issued on
        ``side`` after that wait point; the caller joins ``side`` before the first of those
        layers."""
        cdt = self.compute_dtype
        if self._prep is None or self._prep[0] != cdt:
            first, enc_jobs, rest = [], [], []
            for i, b in enumerate(self.encoder.layer_stack):
                b.prep(cdt, first if i == 0 else enc_jobs)
            va = self.variance_adaptor
            for v in (va.duration_predictor, va.pitch_predictor, va.energy_predictor):
                v.prep(cdt, rest)
            for b in self.decoder.layer_stack:
                b.prep(cdt, rest)
            self.postnet.prep(cdt, rest)
            _linear_prep(self.mel_linear, cdt, jobs=rest)
            ct = K.lib.fs2_weight_prep_tile_channels(K.code(cdt))

            def table(jobs):
                rows, first = [], 0
                for (w, co, ci, k, wf, wb) in jobs:
                    assert k <= 9
                    n = -(-co // 64) * -(-ci // ct)
                    rows.append([w, co, ci, k, wf, wb, first, first + n])
                    first += n
                t = torch.tensor(rows, dtype=torch.int64).to(self._arena.flat.device)
                return t, len(rows), first
            self._prep = (cdt, table(first), table(enc_jobs) if enc_jobs else None, table(rest),
                          table(enc_jobs + rest))
        cdt, t_first, t_enc, t_rest, t_all = self._prep
        code = K.code(cdt)

        def run(t, stream):
            K.lib.fs2_weight_prep_batch(code, K.ptr(t[0]), t[1], t[2], stream)
        if side is None:
            run(t_first, K.stream())
            run(t_all, K.stream())
            return None
        run(t_first, K.stream())
        K.lib.fs2_stream_wait(side.cuda_stream, K.stream())
        if t_enc is not None:
            run(t_enc, side.cuda_stream)

        def after_first_block():
            if t_enc is not None:
                K.lib.fs2_stream_wait(K.stream(), side.cuda_stream)
            run(t_rest, side.cuda_stream)
        return after_first_block

    # -- forward ----------------------------------------------------------------------
    def forward(self, speakers, texts, src_lens, max_src_len, mels=None, mel_lens=None,
                max_mel_len=None, p_targets=None, e_targets=None, d_targets=None,
                p_control=1.0, e_control=1.0, d_control=1.0, accents=None, speaker_meta=None):
        if accents is None:
            raise ValueError("accents are required (transformer/Models.py:101)")
        teacher = not (p_targets is None or e_targets is None or d_targets is None or
                       mel_lens is None)
        if not (self.training and teacher):
            if self.training and torch.is_grad_enabled():
                raise ValueError("training needs p/e/d targets and mel_lens (train.py:145); "
                                 "run inference under torch.no_grad() or model.eval()")
            return self._forward_infer(speakers, texts, src_lens, max_src_len, mel_lens,
                                       max_mel_len, p_targets, e_targets, d_targets, p_control,
                                       e_control, d_control, accents, speaker_meta=speaker_meta)
        self.arena()
        side = self.side_stream() if self.training else None
        after_first = self.prep_weights(side)
        seed = self._step_seed() if (self.training and self.dropout) else 0
        ctx = StepCtx(seed, self.training, self.dropout, self.compute_dtype)
        ctx.hook = self._hooks["grad"]
        ctx.side = side
        ctx.ws_cache = self._ws_cache
        B, Ts = texts.shape
        max_src_len = int(max_src_len)
        max_mel_len = int(max_mel_len)
        assert Ts == max_src_len, "texts must be padded to max_src_len"
        src_lens = src_lens.contiguous().long()
        mel_lens = mel_lens.contiguous().long()
        src_masks = K.length_mask(src_lens, max_src_len)
        T_dec = min(max_mel_len, self.decoder.max_seq_len)  # Models.py:166-174
        mel_masks = K.length_mask(mel_lens, T_dec)

        tok = self._token
        ctx.after_first = after_first  # the encoder calls it after issuing its first block
        enc = EncoderFn.apply(tok, self.encoder, texts.contiguous(), accents.contiguous(), src_lens,
                              B, Ts, ctx)
        speaker_emb_s = K.embedding_fwd(speakers.contiguous(), self.speaker_emb.weight)
        gmm = self.speaker_enc(speaker_meta)
        if side is not None:  # the weights prepared on the side stream (prep_weights)
            K.lib.fs2_stream_wait(K.stream(), side.cuda_stream)
        x_lr, log_d, p, e, mel_len, x_lr_t = VarianceAdaptorFn.apply(
            tok, enc, self, speakers.contiguous(), src_lens, p_targets, e_targets, d_targets, B, Ts,
            T_dec, ctx)
        x, x_t = DecoderFn.apply(tok, x_lr, x_lr_t, self.decoder, mel_lens, B, T_dec, ctx)
        output, postnet_output = MelHeadFn.apply(tok, x, x_t, self, B, T_dec, ctx)
        return (output, postnet_output, p, e, log_d, d_targets, src_masks, mel_masks, src_lens,
                mel_len, gmm, speaker_emb_s)

    # -- inference ----------------------------------------------------------------------
    def _posenc(self, T):
        """Decoder position table for T frames: ``position_enc`` (1001 rows) or, past
        ``max_seq_len`` in eval mode, a fresh table of T rows (Models.py:160-165)."""
        tab = self.decoder.position_enc
        if T <= tab.shape[1]:
            return tab
        cache = self.__dict__.setdefault("_long_posenc", {})
        n = 1 << (T - 1).bit_length()  # power-of-two buckets (rows depend on position only)
        if n not in cache:
            cache.clear()
            cache[n] = sinusoid_table(n, self.decoder.d).to(tab.device)[None]
        return cache[n]

    def _forward_infer(self, speakers, texts, src_lens, max_src_len, mel_lens, max_mel_len,
                       p_targets, e_targets, d_targets, p_control, e_control, d_control, accents,
                       speaker_meta=None, speaker_vec=None):
        """Forward without autograd: ``model/fastspeech2.py:52-174`` under ``torch.no_grad()``
        (evaluate.py, synthesize.py), any of the p/e/d targets optional.

        * pitch / energy without a target: prediction * control, bucketized
          (``modules.py:80-100``); energy uses ``p_control`` (``modules.py:124``, quirk kept,
          so ``e_control`` is accepted and unused as in the reference);
        * durations without a target: ``fs2_duration_round`` then the LengthRegulator; the
          frame count max(mel_len) is the one device->host read (``utils/tools.py:157``);
        * eval-mode decoder past ``max_seq_len``: no truncation, fresh position table
          (``Models.py:160-165``); training mode truncates to ``max_seq_len``;
        * eval-mode PostNet: BatchNorm on the running statistics.
        """
        del e_control  # modules.py:124 passes p_control to the energy branch
        self.arena()
        self.prep_weights()
        ctx = StepCtx(0, False, False, self.compute_dtype)  # no dropout outside training
        ctx.ws_cache = self._ws_cache
        B, Ts = texts.shape
        max_src_len = int(max_src_len)
        assert Ts == max_src_len, "texts must be padded to max_src_len"
        src_lens = src_lens.contiguous().long()
        src_masks = K.length_mask(src_lens, Ts)
        va, enc, dec = self.variance_adaptor, self.encoder, self.decoder
        with torch.no_grad():
            x, x_t = K.encoder_embed(texts.contiguous(), accents.contiguous(),
                                     enc.src_word_emb.weight, enc.src_accent_emb.weight,
                                     enc.position_enc, B, Ts, enc.d, copy=ctx.copy)
            for layer in enc.layer_stack:
                x, x_t, _ = layer.fwd(x, x_t, src_lens, B, Ts, ctx)
            if speaker_vec is None:
                ids, table = speakers.contiguous(), self.speaker_emb.weight
                speaker_emb_s = K.embedding_fwd(ids, table)
            else:  # synthesize_from_speaker_emb: one (1 or B, d) vector per utterance
                table = speaker_vec.detach().float().contiguous().view(-1, enc.d)
                ids = torch.arange(B, device=table.device) if table.shape[0] == B else \
                    torch.zeros(B, dtype=torch.int64, device=table.device)
                speaker_emb_s = None
            gmm = self.speaker_enc(speaker_meta) if speaker_meta is not None else None
            x0, x0_t = K.rowvec_add(x, ids, table, B, Ts, copy=ctx.copy)
            log_d, _ = va.duration_predictor.fwd(x0, x0_t, src_lens, B, Ts, ctx)
            p, _ = va.pitch_predictor.fwd(x0, x0_t, src_lens, B, Ts, ctx)
            if p_targets is None:
                if p_control != 1.0:
                    K.scale_(p, p_control)
                p_vals = p
            else:
                p_vals = p_targets
            x1, x1_t, _ = K.bucket_embed(x0, p_vals.contiguous().view(-1), va.pitch_bins,
                                         va.pitch_embedding.weight, copy=ctx.copy)
            e, _ = va.energy_predictor.fwd(x1, x1_t, src_lens, B, Ts, ctx)
            if e_targets is None:
                if p_control != 1.0:
                    K.scale_(e, p_control)
                e_vals = e
            else:
                e_vals = e_targets
            x2, _, _ = K.bucket_embed(x1, e_vals.contiguous().view(-1), va.energy_bins,
                                      va.energy_embedding.weight)
            if d_targets is not None:
                if mel_lens is None:
                    raise ValueError("d_targets without mel_lens: the decoder has no mask "
                                     "(model/fastspeech2.py:71-75)")
                d_rounded = d_targets
                cum, mel_len = K.lr_index(d_targets.contiguous())
                dec_lens = mel_lens.contiguous().long()
                T = int(max_mel_len) if max_mel_len is not None else int(mel_len.max())
            else:
                d_rounded = K.duration_round(log_d, d_control)
                cum, mel_len = K.lr_index(d_rounded)
                dec_lens = mel_len
                T_mask = int(mel_len.max())  # get_mask_from_lengths(mel_len), modules.py:137
                T = T_mask if max_mel_len is None else int(max_mel_len)
                if T > T_mask:
                    raise ValueError(f"max_mel_len {T} exceeds the predicted length {T_mask}: "
                                     "the reference's decoder mask would not broadcast")
            T_dec = T if (not self.training and T > dec.max_seq_len) else min(T, dec.max_seq_len)
            mel_masks = K.length_mask(dec_lens, T_dec)
            x, x_t = K.lr_expand(x2, cum, T_dec, posenc=self._posenc(T_dec), copy=ctx.copy)
            for layer in dec.layer_stack:
                x, x_t, _ = layer.fwd(x, x_t, dec_lens, B, T_dec, ctx)
            lin = self.mel_linear
            M = B * T_dec
            out = K.conv_gemm(_t(x, x_t), lin._w_fwd, M, T_dec, lin.in_features,
                              lin.out_features, 1, 0, bias=lin.bias)
            out_t = K.cast_bf16(out) if ctx.copy is not None else None
            post, _ = self.postnet.fwd(out, out_t, B, T_dec, ctx)
        out, post = out.view(B, T_dec, -1), post.view(B, T_dec, -1)
        head = (out, post, p, e, log_d, d_rounded, src_masks, mel_masks, src_lens, mel_len)
        if speaker_vec is not None:
            return head
        return head + (gmm, speaker_emb_s)

    def synthesize_from_speaker_emb(self, speakers, texts, src_lens, max_src_len, mels=None,
                                    mel_lens=None, max_mel_len=None, p_targets=None,
                                    e_targets=None, d_targets=None, p_control=1.0, e_control=1.0,
                                    d_control=1.0, accents=None, speaker_emb=None):
        """``model/fastspeech2.py:186-303``: the forward with a given speaker embedding (e.g.
        drawn by ``speaker_gen`` / a mid-attribute GMM) in place of the speaker table;
        ``speakers`` is unused, as in the reference.  Returns the 10-tuple."""
        if speaker_emb is None:
            raise ValueError("speaker_emb is required")
        if accents is None:
            raise ValueError("accents are required (transformer/Models.py:101)")
        if not torch.is_tensor(speaker_emb):
            speaker_emb = torch.as_tensor(np.asarray(speaker_emb), dtype=torch.float32)
        dev = self.encoder.position_enc.device
        return self._forward_infer(None, texts, src_lens, max_src_len, mel_lens, max_mel_len,
                                   p_targets, e_targets, d_targets, p_control, e_control,
                                   d_control, accents, speaker_vec=speaker_emb.to(dev))

    def speaker_gen(self, speaker_meta, seed=None):
        """``model/fastspeech2.py:176-180``: one embedding drawn from the attribute prior."""
        with torch.no_grad():
            gmm = self.speaker_enc(speaker_meta)
            return gmm.sample(seed=seed)

    def speaker_distribution(self, speaker_meta):
        with torch.no_grad():
            return self.speaker_enc(speaker_meta)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = super().load_state_dict(state_dict, strict=strict, assign=False)
        if self._arena is not None:
            self._arena.version += 1
        return r


def build(config_name="JVS-VCTK", device="cuda", compute_dtype=torch.float32):
    """Model + configs from a bundled config (``configs/<name>``)."""
    pp, mc, tc, path = cfg.load_configs(config_name)
    return FastSpeech2(pp, mc, path, device=device, compute_dtype=compute_dtype), (pp, mc, tc)
