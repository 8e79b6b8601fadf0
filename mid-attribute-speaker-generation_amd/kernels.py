"""Tensor-level wrappers over the C-ABI (``include/fs2hip.h``).

Each wrapper checks device/dtype/contiguity on the host, allocates outputs and workspaces
from PyTorch's caching allocator, and launches on the current HIP stream.  The storage type
of a GEMM/attention operand is taken from the tensor (float32 -> exact f32 MFMA path,
bfloat16 -> bf16 MFMA path, fp32 accumulation either way).  Norm/embedding kernels always
compute in fp32 and can emit a bf16 *compute copy* of their output (``copy=torch.bfloat16``)
for the next GEMM.  There is no PyTorch-math fallback: a wrong input raises, a missing
library raises.
"""
import ctypes

import torch

from ._lib import lib

F32 = 0
BF16 = 1
F64 = 2
EPI_BIAS, EPI_RELU, EPI_ADD_AUX, EPI_RELU_MASK_AUX, EPI_OUT_BF16, EPI_AUX_BF16 = 1, 2, 4, 8, 16, 32
EPI_LRELU, EPI_ACC_Y, EPI_Y2, EPI_SKIP_NOSTORE = 64, 128, 256, 512
_CODE = {torch.float32: F32, torch.bfloat16: BF16}


_DEV_INDEX = []


def stream():
    """Raw handle of the calling thread's current HIP stream (one device per process)."""
    if not _DEV_INDEX:
        _DEV_INDEX.append(torch.cuda.current_device())
    return torch._C._cuda_getCurrentRawStream(_DEV_INDEX[0])


def ptr(t):
    return None if t is None else t.data_ptr()


def _dev(*ts):
    for t in ts:
        if t is not None:
            if not t.is_cuda:
                raise RuntimeError("fs2 kernels need tensors on the GPU (no CPU path exists)")
            if not t.is_contiguous():
                raise RuntimeError("fs2 kernels need contiguous tensors")


def code(dtype):
    try:
        return _CODE[dtype]
    except KeyError:
        raise RuntimeError(f"unsupported compute dtype {dtype}") from None


def seed_arg(seed, device):
    """Dropout seed as the device pointer the kernels read: a device int64 tensor is passed
    through (the model's per-step seed), a host int is uploaded (tests, one-off calls)."""
    if torch.is_tensor(seed):
        if not seed.is_cuda or seed.dtype != torch.int64:
            raise RuntimeError("seed tensor must be a CUDA int64 tensor")
        return seed
    return torch.tensor([int(seed) & (2 ** 63 - 1)], dtype=torch.int64, device=device)


def ws(nbytes, device):
    return torch.empty(max(int(nbytes) // 4, 1), dtype=torch.float32, device=device)


def _copy(shape, copy, device):
    return None if copy is None else torch.empty(shape, dtype=copy, device=device)


# ------------------------------------------------------------------ GEMM / conv
def conv_gemm(x, wk, rows, seq_len, c_in, c_out, taps, pad, bias=None, flags=0, aux=None,
              out=None, ldx=None, out_dtype=torch.float32, lens=None):
    """y = conv(x) (+bias, epilogue flags); x/wk fp32 or bf16 (same), y fp32 or bf16.
    ``lens``: all-padding row tiles are not computed (see fs2_conv_gemm)."""
    _dev(x, wk, bias, aux, lens)
    if x.dtype != wk.dtype:
        raise RuntimeError(f"conv_gemm operand dtypes differ: {x.dtype} vs {wk.dtype}")
    if out is None:
        out = torch.empty(rows, c_out, dtype=out_dtype, device=x.device)
    if bias is not None:
        flags |= EPI_BIAS
    if out.dtype == torch.bfloat16:
        flags |= EPI_OUT_BF16
    if aux is not None and aux.dtype == torch.bfloat16:
        flags |= EPI_AUX_BF16
    lib.fs2_conv_gemm(code(x.dtype), ptr(x), ldx or c_in, ptr(wk), ptr(out), c_out, rows, seq_len,
                      c_in, c_out, taps, pad, ptr(lens), ptr(bias), flags, ptr(aux), c_out,
                      stream())
    return out


def conv_gemm_ln(x, wk, rows, seq_len, c_in, c_out, taps, pad, gamma, beta, bias=None, res=None,
                 lens=None, p_in=0.0, seed=0, site_in=0, copy=torch.bfloat16):
    """bf16 conv/Linear with the post-LayerNorm fused in (fs2_conv_gemm_ln): returns
    ``ln_fwd(conv_gemm(x) + bias, res=res, p_in=...)``'s (out fp32, out compute copy, xhat,
    rstd), bitwise, without the fp32 intermediate."""
    _dev(x, wk, gamma, beta, bias, res, lens)
    if x.dtype != torch.bfloat16 or wk.dtype != torch.bfloat16:
        raise RuntimeError("conv_gemm_ln: bf16 operands only")
    out = torch.empty(rows, c_out, dtype=torch.float32, device=x.device)
    out_t = _copy((rows, c_out), copy, x.device)
    xhat = torch.empty_like(out)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    sd = seed_arg(seed, x.device) if p_in > 0 else None
    lib.fs2_conv_gemm_ln(ptr(x), c_in, ptr(wk), rows, seq_len, c_in, c_out, taps, pad, ptr(lens),
                         ptr(bias), ptr(res), ptr(gamma), ptr(beta), ptr(out), ptr(out_t),
                         ptr(xhat), ptr(rstd), p_in, ptr(sd), site_in, stream())
    return out, out_t, xhat, rstd


def conv_gemm_ln_bwd(x, wk, rows, seq_len, c_in, c_out, taps, pad, xhat, rstd, gamma, dgamma,
                     dbeta, aux=None, lens=None, p_in=0.0, seed=0, site_in=0, dres=None,
                     dres_add=False, dbias_in=None, copy=torch.bfloat16):
    """bf16 conv/Linear whose output (+ aux) is a post-LayerNorm's upstream gradient, with that
    LayerNorm's backward in the epilogue (fs2_conv_gemm_ln_bwd): returns ``ln_bwd(conv_gemm(x,
    flags=ADD_AUX, aux=aux), ...)``'s (dy compute copy, dres); dgamma / dbeta / dbias_in
    accumulate."""
    _dev(x, wk, aux, xhat, rstd, gamma, dgamma, dbeta, dbias_in, lens, dres)
    if x.dtype != torch.bfloat16 or wk.dtype != torch.bfloat16:
        raise RuntimeError("conv_gemm_ln_bwd: bf16 operands only")
    if dres is None:
        dres = torch.empty(rows, c_out, dtype=torch.float32, device=x.device)
    dy_t = _copy((rows, c_out), copy, x.device)
    n = lib.fs2_ln_bwd_ws_bytes(rows, c_out)
    w = ws(n, x.device)
    sd = seed_arg(seed, x.device) if p_in > 0 else None
    lib.fs2_conv_gemm_ln_bwd(ptr(x), c_in, ptr(wk), rows, seq_len, c_in, c_out, taps, pad,
                             ptr(lens), ptr(aux), ptr(xhat), ptr(rstd), ptr(gamma), ptr(dgamma),
                             ptr(dbeta), ptr(dbias_in), p_in, ptr(sd), site_in, ptr(dres),
                             int(dres_add), ptr(dy_t), ptr(w), n, stream())
    return dy_t, dres


def conv_gemm_ex(x, wk, rows, seq_len, c_in, c_out, taps, pad, dilation=1, bias=None, flags=0,
                 aux=None, out=None, y2=None, alpha=0.1, scale=1.0, alpha2=0.1, lens=None):
    """Dilated conv with the vocoder epilogue (fs2_conv_gemm_ex): out and/or y2 (the
    leaky-ReLU'd compute copy, dtype of x) must be given; ACC_Y reads ``out`` first.
    ``lens`` (int64 per utterance, rows of this resolution): tiles past it may be skipped."""
    _dev(x, wk, bias, aux, out, y2, lens)
    if x.dtype != wk.dtype:
        raise RuntimeError(f"conv_gemm_ex operand dtypes differ: {x.dtype} vs {wk.dtype}")
    if out is None and y2 is None:
        raise RuntimeError("conv_gemm_ex: give out and/or y2")
    if y2 is not None:
        if y2.dtype != x.dtype or y2.shape != (rows, c_out):
            raise RuntimeError("conv_gemm_ex: y2 must be (rows, c_out) in the compute dtype")
        flags |= EPI_Y2
    if bias is not None:
        flags |= EPI_BIAS
    if out is not None and out.dtype == torch.bfloat16:
        flags |= EPI_OUT_BF16
    if aux is not None and aux.dtype == torch.bfloat16:
        flags |= EPI_AUX_BF16
    lib.fs2_conv_gemm_ex(code(x.dtype), ptr(x), c_in, ptr(wk), ptr(out), c_out, rows, seq_len,
                         c_in, c_out, taps, pad, dilation, ptr(lens), ptr(bias), flags, ptr(aux),
                         c_out, alpha, scale, ptr(y2), alpha2, stream())
    return out, y2


def convT_weight_prep(w, bias, stride):
    """ConvTranspose1d (c_in, c_out, 2*stride) weight -> (stride*c_out, c_in, 3) conv weight
    and the phase-tiled bias (fs2_convT_weight_prep)."""
    _dev(w, bias)
    c_in, c_out, k = w.shape
    if k != 2 * stride:
        raise RuntimeError(f"convT_weight_prep: kernel {k} != 2 * stride {stride}")
    wc = torch.empty(stride * c_out, c_in, 3, dtype=torch.float32, device=w.device)
    bc = torch.empty(stride * c_out, dtype=torch.float32, device=w.device)
    lib.fs2_convT_weight_prep(ptr(w), ptr(bias), c_in, c_out, stride, ptr(wc), ptr(bc), stream())
    return wc, bc


def resblock1_supported(channels, seq_len, kernel_size, dilations):
    d = (ctypes.c_int * 3)(*dilations)
    return bool(lib.fs2_resblock1_supported(channels, seq_len, kernel_size, ctypes.addressof(d)))


def resblock1_fused(x, rows, seq_len, channels, kernel_size, dilations, w1, w2, b1, b2, xs,
                    acc, scale, store_xs=True, hc=None, alpha2=0.1, lens=None):
    """One HiFi-GAN ResBlock1 in one launch (fs2_resblock1_fused): x (rows, C) fp32 ->
    xs (= (xs + out) * scale when acc, else out * scale) and / or hc (bf16 leaky ReLU)."""
    _dev(x, xs, hc, lens, *w1, *w2, *b1, *b2)
    if x.dtype != torch.float32 or xs.dtype != torch.float32:
        raise RuntimeError("resblock1_fused: x and xs are fp32")
    if any(w.dtype != torch.bfloat16 for w in (*w1, *w2)):
        raise RuntimeError("resblock1_fused: bf16 weights (fs2_conv_weight_prep)")
    P = lambda ts: (ctypes.c_void_p * 3)(*[t.data_ptr() for t in ts])
    d = (ctypes.c_int * 3)(*dilations)
    pw1, pw2, pb1, pb2 = P(w1), P(w2), P(b1), P(b2)
    rc = lib.fs2_resblock1_fused(ptr(x), rows, seq_len, channels, kernel_size,
                                 ctypes.addressof(d), ctypes.addressof(pw1), ctypes.addressof(pw2),
                                 ctypes.addressof(pb1), ctypes.addressof(pb2), ptr(xs), int(acc),
                                 float(scale), int(store_xs), ptr(hc), float(alpha2), ptr(lens),
                                 stream())
    return rc


def vocoder_post(x, rows, seq_len, c_in, w, bias, max_wav_value=32768.0, pcm=True, lens=None):
    _dev(x, w, bias, lens)
    wav = torch.empty(rows, dtype=torch.float32, device=x.device)
    p = torch.empty(rows, dtype=torch.int16, device=x.device) if pcm else None
    lib.fs2_vocoder_post(code(x.dtype), ptr(x), rows, seq_len, c_in, ptr(lens), ptr(w), ptr(bias),
                         max_wav_value, ptr(wav), ptr(p), stream())
    return wav, p


def weight_prep(w, c_out, c_in, taps, w_fwd=None, w_bwd=None):
    _dev(w)
    dt = (w_fwd if w_fwd is not None else w_bwd).dtype
    lib.fs2_conv_weight_prep(code(dt), ptr(w), c_out, c_in, taps, ptr(w_fwd), ptr(w_bwd), stream())


def conv_wgrad(dy, x, dw, rows, seq_len, c_in, c_out, taps, pad, db=None, ws_buf=None,
               on_stream=None, lens=None):
    """dw (+)= conv weight gradient; db (+)= column sums of dy when given (same launch).
    ``ws_buf``: caller-owned fp32 workspace (else one is allocated on the current stream)."""
    _dev(dy, x, dw, db)
    if dy.dtype != x.dtype:
        raise RuntimeError(f"conv_wgrad operand dtypes differ: {dy.dtype} vs {x.dtype}")
    n = lib.fs2_conv_wgrad_ws_bytes(rows, c_in, c_out, taps)
    if ws_buf is not None:
        if ws_buf.numel() * 4 < n:
            raise RuntimeError("conv_wgrad: workspace too small")
        w, n = ws_buf, ws_buf.numel() * 4
    else:
        w = ws(n, dy.device)
    lib.fs2_conv_wgrad(code(dy.dtype), ptr(dy), c_out, ptr(x), c_in, ptr(dw), ptr(db), rows,
                       seq_len, c_in, c_out, taps, pad, ptr(lens), ptr(w), n,
                       stream() if on_stream is None else on_stream)


def _k1_jobs(jobs):
    """ctypes int64 table {dy, ldy, x, ldx, dw, db, c_in, c_out} per job (host memory)."""
    arr = (ctypes.c_int64 * (8 * len(jobs)))()
    for j, (dy, x, dw, db, c_in, c_out) in enumerate(jobs):
        _dev(dy, x, dw, db)
        if dy.dtype != x.dtype:
            raise RuntimeError(f"conv_wgrad_k1_multi operand dtypes differ: {dy.dtype} vs {x.dtype}")
        arr[8 * j:8 * j + 8] = [dy.data_ptr(), c_out, x.data_ptr(), c_in, dw.data_ptr(),
                                0 if db is None else db.data_ptr(), c_in, c_out]
    return arr


def conv_wgrad_k1_multi_ws_bytes(jobs, rows):
    return lib.fs2_conv_wgrad_k1_multi_ws_bytes(_k1_jobs(jobs), len(jobs), rows)


def conv_wgrad_k1_multi(jobs, rows, seq_len, lens=None, ws_buf=None, on_stream=None):
    """Several k = 1 weight gradients over the same rows in one grouped launch:
    jobs = [(dy, x, dw, db_or_None, c_in, c_out), ...] (at most 4); dw (+)= dy^T x, db (+)=
    column sums of dy.  ``ws_buf``: caller-owned fp32 workspace."""
    arr = _k1_jobs(jobs)
    n = lib.fs2_conv_wgrad_k1_multi_ws_bytes(arr, len(jobs), rows)
    if ws_buf is not None:
        if ws_buf.numel() * 4 < n:
            raise RuntimeError("conv_wgrad_k1_multi: workspace too small")
        w, n = ws_buf, ws_buf.numel() * 4
    else:
        w = ws(n, jobs[0][0].device)
    lib.fs2_conv_wgrad_k1_multi(code(jobs[0][0].dtype), arr, len(jobs), rows, seq_len, ptr(lens),
                                ptr(w), n, stream() if on_stream is None else on_stream)


def colsum(x, rows, cols, out, accumulate=True):
    _dev(x, out)
    n = lib.fs2_colsum_ws_bytes(rows, cols)
    w = ws(n, x.device)
    lib.fs2_colsum(code(x.dtype), ptr(x), cols, rows, cols, ptr(out), int(accumulate), ptr(w), n,
                   stream())


def cast_bf16(x):
    _dev(x)
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    lib.fs2_cast_bf16(ptr(x), ptr(y), x.numel(), stream())
    return y


# ------------------------------------------------------------------ attention
def attn_fwd(qkv, lens, batch, seq_len, heads, d_head, scale):
    _dev(qkv, lens)
    o = torch.empty(batch * seq_len, heads * d_head, dtype=qkv.dtype, device=qkv.device)
    lse = torch.empty(batch * heads, seq_len, dtype=torch.float32, device=qkv.device)
    lib.fs2_attn_fwd(code(qkv.dtype), ptr(qkv), ptr(o), ptr(lse), ptr(lens), batch, seq_len, heads,
                     d_head, scale, stream())
    return o, lse


def attn_bwd(qkv, o, d_o, lse, lens, batch, seq_len, heads, d_head, scale):
    _dev(qkv, o, d_o, lse, lens)
    if not (qkv.dtype == o.dtype == d_o.dtype):
        raise RuntimeError("attn_bwd operands must share a dtype")
    dqkv = torch.empty_like(qkv)
    n = lib.fs2_attn_bwd_ws_bytes(batch, seq_len, heads)
    w = ws(n, qkv.device)
    lib.fs2_attn_bwd(code(qkv.dtype), ptr(qkv), ptr(o), ptr(d_o), ptr(lse), ptr(dqkv), ptr(lens),
                     batch, seq_len, heads, d_head, scale, ptr(w), n, stream())
    return dqkv


# ------------------------------------------------------------------ LayerNorm
def ln_fwd(y, gamma, beta, res=None, lens=None, seq_len=1, p_in=0.0, p_out=0.0, seed=0,
           site_in=0, site_out=0, dot_w=None, dot_b=None, copy=None):
    """Returns (out fp32, out compute copy or None, xhat, rstd, dot)."""
    _dev(y, gamma, beta, res, lens, dot_w, dot_b)
    rows, d = y.shape
    out = torch.empty_like(y)
    out_t = _copy(y.shape, copy, y.device)
    xhat = torch.empty_like(y)
    rstd = torch.empty(rows, dtype=torch.float32, device=y.device)
    dot = torch.empty(rows, dtype=torch.float32, device=y.device) if dot_w is not None else None
    sd = seed_arg(seed, y.device) if (p_in > 0 or p_out > 0) else None
    lib.fs2_ln_fwd(BF16 if copy is not None else F32, ptr(y), ptr(res), ptr(gamma), ptr(beta),
                   ptr(out), ptr(out_t), ptr(xhat), ptr(rstd), ptr(lens), seq_len, rows, d, p_in,
                   p_out, ptr(sd), site_in, site_out, ptr(dot_w), ptr(dot_b), ptr(dot), stream())
    return out, out_t, xhat, rstd, dot


def ln_bwd(xhat, rstd, gamma, beta, dgamma, dbeta, dout=None, ddot=None, dot_w=None,
           dw_dot=None, db_dot=None, lens=None, seq_len=1, p_in=0.0, p_out=0.0, seed=0,
           site_in=0, site_out=0, relu_y=None, dres=None, copy=None, dbias_in=None,
           dres_add=True):
    """Returns (dy fp32, dy compute copy or None); dbias_in (+)= column sums of dy.
    With a compute copy the fp32 dy is not produced (None): only the copy feeds the GEMMs."""
    _dev(xhat, rstd, gamma, beta, dout, ddot, dot_w, relu_y, dres, lens)
    rows, d = xhat.shape
    dy = torch.empty_like(xhat) if copy is None else None
    dy_t = _copy(xhat.shape, copy, xhat.device)
    n = lib.fs2_ln_bwd_ws_bytes(rows, d)
    w = ws(n, xhat.device)
    sd = seed_arg(seed, xhat.device) if (p_in > 0 or p_out > 0) else None
    lib.fs2_ln_bwd(BF16 if copy is not None else F32, ptr(dout), ptr(ddot), ptr(dot_w), ptr(xhat),
                   ptr(rstd), ptr(gamma), ptr(beta), ptr(lens), seq_len, rows, d, p_in, p_out,
                   ptr(sd), site_in, site_out, ptr(relu_y), ptr(dy), ptr(dy_t), ptr(dres),
                   int(dres_add), ptr(dgamma), ptr(dbeta), ptr(dw_dot), ptr(db_dot), ptr(dbias_in),
                   ptr(w), n, stream())
    return dy, dy_t


# ------------------------------------------------------------------ BatchNorm
def bn_fwd(z, gamma, beta, running_mean, running_var, act_tanh, p, seed, site, res=None,
           eps=1e-5, momentum=0.1, copy=None, want_out=True, num_batches_tracked=None):
    """(out fp32 or None when only the copy is wanted, out copy or None, mean, rstd);
    ``num_batches_tracked`` (device int64) is incremented in the statistics launch."""
    _dev(z, gamma, beta, running_mean, running_var, res, num_batches_tracked)
    rows, c = z.shape
    out = torch.empty_like(z) if (want_out or copy is None) else None
    out_t = _copy(z.shape, copy, z.device)
    mean = torch.empty(c, dtype=torch.float32, device=z.device)
    rstd = torch.empty(c, dtype=torch.float32, device=z.device)
    n = lib.fs2_bn_ws_bytes(rows, c)
    w = ws(n, z.device)
    sd = seed_arg(seed, z.device) if p > 0 else None
    lib.fs2_bn_fwd(BF16 if copy is not None else F32, ptr(z), rows, c, ptr(gamma), ptr(beta), eps,
                   momentum, ptr(running_mean), ptr(running_var), ptr(mean), ptr(rstd),
                   int(act_tanh), p, ptr(sd), site, ptr(res), ptr(out), ptr(out_t), ptr(w), n,
                   ptr(num_batches_tracked), stream())
    return out, out_t, mean, rstd


def bn_eval_fwd(z, gamma, beta, running_mean, running_var, act_tanh, res=None, eps=1e-5,
                copy=None, want_out=True):
    """Eval-mode BatchNorm1d (running statistics, no dropout): (out or None, out copy or None)."""
    _dev(z, gamma, beta, running_mean, running_var, res)
    rows, c = z.shape
    out = torch.empty_like(z) if (want_out or copy is None) else None
    out_t = _copy(z.shape, copy, z.device)
    mean = torch.empty(c, dtype=torch.float32, device=z.device)
    rstd = torch.empty(c, dtype=torch.float32, device=z.device)
    lib.fs2_bn_eval_fwd(BF16 if copy is not None else F32, ptr(z), rows, c, ptr(gamma), ptr(beta),
                        eps, ptr(running_mean), ptr(running_var), ptr(mean), ptr(rstd),
                        int(act_tanh), ptr(res), ptr(out), ptr(out_t), stream())
    return out, out_t


def bn_bwd(dout, z, mean, rstd, gamma, beta, dgamma, dbeta, act_tanh, p, seed, site, copy=None):
    _dev(dout, z, mean, rstd, gamma, beta, dgamma, dbeta)
    rows, c = z.shape
    dz = torch.empty_like(z) if copy is None else None  # with a copy only it feeds the GEMMs
    dz_t = _copy(z.shape, copy, z.device)
    n = lib.fs2_bn_ws_bytes(rows, c)
    w = ws(n, z.device)
    sd = seed_arg(seed, z.device) if p > 0 else None
    lib.fs2_bn_bwd(BF16 if copy is not None else F32, ptr(dout), ptr(z), ptr(mean), ptr(rstd),
                   ptr(gamma), ptr(beta), rows, c, int(act_tanh), p, ptr(sd), site, ptr(dz),
                   ptr(dz_t), ptr(dgamma), ptr(dbeta), ptr(w), n, stream())
    return dz, dz_t


# ------------------------------------------------------------------ embeddings / adaptor
def encoder_embed(texts, accents, word_emb, accent_emb, posenc, batch, seq_len, d, copy=None):
    _dev(texts, accents, word_emb, accent_emb, posenc)
    out = torch.empty(batch * seq_len, d, dtype=torch.float32, device=word_emb.device)
    out_t = _copy(out.shape, copy, out.device)
    lib.fs2_encoder_embed_fwd(ptr(texts), ptr(accents), ptr(word_emb), ptr(accent_emb), ptr(posenc),
                              batch, seq_len, d, ptr(out), ptr(out_t), stream())
    return out, out_t


def embedding_fwd(ids, table):
    _dev(ids, table)
    n, d = ids.numel(), table.shape[1]
    out = torch.empty(n, d, dtype=torch.float32, device=table.device)
    lib.fs2_embedding_fwd(ptr(ids), ptr(table), n, d, ptr(out), stream())
    return out


def embedding_bwd(dout, ids, dtable, padding_idx=-1):
    _dev(dout, ids, dtable)
    n = lib.fs2_embedding_bwd_ws_bytes(ids.numel(), dtable.shape[1], dtable.shape[0])
    w = ws(n, dout.device)
    lib.fs2_embedding_bwd(ptr(dout), ptr(ids), ids.numel(), dtable.shape[1], padding_idx,
                          ptr(dtable), dtable.shape[0], ptr(w), n, stream())


def length_mask(lens, max_len):
    _dev(lens)
    m = torch.empty(lens.numel(), max_len, dtype=torch.bool, device=lens.device)
    lib.fs2_length_mask(ptr(lens), lens.numel(), max_len, ptr(m), stream())
    return m


def rowvec_add(x, ids, table, batch, seq_len, copy=None):
    _dev(x, ids, table)
    out = torch.empty_like(x)
    out_t = _copy(x.shape, copy, x.device)
    lib.fs2_rowvec_add_fwd(ptr(x), ptr(ids), ptr(table), batch, seq_len, x.shape[1], ptr(out),
                           ptr(out_t), stream())
    return out, out_t


def rowvec_add_bwd(dout, ids, dtable, batch, seq_len):
    _dev(dout, ids, dtable)
    lib.fs2_rowvec_add_bwd(ptr(dout), ptr(ids), batch, seq_len, dout.shape[1], ptr(dtable), stream())


def _vals_dtype(v):
    if v.dtype == torch.float32:
        return F32
    if v.dtype == torch.float64:
        return F64
    raise RuntimeError(f"bucketize values must be float32/float64, got {v.dtype}")


def bucket_embed(x, values, bins, table, copy=None):
    _dev(x, values, bins, table)
    rows, d = x.shape
    out = torch.empty_like(x)
    out_t = _copy(x.shape, copy, x.device)
    idx = torch.empty(rows, dtype=torch.int32, device=x.device)
    lib.fs2_bucket_embed_fwd(ptr(x), ptr(values), _vals_dtype(values), ptr(bins), bins.numel(),
                             ptr(table), rows, d, ptr(out), ptr(out_t), ptr(idx), stream())
    return out, out_t, idx


def bucket_embed_bwd(dout, idx, dtable):
    _dev(dout, idx, dtable)
    n = lib.fs2_embedding_bwd_ws_bytes(idx.numel(), dout.shape[1], dtable.shape[0])
    w = ws(n, dout.device)
    lib.fs2_bucket_embed_bwd(ptr(dout), ptr(idx), idx.numel(), dout.shape[1], ptr(dtable),
                             dtable.shape[0], ptr(w), n, stream())


def bucketize(values, bins):
    _dev(values, bins)
    idx = torch.empty(values.shape, dtype=torch.int32, device=values.device)
    lib.fs2_bucketize(ptr(values), _vals_dtype(values), ptr(bins), bins.numel(), values.numel(),
                      ptr(idx), stream())
    return idx


def lr_index(durations):
    _dev(durations)
    B, Ts = durations.shape
    if durations.dtype == torch.int64:
        dt = 0
    elif durations.dtype == torch.float32:
        dt = 1
    else:
        raise RuntimeError(f"durations must be int64 or float32, got {durations.dtype}")
    cum = torch.empty(B, Ts, dtype=torch.int32, device=durations.device)
    mel_len = torch.empty(B, dtype=torch.int64, device=durations.device)
    lib.fs2_lr_index(ptr(durations), dt, B, Ts, ptr(cum), ptr(mel_len), stream())
    return cum, mel_len


def duration_round(log_d, d_control=1.0):
    """Inference durations: clamp(round(exp(log_d) - 1) * d_control, min=0) (f32)."""
    _dev(log_d)
    if log_d.dtype != torch.float32:
        raise RuntimeError(f"log durations must be float32, got {log_d.dtype}")
    x = log_d.contiguous()
    out = torch.empty_like(x)
    lib.fs2_duration_round(ptr(x), x.numel(), float(d_control), ptr(out), stream())
    return out


def lr_source(cum, out_len):
    _dev(cum)
    B, Ts = cum.shape
    src = torch.empty(B, out_len, dtype=torch.int32, device=cum.device)
    lib.fs2_lr_source(ptr(cum), B, Ts, out_len, ptr(src), stream())
    return src


def lr_expand(x, cum, out_len, posenc=None, copy=None):
    _dev(x, cum, posenc)
    B, Ts = cum.shape
    d = x.shape[-1]
    out = torch.empty(B * out_len, d, dtype=torch.float32, device=x.device)
    out_t = _copy(out.shape, copy, x.device)
    lib.fs2_lr_expand_fwd(ptr(x), ptr(cum), B, Ts, out_len, d, ptr(posenc), ptr(out), ptr(out_t),
                          stream())
    return out, out_t


def lr_expand_bwd(dout, cum, out_len, d):
    _dev(dout, cum)
    B, Ts = cum.shape
    dx = torch.empty(B * Ts, d, dtype=torch.float32, device=dout.device)
    lib.fs2_lr_expand_bwd(ptr(dout), ptr(cum), B, Ts, out_len, d, ptr(dx), stream())
    return dx


# ------------------------------------------------------------------ losses / GMM
def fs2loss_fwd(mel_out, post_out, mel_tgt, p, e, logd, p_t, e_t, d_t, src_pad, mel_pad,
                denoms=None):
    _dev(mel_out, post_out, mel_tgt, p, e, logd, p_t, e_t, d_t, src_pad, mel_pad, denoms)
    B, Tm, n_mel = mel_out.shape
    Ts = p.shape[1]
    losses = torch.empty(6, dtype=torch.float32, device=mel_out.device)
    n = lib.fs2_fs2loss_ws_bytes(B, Tm)
    w = ws(n, mel_out.device)
    lib.fs2_fs2loss_fwd(ptr(mel_out), ptr(post_out), ptr(mel_tgt), mel_tgt.shape[1], ptr(p), ptr(e),
                        ptr(logd), ptr(p_t), ptr(e_t), ptr(d_t), ptr(src_pad), ptr(mel_pad), B, Ts,
                        Tm, n_mel, ptr(denoms), ptr(losses), ptr(w), n, stream())
    return losses, w


def fs2loss_bwd(mel_out, post_out, mel_tgt, p, e, logd, p_t, e_t, d_t, src_pad, mel_pad, w, g6):
    B, Tm, n_mel = mel_out.shape
    Ts = p.shape[1]
    outs = [torch.empty_like(t) for t in (mel_out, post_out, p, e, logd)]
    lib.fs2_fs2loss_bwd(ptr(mel_out), ptr(post_out), ptr(mel_tgt), mel_tgt.shape[1], ptr(p), ptr(e),
                        ptr(logd), ptr(p_t), ptr(e_t), ptr(d_t), ptr(src_pad), ptr(mel_pad), B, Ts,
                        Tm, n_mel, ptr(w), ptr(g6), *[ptr(o) for o in outs], stream())
    return outs


def gmm_head_fwd(meta, w_pi, b_pi, w_s, b_s, w_mu, b_mu, K, D):
    _dev(meta, w_pi, b_pi, w_s, b_s, w_mu, b_mu)
    B, in_dim = meta.shape
    dev = meta.device
    pi = torch.empty(B, K, dtype=torch.float32, device=dev)
    sigma = torch.empty(B, K, D, dtype=torch.float32, device=dev)
    mu = torch.empty(B, K, D, dtype=torch.float32, device=dev)
    sigma_pre = torch.empty(B, K, D, dtype=torch.float32, device=dev)
    lib.fs2_gmm_head_fwd(ptr(meta), B, in_dim, K, D, ptr(w_pi), ptr(b_pi), ptr(w_s), ptr(b_s),
                         ptr(w_mu), ptr(b_mu), ptr(pi), ptr(sigma), ptr(mu), ptr(sigma_pre), stream())
    return pi, mu, sigma, sigma_pre


def gmm_logprob(e, pi, mu, sigma, want_mean=False, denom=None):
    _dev(e, pi, mu, sigma, denom)
    B, K, D = mu.shape
    logp = torch.empty(B, dtype=torch.float32, device=e.device)
    resp = torch.empty(B, K, dtype=torch.float32, device=e.device)
    mean = torch.empty((), dtype=torch.float32, device=e.device) if want_mean else None
    lib.fs2_gmm_logprob(ptr(e), ptr(pi), ptr(mu), ptr(sigma), B, K, D, ptr(logp), ptr(resp),
                        ptr(mean), ptr(denom), stream())
    return logp, resp, mean


def dp_counts(src_lens, mel_lens, src_len, mel_len, n_mel):
    _dev(src_lens, mel_lens)
    out = torch.empty(3, dtype=torch.float32, device=src_lens.device)
    lib.fs2_dp_counts(ptr(src_lens), ptr(mel_lens), src_lens.numel(), src_len, mel_len, n_mel,
                      ptr(out), stream())
    return out


def gmm_head_bwd(meta, e, pi, mu, sigma, sigma_pre, resp, g_logp, grads):
    B, K, D = mu.shape
    lib.fs2_gmm_head_bwd(ptr(meta), ptr(e), ptr(pi), ptr(mu), ptr(sigma), ptr(sigma_pre), ptr(resp),
                         ptr(g_logp), B, meta.shape[1], K, D, *[ptr(g) for g in grads], stream())


def gmm_sample(pi, mu, sigma, seed, offset=0):
    _dev(pi, mu, sigma)
    B, K, D = mu.shape
    out = torch.empty(B, D, dtype=torch.float32, device=mu.device)
    comp = torch.empty(B, dtype=torch.int32, device=mu.device)
    lib.fs2_gmm_sample(ptr(pi), ptr(mu), ptr(sigma), B, K, D, seed, offset, ptr(out), ptr(comp),
                       stream())
    return out, comp


# ------------------------------------------------------------------ optimiser / misc
def grad_norm(g, max_norm, norm_coef):
    n = lib.fs2_grad_norm_ws_bytes(g.numel())
    w = ws(n, g.device)
    lib.fs2_grad_norm(ptr(g), g.numel(), float(max_norm), ptr(norm_coef), ptr(w), n, stream())


def adam_step(p, g, m, v, norm_coef, lr, beta1, beta2, eps, bc1, bc2_sqrt, hyper=None):
    """Adam over flat buffers; with ``hyper`` (device [lr, bc1, bc2_sqrt], see sched_step) the
    scalar lr/bc1/bc2_sqrt arguments are ignored."""
    lib.fs2_adam_step(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), ptr(norm_coef), float(lr),
                      float(beta1), float(beta2), float(eps), float(bc1), float(bc2_sqrt),
                      ptr(hyper), stream())


def sched_step(steps, hyper, init_lr, n_warmup, anneal_steps, anneal_rate, beta1, beta2,
               advance_lr=True):
    """Device-side LR schedule + Adam bias corrections for one step (fs2_sched_step)."""
    an = (ctypes.c_int64 * 3)(*[int(a) for a in anneal_steps][:3])
    lib.fs2_sched_step(ptr(steps), ptr(hyper), float(init_lr), int(n_warmup), ctypes.addressof(an),
                       len(anneal_steps), float(anneal_rate), float(beta1), float(beta2),
                       int(advance_lr), stream())


def seed_next(state):
    """state: device int64[3] {base, counter, current}; advances the per-step dropout seed."""
    lib.fs2_seed_next(ptr(state), stream())


def fill_(t, value):
    _dev(t)
    lib.fs2_fill(ptr(t), t.numel(), float(value), stream())
    return t


def zeros(shape, device):
    return fill_(torch.empty(shape, dtype=torch.float32, device=device), 0.0)


def add(a, b, out=None):
    _dev(a, b)
    out = torch.empty_like(a) if out is None else out
    lib.fs2_add(ptr(out), ptr(a), ptr(b), a.numel(), stream())
    return out


def scale_(t, value):
    """t *= value in place (f32)."""
    _dev(t)
    lib.fs2_scale(ptr(t), t.numel(), float(value), stream())
    return t


def add_i64_(t, value):
    _dev(t)
    lib.fs2_add_i64(ptr(t), t.numel(), int(value), stream())
    return t


# ------------------------------------------------------------------ mid-attribute GMMs
def gmm_w2_cost(mu_a, sd_a, mu_b, sd_b):
    """(ka, kb) float64 cost of InterpolateGMM._w2sq (distributions.py:64-77)."""
    _dev(mu_a, sd_a, mu_b, sd_b)
    ka, d = mu_a.shape
    kb = mu_b.shape[0]
    cost = torch.empty(ka, kb, dtype=torch.float64, device=mu_a.device)
    lib.fs2_gmm_w2_cost(ptr(mu_a), ptr(sd_a), ka, ptr(mu_b), ptr(sd_b), kb, d, ptr(cost), stream())
    return cost


def ot_emd(a, b, cost, max_iter=10000):
    """Exact OT plan (ot.emd): (plan float64 (ka, kb), status int32[1] = iterations or -1)."""
    _dev(a, b, cost)
    ka, kb = cost.shape
    plan = torch.empty(ka, kb, dtype=torch.float64, device=cost.device)
    status = torch.empty(1, dtype=torch.int32, device=cost.device)
    lib.fs2_ot_emd(ptr(a), ptr(b), ptr(cost), ka, kb, int(max_iter), ptr(plan), ptr(status),
                   stream())
    return plan, status


def gmm_interpolate(plan, mu_a, sd_a, mu_b, sd_b, t):
    _dev(plan, mu_a, sd_a, mu_b, sd_b)
    ka, d = mu_a.shape
    kb = mu_b.shape[0]
    n = ka * kb
    pi = torch.empty(n, dtype=torch.float32, device=mu_a.device)
    mu = torch.empty(n, d, dtype=torch.float32, device=mu_a.device)
    sd = torch.empty(n, d, dtype=torch.float32, device=mu_a.device)
    lib.fs2_gmm_interpolate(ptr(plan), ptr(mu_a), ptr(sd_a), ka, ptr(mu_b), ptr(sd_b), kb, d,
                            float(t), ptr(pi), ptr(mu), ptr(sd), stream())
    return pi, mu, sd


def gmm_barycenter(mu, sd, rate32, iters=60):
    """Barycenter mean/std of every position of product(range(k), repeat=m)."""
    _dev(mu, sd, rate32)
    m, k, d = mu.shape
    n_pos = lib.fs2_gmm_barycenter_positions(m, k)
    if n_pos <= 0:
        raise RuntimeError(f"{k}^{m} barycenter positions exceed the kernel's limit")
    bm = torch.empty(n_pos, d, dtype=torch.float32, device=mu.device)
    bs = torch.empty(n_pos, d, dtype=torch.float32, device=mu.device)
    lib.fs2_gmm_barycenter(ptr(mu), ptr(sd), m, k, d, ptr(rate32), int(iters), ptr(bm), ptr(bs),
                           stream())
    return bm, bs


def gmm_bary_mix(pi, mu, sd, rate64, bm, bs):
    """Nearest-barycenter mixture: (n_used int32[1], used, pi, mu, sd) with capacity m*k
    (rows past n_used are unwritten)."""
    _dev(pi, mu, sd, rate64, bm, bs)
    m, k, d = mu.shape
    dev = mu.device
    n_used = torch.empty(1, dtype=torch.int32, device=dev)
    used = torch.empty(m * k, dtype=torch.int32, device=dev)
    pi_o = torch.empty(m * k, dtype=torch.float32, device=dev)
    mu_o = torch.empty(m * k, d, dtype=torch.float32, device=dev)
    sd_o = torch.empty(m * k, d, dtype=torch.float32, device=dev)
    n = lib.fs2_gmm_bary_mix_ws_bytes(m, k)
    w = torch.empty(max(n // 8, 1), dtype=torch.float64, device=dev)
    lib.fs2_gmm_bary_mix(ptr(pi), ptr(mu), ptr(sd), m, k, d, ptr(rate64), ptr(bm), ptr(bs),
                         ptr(n_used), ptr(used), ptr(pi_o), ptr(mu_o), ptr(sd_o), ptr(w), n,
                         stream())
    return n_used, used, pi_o, mu_o, sd_o
