"""Per-kernel numerics on the GPU: each HIP entry point against a plain PyTorch fp32
reference of the same op (and against the oracle's bit-exact index math where the op is
integer).  Tolerances: fp32 GEMM/attention/norm paths 1e-4 relative-to-scale."""
import importlib
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from oracle import index_math

pytestmark = pytest.mark.gpu
K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
DEV = "cuda"


def close(a, b, tol=1e-4):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    scale = max(b.abs().max().item(), 1e-6)
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"max abs err {err:.3e} vs scale {scale:.3e}"


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def ref_conv(x, w, b, B, T, pad):
    """x (B*T, Cin), w (Cout, Cin, k) -> (B*T, Cout), zero padding per utterance."""
    y = F.conv1d(x.view(B, T, -1).transpose(1, 2), w, b, padding=pad)
    return y.transpose(1, 2).reshape(B * T, -1)


@pytest.mark.parametrize("B,T,cin,cout,k", [(2, 37, 256, 1024, 9), (3, 50, 1024, 256, 1),
                                            (2, 64, 80, 512, 5), (1, 33, 512, 80, 5),
                                            (4, 16, 256, 768, 1), (5, 130, 256, 256, 3)])
def test_conv_gemm_fwd_dx_dw(B, T, cin, cout, k):
    pad = (k - 1) // 2
    x = rnd(B * T, cin, seed=1)
    w = rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=2)
    b = rnd(cout, seed=3)
    wf = torch.empty(cout * cin * k, device=DEV)
    wb = torch.empty(cout * cin * k, device=DEV)
    K.weight_prep(w, cout, cin, k, wf, wb)
    y = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b)
    close(y, ref_conv(x, w, b, B, T, pad))
    yr = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b, flags=K.EPI_RELU)
    close(yr, F.relu(ref_conv(x, w, b, B, T, pad)))
    # data gradient through the flipped weights, with residual fusion
    dy = rnd(B * T, cout, seed=4)
    xr = x.clone().requires_grad_()
    ref_y = ref_conv(xr, w, b, B, T, pad)
    ref_y.backward(dy)
    aux = rnd(B * T, cin, seed=5)
    dx = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX, aux=aux)
    close(dx, xr.grad + aux)
    # weight gradient (accumulating) and bias gradient
    wr = w.clone().requires_grad_()
    br = b.clone().requires_grad_()
    ref_conv(x, wr, br, B, T, pad).backward(dy)
    dw = torch.full_like(w, 0.5)
    K.conv_wgrad(dy, x, dw, B * T, T, cin, cout, k, pad)
    close(dw, wr.grad + 0.5)
    db = torch.zeros(cout, device=DEV)
    K.colsum(dy, B * T, cout, db)
    close(db, br.grad)
    dw2, db2 = torch.zeros_like(w), torch.full((cout,), 0.25, device=DEV)
    K.conv_wgrad(dy, x, dw2, B * T, T, cin, cout, k, pad, db=db2)
    close(dw2, wr.grad)
    close(db2, br.grad + 0.25)


def test_conv_gemm_relu_mask():
    M, cin, cout = 200, 256, 512
    x, w = rnd(M, cin, seed=1), rnd(cout, cin, 1, scale=0.06, seed=2)
    aux = rnd(M, cout, seed=3)
    y = K.conv_gemm(x, w.reshape(cout, cin).contiguous(), M, M, cin, cout, 1, 0,
                    flags=K.EPI_RELU_MASK_AUX, aux=aux)
    close(y, (x @ w.view(cout, cin).t()) * (aux > 0))


def ref_attn(qkv, lens, B, T, H, dh):
    q, k, v = qkv.view(B, T, 3, H, dh).unbind(2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(dh)
    pad = torch.arange(T, device=qkv.device)[None, :] >= lens[:, None]
    s = s.masked_fill(pad[:, None, None, :], -float("inf"))
    o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v)
    return o.reshape(B * T, H * dh)


@pytest.mark.parametrize("B,T,lens", [(2, 64, [64, 40]), (3, 130, [130, 77, 1]),
                                      (2, 512, [512, 300])])
def test_attention_fwd_bwd(B, T, lens):
    H, dh = 2, 128
    lens_t = torch.tensor(lens, device=DEV)
    qkv = rnd(B * T, 3 * H * dh, seed=7)
    o, lse = K.attn_fwd(qkv, lens_t, B, T, H, dh, 1 / math.sqrt(dh))
    qr = qkv.clone().requires_grad_()
    ro = ref_attn(qr, lens_t, B, T, H, dh)
    valid = (torch.arange(T, device=DEV)[None, :] < lens_t[:, None]).reshape(-1)
    close(o[valid], ro[valid])
    # padded query rows are don't-care downstream (Layers.py:25 zeroes them) but must be
    # finite; query tiles entirely past the length are not computed and hold zeros
    assert torch.isfinite(o[~valid].float()).all()
    skipped = (torch.arange(T, device=DEV)[None, :] >= (lens_t[:, None] + 127) // 128 * 128).reshape(-1)
    assert torch.all(o[skipped] == 0)
    do = rnd(B * T, H * dh, seed=8) * valid[:, None]
    ro.backward(do)
    dqkv = K.attn_bwd(qkv, o, do, lse, lens_t, B, T, H, dh, 1 / math.sqrt(dh))
    close(dqkv, qr.grad)


@pytest.mark.parametrize("mode", ["res_mask", "plain_dropout", "dot", "relu_drop"])
def test_layernorm(mode):
    B, T, d = 3, 40, 256
    M = B * T
    lens = torch.tensor([40, 23, 7], device=DEV)
    pad = (torch.arange(T, device=DEV)[None] >= lens[:, None]).reshape(-1)
    y = rnd(M, d, seed=1)
    if mode == "relu_drop":
        y = F.relu(y)
    res = rnd(M, d, seed=2)
    g, bta = 1 + 0.1 * rnd(d, seed=3), 0.1 * rnd(d, seed=4)
    w, wb = rnd(d, seed=5) * 0.1, rnd(1, seed=6)
    p = 0.0 if mode in ("res_mask", "dot") else 0.3
    kw = dict(seed=123, site_in=7, site_out=9)
    if mode == "res_mask":
        out, _, xh, rs, _ = K.ln_fwd(y, g, bta, res=res, lens=lens, seq_len=T, **kw)
        ref = F.layer_norm(y + res, (d,), g, bta, 1e-5).masked_fill(pad[:, None], 0)
        close(out, ref, 2e-5)
    elif mode == "dot":
        out, _, xh, rs, dot = K.ln_fwd(y, g, bta, lens=lens, seq_len=T, dot_w=w, dot_b=wb, **kw)
        ref_u = F.layer_norm(y, (d,), g, bta, 1e-5)
        close(out, ref_u, 2e-5)
        close(dot, (ref_u @ w + wb).masked_fill(pad, 0), 2e-5)
    else:
        out, _, xh, rs, _ = K.ln_fwd(y, g, bta, p_out=p, **kw)
        ref_u = F.layer_norm(y, (d,), g, bta, 1e-5)
        keep = out != 0
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 0.03, frac  # Philox keep-rate
        close(out[keep], (ref_u / (1 - p))[keep], 2e-5)
        mask = keep.float() / (1 - p)
    # backward against autograd on the same (recovered) dropout mask
    yr, gr, br = y.clone().requires_grad_(), g.clone().requires_grad_(), bta.clone().requires_grad_()
    dg, db = torch.zeros(d, device=DEV), torch.zeros(d, device=DEV)
    if mode == "res_mask":
        rr = res.clone().requires_grad_()
        ref = F.layer_norm(yr + rr, (d,), gr, br, 1e-5).masked_fill(pad[:, None], 0)
        dout = rnd(M, d, seed=11)
        ref.backward(dout)
        dres = torch.zeros(M, d, device=DEV)
        dy, _ = K.ln_bwd(xh, rs, g, bta, dg, db, dout=dout, lens=lens, seq_len=T, dres=dres, **kw)
        close(dy, yr.grad)
        close(dres, rr.grad)
        dres2 = torch.full((M, d), 7.0, device=DEV)  # overwrite mode ignores the old contents
        K.ln_bwd(xh, rs, g, bta, dg.clone(), db.clone(), dout=dout, lens=lens, seq_len=T,
                 dres=dres2, dres_add=False, **kw)
        close(dres2, rr.grad)
    elif mode == "dot":
        wr, wbr = w.clone().requires_grad_(), wb.clone().requires_grad_()
        ref = (F.layer_norm(yr, (d,), gr, br, 1e-5) @ wr + wbr).masked_fill(pad, 0)
        ddot = rnd(M, seed=12)
        ref.backward(ddot)
        dw, dwb = torch.zeros(d, device=DEV), torch.zeros(1, device=DEV)
        dy, _ = K.ln_bwd(xh, rs, g, bta, dg, db, ddot=ddot, dot_w=w, dw_dot=dw, db_dot=dwb,
                      lens=lens, seq_len=T, **kw)
        close(dy, yr.grad)
        close(dw, wr.grad)
        close(dwb, wbr.grad)
    else:
        ref = F.layer_norm(yr, (d,), gr, br, 1e-5) * mask
        dout = rnd(M, d, seed=13)
        ref.backward(dout)
        relu_y = y if mode == "relu_drop" else None
        dy, _ = K.ln_bwd(xh, rs, g, bta, dg, db, dout=dout, p_out=p, relu_y=relu_y, **kw)
        want = yr.grad * (y > 0) if relu_y is not None else yr.grad
        close(dy, want)
    close(dg, gr.grad)
    close(db, br.grad)


@pytest.mark.parametrize("act,res", [(True, False), (False, True)])
def test_batchnorm(act, res):
    M, c = 700, 80 if res else 512
    z = rnd(M, c, seed=1) * 3 + 1
    g, b = 1 + 0.1 * rnd(c, seed=2), 0.1 * rnd(c, seed=3)
    rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    r = rnd(M, c, seed=4) if res else None
    nbt = torch.tensor(5, dtype=torch.int64, device=DEV)
    out, _, mean, rstd = K.bn_fwd(z, g, b, rm, rv, act, 0.0, 1, 2, res=r, num_batches_tracked=nbt)
    assert nbt.item() == 6  # BatchNorm1d's counter, advanced in the statistics launch
    zr, gr, br = z.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    rm2, rv2 = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    ref = F.batch_norm(zr, rm2, rv2, gr, br, training=True, momentum=0.1, eps=1e-5)
    if act:
        ref = torch.tanh(ref)
    if res:
        ref = ref + r
    close(out, ref, 2e-5)
    close(rm, rm2, 1e-5)
    close(rv, rv2, 1e-5)
    dout = rnd(M, c, seed=5)
    ref.backward(dout)
    dg, db = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)
    dz, _ = K.bn_bwd(dout, z, mean, rstd, g, b, dg, db, act, 0.0, 1, 2)
    close(dz, zr.grad)
    close(dg, gr.grad)
    close(db, br.grad)


def test_length_regulator_golden_and_random():
    g = load_golden("g1_lr.npz")
    for name in ("int", "flt", "crop", "pad"):
        d = torch.from_numpy(g[f"d_{name}"]).to(DEV)
        d = d.float() if d.dtype == torch.float64 else d
        ml = int(g[f"maxlen_{name}"])
        x = torch.from_numpy(g["x"]).to(DEV)
        cum, mel_len = K.lr_index(d)
        T = ml if ml >= 0 else int(mel_len.max())
        src = K.lr_source(cum, T)
        want_src, want_len = index_math.lr_source_map(g[f"d_{name}"], None if ml < 0 else ml)
        np.testing.assert_array_equal(src.cpu().numpy(), want_src)
        np.testing.assert_array_equal(mel_len.cpu().numpy(), g[f"len_{name}"])
    # random ragged durations at model width, fwd (+posenc) and segmented-sum bwd
    rng = np.random.default_rng(5)
    B, Ts, d = 6, 37, 256
    dur = torch.from_numpy(rng.integers(-1, 9, size=(B, Ts))).to(DEV)
    x = rnd(B * Ts, d, seed=3)
    pos = rnd(300, d, seed=4)
    cum, mel_len = K.lr_index(dur)
    for T in (int(mel_len.max()), 100):
        out, _ = K.lr_expand(x, cum, T, posenc=pos)
        src, ml = index_math.lr_source_map(dur.cpu().numpy(), T)
        np.testing.assert_array_equal(K.lr_source(cum, T).cpu().numpy(), src)
        np.testing.assert_array_equal(mel_len.cpu().numpy(), ml)
        xs = x.view(B, Ts, d)
        want = torch.stack([torch.where(torch.from_numpy(src[b] >= 0).to(DEV)[:, None],
                                        xs[b][torch.from_numpy(np.maximum(src[b], 0)).to(DEV)], 0)
                            for b in range(B)]).reshape(B * T, d) + pos[:T].repeat(B, 1)
        close(out, want, 1e-6)
        dout = rnd(B * T, d, seed=9)
        dx = K.lr_expand_bwd(dout, cum, T, d)
        xr = xs.clone().requires_grad_()
        idx = torch.from_numpy(np.maximum(src, 0)).to(DEV)
        g2 = torch.stack([xr[b][idx[b]] for b in range(B)]) * torch.from_numpy(src >= 0).to(DEV)[..., None]
        g2.backward(dout.view(B, T, d))
        close(dx, xr.grad.reshape(B * Ts, d), 1e-5)


def test_bucketize_golden():
    g = load_golden("g3_bucket.npz")
    bins = torch.from_numpy(g["bins"]).to(DEV)
    assert K.bucketize(torch.from_numpy(g["v"]).to(DEV), bins).cpu().tolist() == g["idx"].tolist()
    pb = torch.from_numpy(g["pitch_bins"]).to(DEV)
    eb = torch.from_numpy(g["energy_bins"]).to(DEV)
    v = torch.from_numpy(g["v_rand"]).to(DEV)
    np.testing.assert_array_equal(K.bucketize(v, pb).cpu().numpy(), g["pitch_idx"])
    np.testing.assert_array_equal(K.bucketize(v, eb).cpu().numpy(), g["energy_idx"])
    np.testing.assert_array_equal(K.bucketize(torch.from_numpy(g["v_edge"]).to(DEV), pb).cpu().numpy(),
                                  g["edge_idx"])
    np.testing.assert_array_equal(K.bucketize(v.double(), pb).cpu().numpy(),
                                  index_math.bucketize(g["v_rand"].astype(np.float64), g["pitch_bins"]))


def test_embeddings():
    B, T, d = 3, 11, 256
    texts = torch.randint(0, 429, (B, T), device=DEV)
    texts[0, -3:] = 0
    acc = torch.randint(0, 5, (B, T), device=DEV)
    wt, at, pos = rnd(429, d, seed=1), rnd(5, d, seed=2), rnd(20, d, seed=3)
    out, _ = K.encoder_embed(texts, acc, wt, at, pos, B, T, d)
    close(out, (wt[texts] + at[acc] + pos[:T]).reshape(B * T, d), 1e-6)
    dout = rnd(B * T, d, seed=4)
    dwt = torch.zeros_like(wt)
    K.embedding_bwd(dout, texts, dwt, 0)
    ref = torch.zeros_like(wt).index_add_(0, texts.reshape(-1), dout)
    ref[0] = 0
    close(dwt, ref, 1e-5)
    spk = torch.tensor([3, 3, 7], device=DEV)
    st = rnd(9, d, seed=5)
    x = rnd(B * T, d, seed=6)
    close(K.rowvec_add(x, spk, st, B, T)[0], (x.view(B, T, d) + st[spk][:, None]).reshape(-1, d), 1e-6)
    dst = torch.zeros_like(st)
    K.rowvec_add_bwd(dout, spk, dst, B, T)
    close(dst, torch.zeros_like(st).index_add_(0, spk, dout.view(B, T, d).sum(1)), 1e-5)
    close(K.embedding_fwd(spk, st), st[spk], 0)
    m = K.length_mask(torch.tensor([3, 0, 11], device=DEV), 11)
    assert m.cpu().tolist() == (torch.arange(11)[None] >= torch.tensor([3, 0, 11])[:, None]).tolist()


@pytest.mark.parametrize("n,n_table", [(6144, 429), (5000, 5), (2049, 256), (6144, 1)])
def test_embedding_bwd_chunks(n, n_table):
    """The scatter-add of the embedding / bucket-embedding backward over several 1,024-row chunks,
    a ragged last chunk, table sizes that are not a multiple of the 8 ids a block lists, and a
    skewed id distribution (half the rows on one id): against a float64 index_add, padding row
    untouched, accumulation into the table, and bitwise repeatable."""
    g = torch.Generator(device="cpu").manual_seed(n + n_table)
    ids = torch.randint(0, n_table, (n,), generator=g)
    ids[::2] = min(7, n_table - 1)
    ids = ids.to(DEV)
    dout = rnd(n, 256, seed=11)
    base = rnd(n_table, 256, seed=12)
    ref = base.double().index_add(0, ids, dout.double())
    pad = 0 if n_table > 1 else -1
    if pad == 0:
        ref[0] = base[0].double()
    outs = []
    for _ in range(2):
        t = base.clone()
        K.embedding_bwd(dout, ids, t, pad)
        outs.append(t)
    close(outs[0], ref, 1e-5)
    assert torch.equal(outs[0], outs[1])
    t32 = base.clone()
    K.bucket_embed_bwd(dout, ids.to(torch.int32), t32)
    ref32 = base.double().index_add(0, ids, dout.double())
    close(t32, ref32, 1e-5)


def test_grad_norm_adam():
    n = 10_003
    g = rnd(n, seed=1)
    p = rnd(n, seed=2)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    nc = torch.empty(2, device=DEV)
    K.grad_norm(g, 1.0, nc)
    close(nc[0], g.norm(), 1e-6)
    big = rnd(4 * 1024 * 256 * 5 + 4 * 777 + 3, seed=3)  # several grid-stride trips + tail
    nc_big = torch.empty(2, device=DEV)
    K.grad_norm(big, 1.0, nc_big)
    close(nc_big[0], big.double().norm(), 1e-6)
    pr = p.clone().requires_grad_()
    opt = torch.optim.Adam([pr], lr=1e-3, betas=(0.9, 0.98), eps=1e-9)
    for t in range(1, 4):
        pr.grad = g.clone()
        torch.nn.utils.clip_grad_norm_([pr], 1.0)
        opt.step()
        K.adam_step(p, g, m, v, nc, 1e-3, 0.9, 0.98, 1e-9, 1 - 0.9 ** t, math.sqrt(1 - 0.98 ** t))
    close(p, pr.detach(), 1e-5)


# ------------------------------------------------------------------ bf16 path
def bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("B,T,cin,cout,k", [(2, 37, 256, 1024, 9), (3, 50, 1024, 256, 1),
                                            (2, 64, 80, 512, 5), (1, 33, 512, 80, 5),
                                            (4, 16, 256, 768, 1), (5, 130, 256, 256, 3),
                                            (48, 128, 256, 1024, 9), (3, 50, 256, 1, 1)])
def test_conv_gemm_bf16(B, T, cin, cout, k):
    """bf16 operands, fp32 accumulation: compare with fp32 math on the same bf16-rounded data."""
    pad = (k - 1) // 2
    x = bf(rnd(B * T, cin, seed=1))
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=2)).float()
    b = rnd(cout, seed=3)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    ref = ref_conv(x.float(), w, b, B, T, pad)
    y = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b)
    close(y, ref, 1e-5)
    yb = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b, flags=K.EPI_RELU,
                     out_dtype=torch.bfloat16)
    close(yb.float(), F.relu(ref), 8e-3)
    if cout % 8:
        return  # the transposed products need 8-channel multiples (ragged N only in forward)
    dy = bf(rnd(B * T, cout, seed=4))
    xr = x.float().clone().requires_grad_()
    wr = w.clone().requires_grad_()
    ref_conv(xr, wr, b, B, T, pad).backward(dy.float())
    aux = rnd(B * T, cin, seed=5)
    dx = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX, aux=aux)
    close(dx, xr.grad + aux, 1e-5)
    auxb = bf(rnd(B * T, cin, seed=6))
    dm = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, pad, flags=K.EPI_RELU_MASK_AUX, aux=auxb,
                     out_dtype=torch.bfloat16)
    close(dm.float(), xr.grad * (auxb.float() > 0), 8e-3)
    dw = torch.zeros_like(w)
    K.conv_wgrad(dy, x, dw, B * T, T, cin, cout, k, pad)
    close(dw, wr.grad, 1e-5)
    db = torch.zeros(cout, device=DEV)
    K.colsum(dy, B * T, cout, db)
    close(db, dy.float().sum(0), 1e-5)
    # fused bias gradient, accumulating into existing gradients
    dw2, db2 = torch.ones_like(w), torch.ones(cout, device=DEV)
    K.conv_wgrad(dy, x, dw2, B * T, T, cin, cout, k, pad, db=db2)
    close(dw2, wr.grad + 1, 1e-5)
    close(db2, dy.float().sum(0) + 1, 1e-5)


@pytest.mark.parametrize("B,T,cin,cout", [(48, 512, 256, 768), (48, 512, 256, 1024), (7, 130, 256, 256),
                                          (3, 50, 1024, 256)])
def test_conv_gemm_k1_bf16_epilogue(B, T, cin, cout):
    """The k = 1 GEMMs' bf16 whole-tile epilogue (bias / ReLU in the accumulator layout, ReLU
    mask on the bf16 row vectors) bitwise against the general epilogue of the tap-walking build
    (FS2_TUNE_NT_K1 = -1), with and without utterance lengths; aux values include zeros,
    negative zeros, infinities and NaN (a NaN aux masks, as NaN > 0 is false)."""
    x = bf(rnd(B * T, cin, seed=91))
    w = bf(rnd(cout, cin, scale=1 / math.sqrt(cin), seed=92))
    b = rnd(cout, seed=93)
    aux = bf(rnd(B * T, cout, seed=94))
    aux[::7, ::5] = 0.0
    aux[::11, ::3] = -0.0
    aux[5, :8] = float("inf")
    aux[6, :8] = float("-inf")
    aux[7, :8] = float("nan")
    lens = torch.tensor([max(1, T - 37 * i) for i in range(B)], device=DEV)
    res = {}
    try:
        for knob in (0, -1):
            K.lib.fs2_set_tuning(13, knob)  # FS2_TUNE_NT_K1
            res[knob] = [
                K.conv_gemm(x, w, B * T, T, cin, cout, 1, 0, bias=b, out_dtype=torch.bfloat16),
                K.conv_gemm(x, w, B * T, T, cin, cout, 1, 0, bias=b, flags=K.EPI_RELU,
                            out_dtype=torch.bfloat16, lens=lens),
                K.conv_gemm(x, w, B * T, T, cin, cout, 1, 0, out_dtype=torch.bfloat16),
                K.conv_gemm(x, w, B * T, T, cin, cout, 1, 0, flags=K.EPI_RELU_MASK_AUX, aux=aux,
                            out_dtype=torch.bfloat16),
                K.conv_gemm(x, w, B * T, T, cin, cout, 1, 0, flags=K.EPI_RELU_MASK_AUX, aux=aux,
                            out_dtype=torch.bfloat16, lens=lens)]
    finally:
        K.lib.fs2_set_tuning(13, 0)
    for i, (r0, r1) in enumerate(zip(res[0], res[-1])):
        assert torch.equal(r0, r1), i
    ref = (x.float() @ w.float().t() + b).to(torch.bfloat16)
    close(res[0][0].float(), ref.float(), 8e-3)


@pytest.mark.parametrize("knob", [0, 1, -1, 2])  # FS2_TUNE_ATTN: kernel variants (fs2hip.h)
@pytest.mark.parametrize("B,T,lens", [(2, 64, [64, 40]), (3, 130, [130, 77, 1]),
                                      (2, 512, [512, 300]), (3, 300, [300, 129, 64])])
def test_attention_bf16(B, T, lens, knob):
    K.lib.fs2_set_tuning(9, knob)
    try:
        _attention_bf16(B, T, lens)
    finally:
        K.lib.fs2_set_tuning(9, 0)


def _attention_bf16(B, T, lens):
    H, dh = 2, 128
    lens_t = torch.tensor(lens, device=DEV)
    qkv = bf(rnd(B * T, 3 * H * dh, seed=7))
    o, lse = K.attn_fwd(qkv, lens_t, B, T, H, dh, 1 / math.sqrt(dh))
    assert o.dtype == torch.bfloat16
    qr = qkv.float().clone().requires_grad_()
    ro = ref_attn(qr, lens_t, B, T, H, dh)
    valid = (torch.arange(T, device=DEV)[None, :] < lens_t[:, None]).reshape(-1)
    close(o.float()[valid], ro[valid], 1.5e-2)
    do = bf(rnd(B * T, H * dh, seed=8) * valid[:, None])
    ro.backward(do.float())
    dqkv = K.attn_bwd(qkv, o, do, lse, lens_t, B, T, H, dh, 1 / math.sqrt(dh))
    close(dqkv.float(), qr.grad, 3e-2)


@pytest.mark.parametrize("B,T,lens", [(3, 512, [512, 300, 1]), (3, 300, [300, 129, 64]),
                                      (2, 256, [256, 200])])
def test_attention_dma_vs_register_staged(B, T, lens):
    """The LDS-DMA staged attention kernels (FS2_TUNE_ATTN_DMA = 0 / 1: 2- / 3-slot forward
    ring; exp2 with the scale folded into one FMA, last-tile-only key masks, exact rescale skip)
    against the register-staged ones (-1) on the same inputs: outputs within one bf16 rounding,
    lse within fp32 rounding of the exponent argument, gradients within 2e-3 of their scale,
    padded gradient rows exactly zero in both (T = 300: a partial last tile, rows past T staged
    as zeros by the descriptor range)."""
    H, dh = 2, 128
    lens_t = torch.tensor(lens, device=DEV)
    qkv = bf(rnd(B * T, 3 * H * dh, seed=11))
    valid = (torch.arange(T, device=DEV)[None, :] < lens_t[:, None]).reshape(-1)
    do = bf(rnd(B * T, H * dh, seed=12) * valid[:, None])
    res = {}
    try:
        for knob in (-1, 0, 1):
            K.lib.fs2_set_tuning(14, knob)  # FS2_TUNE_ATTN_DMA
            o, lse = K.attn_fwd(qkv, lens_t, B, T, H, dh, 1 / math.sqrt(dh))
            dqkv = K.attn_bwd(qkv, o, do, lse, lens_t, B, T, H, dh, 1 / math.sqrt(dh))
            res[knob] = (o, lse, dqkv)
    finally:
        K.lib.fs2_set_tuning(14, 0)
    pad = ~valid
    for knob in (0, 1):
        o, lse, dqkv = res[knob]
        o0, lse0, dqkv0 = res[-1]
        close(o.float(), o0.float(), 8e-3)
        close(lse, lse0, 1e-5)
        close(dqkv.float(), dqkv0.float(), 2e-3)
        # padded rows of d_qkv are exact zeros (dQ of padded queries, dK / dV of padded keys)
        assert not dqkv[pad].any() and not dqkv0[pad].any(), knob


def test_norm_copies_bf16():
    M, d = 300, 256
    y, r = rnd(M, d, seed=1), rnd(M, d, seed=2)
    g, b = 1 + 0.1 * rnd(d, seed=3), 0.1 * rnd(d, seed=4)
    out, out_t, xh, rs, _ = K.ln_fwd(y, g, b, res=r, copy=torch.bfloat16)
    assert out_t.dtype == torch.bfloat16 and torch.equal(out_t, out.to(torch.bfloat16))
    dg, db = torch.zeros(d, device=DEV), torch.zeros(d, device=DEV)
    dy, dy_t = K.ln_bwd(xh, rs, g, b, dg, db, dout=rnd(M, d, seed=5), copy=torch.bfloat16)
    assert dy is None  # only the compute copy is produced
    dy32, _ = K.ln_bwd(xh, rs, g, b, dg.clone(), db.clone(), dout=rnd(M, d, seed=5))
    assert torch.equal(dy_t, dy32.to(torch.bfloat16))
    z = rnd(M, 512, seed=6)
    o2, o2_t, mean, rstd = K.bn_fwd(z, torch.ones(512, device=DEV), torch.zeros(512, device=DEV),
                                    None, None, True, 0.0, 0, 0, copy=torch.bfloat16)
    assert torch.equal(o2_t, o2.to(torch.bfloat16))
    x = rnd(M, d, seed=7)
    assert torch.equal(K.cast_bf16(x), x.to(torch.bfloat16))


@pytest.mark.parametrize("B,T,cin,cout", [(48, 512, 256, 768), (48, 512, 1024, 256),
                                          (48, 128, 256, 256), (3, 200, 256, 80), (5, 77, 72, 24),
                                          (1, 1000, 1024, 256)])
def test_wgrad_k1(B, T, cin, cout):
    """The k = 1 weight gradient (the grouped split-K kernel with one job: 128 x 128 tiles of 8
    waves, split slabs + one reduce; FS2_TUNE_WGRAD_K1 = -1: the tap-major kernel, also at a
    forced split count) with its fused bias gradient, accumulating into existing gradients,
    against fp32 math on the same bf16 data -- with and without utterance lengths (all-padding
    k-tiles skipped; dy is zero on padded rows as in the step)."""
    x = bf(rnd(B * T, cin, seed=31))
    lens = torch.tensor([T - (53 * u) % T for u in range(B)], device=DEV)
    lens[-1] = max(1, T // 7)
    valid = (torch.arange(T, device=DEV)[None] < lens[:, None]).reshape(-1)
    dy = bf(rnd(B * T, cout, seed=32) * valid[:, None])
    ref_w = dy.float().t() @ x.float()
    ref_b = dy.float().sum(0)
    try:
        for knob, splits, use_lens in ((0, 0, False), (0, 0, True), (-1, 0, True), (-1, 7, False)):
            K.lib.fs2_set_tuning(12, knob)  # FS2_TUNE_WGRAD_K1
            K.lib.fs2_set_tuning(3, splits)  # FS2_TUNE_WGRAD_SPLITS
            dw, db = torch.ones(cout, cin, device=DEV), torch.ones(cout, device=DEV)
            K.conv_wgrad(dy, x, dw, B * T, T, cin, cout, 1, 0, db=db,
                         lens=lens if use_lens else None)
            close(dw, ref_w + 1, 1e-5)
            close(db, ref_b + 1, 1e-5)
    finally:
        K.lib.fs2_set_tuning(12, 0)
        K.lib.fs2_set_tuning(3, 0)


@pytest.mark.parametrize("stages", [1, 2, 3, 4])
@pytest.mark.parametrize("B,T,cin,cout,k", [(2, 70, 256, 512, 9), (3, 50, 80, 256, 5),
                                            (1, 200, 512, 80, 5)])
def test_conv_gemm_bf16_pipeline_depths(stages, B, T, cin, cout, k):
    """Every LDS-stage count of the bf16 fwd/dX and weight-gradient kernels (the automatic
    choice uses 1 or 2) against fp32 math on the same bf16 data; knob reset afterwards."""
    pad = (k - 1) // 2
    x = bf(rnd(B * T, cin, seed=21))
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=22)).float()
    b = rnd(cout, seed=23)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    dy = bf(rnd(B * T, cout, seed=24))
    xr, wr = x.float().clone().requires_grad_(), w.clone().requires_grad_()
    ref = ref_conv(xr, wr, b, B, T, pad)
    ref.backward(dy.float())
    try:
        for knob in (0, 1):  # FS2_TUNE_GEMM_STAGES, FS2_TUNE_WGRAD_STAGES
            K.lib.fs2_set_tuning(knob, stages)
        for tile in (64, 128):
            K.lib.fs2_set_tuning(2, tile)  # FS2_TUNE_WGRAD_TILE
            y = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b)
            close(y, ref.detach(), 1e-5)
            dx = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, pad)
            close(dx, xr.grad, 1e-5)
            dw, db = torch.zeros_like(w), torch.zeros(cout, device=DEV)
            K.conv_wgrad(dy, x, dw, B * T, T, cin, cout, k, pad, db=db)
            close(dw, wr.grad, 1e-5)
            close(db, dy.float().sum(0), 1e-5)
    finally:
        for knob in (0, 1, 2):
            K.lib.fs2_set_tuning(knob, 0)


@pytest.mark.parametrize("B,T,lens,cin,p,tile", [
    (3, 50, [50, 17, 1], 256, 0.0, 0), (2, 200, [200, 130], 1024, 0.2, 0),
    (4, 128, [128, 70, 33, 128], 256, 0.2, 1), (6, 512, [512, 300, 129, 128, 1, 400], 1024, 0.1, 0),
    (5, 37, None, 256, 0.3, 1), (2, 64, [64, 9], 80, 0.1, 0)])
def test_conv_gemm_ln(B, T, lens, cin, p, tile):
    """fs2_conv_gemm_ln (GEMM + bias + dropout + residual + LayerNorm + row mask in one
    kernel) equals fs2_conv_gemm (fp32 y) -> fs2_ln_fwd bitwise: out, its bf16 copy, and
    xhat / rstd on the rows the backward reads; both row tiles (FS2_TUNE_LN_TILE)."""
    M, d = B * T, 256
    lt = None if lens is None else torch.tensor(lens, device=DEV)
    x = bf(rnd(M, cin, seed=51))
    w = bf(rnd(d, cin, 1, scale=1 / math.sqrt(cin), seed=52)).float()
    b, res = rnd(d, seed=53), rnd(M, d, seed=54)
    g, bt = 1 + 0.1 * rnd(d, seed=55), 0.1 * rnd(d, seed=56)
    wf = torch.empty(d * cin, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty_like(wf)
    K.weight_prep(w, d, cin, 1, wf, wb)
    kw = dict(lens=lt, seq_len=T, p_in=p, seed=99, site_in=5, copy=torch.bfloat16)
    y = K.conv_gemm(x, wf, M, T, cin, d, 1, 0, bias=b, lens=lt)
    o0, t0, xh0, rs0, _ = K.ln_fwd(y, g, bt, res=res, **kw)
    K.lib.fs2_set_tuning(11, tile)  # FS2_TUNE_LN_TILE
    try:
        o1, t1, xh1, rs1 = K.conv_gemm_ln(x, wf, M, T, cin, d, 1, 0, g, bt, bias=b, res=res,
                                          lens=lt, p_in=p, seed=99, site_in=5)
    finally:
        K.lib.fs2_set_tuning(11, 0)
    live = (torch.ones(M, dtype=torch.bool, device=DEV) if lt is None else
            (torch.arange(T, device=DEV)[None] < lt[:, None]).reshape(-1))
    assert torch.equal(o1, o0) and torch.equal(t1, t0)
    assert torch.equal(xh1[live], xh0[live]) and torch.equal(rs1[live], rs0[live])
    # and against fp32 math (no dropout: the reference's LayerNorm of the residual sum)
    if p == 0:
        ref = F.layer_norm(x.float() @ w.view(d, cin).t() + b + res, (d,), g, bt, 1e-5)
        close(o1[live], ref[live], 2e-5)
        assert torch.all(o1[~live] == 0)


@pytest.mark.parametrize("B,T,lens,cin,p,dres_add", [
    (3, 50, [50, 17, 1], 768, 0.0, False), (2, 200, [200, 130], 768, 0.2, False),
    (6, 512, [512, 300, 129, 128, 1, 400], 768, 0.1, True), (5, 37, None, 256, 0.3, False)])
def test_conv_gemm_ln_bwd(B, T, lens, cin, p, dres_add):
    """fs2_conv_gemm_ln_bwd (GEMM + residual-gradient add + LayerNorm backward in one kernel)
    against fs2_conv_gemm(FS2_EPI_ADD_AUX) -> fs2_ln_bwd.  The upstream gradient (acc + aux) is
    the same fp32 value in both; the row arithmetic is the same but compiled in another kernel
    (the compiler may contract a product into an FMA differently), so dres agrees to fp32
    rounding and its bf16 copy to one bf16 ulp; dgamma / dbeta / the fused bias gradient sum the
    same 32-row block partials in another in-block order."""
    M, d = B * T, 256
    lt = None if lens is None else torch.tensor(lens, device=DEV)
    x = bf(rnd(M, cin, seed=61))
    w = bf(rnd(d, cin, 1, scale=1 / math.sqrt(cin), seed=62)).float()
    wf = torch.empty(d * cin, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty_like(wf)
    K.weight_prep(w, d, cin, 1, wf, wb)
    aux = rnd(M, d, seed=63)
    # a LayerNorm forward state to differentiate
    y = rnd(M, d, seed=64)
    g, bt = 1 + 0.1 * rnd(d, seed=65), 0.1 * rnd(d, seed=66)
    _, _, xh, rs, _ = K.ln_fwd(y, g, bt, lens=lt, seq_len=T, p_in=p, seed=5, site_in=3)
    dout = K.conv_gemm(x, wf, M, T, cin, d, 1, 0, flags=K.EPI_ADD_AUX, aux=aux)
    grads = [torch.full((d,), 0.5, device=DEV) for _ in range(6)]
    dres0 = rnd(M, d, seed=67) if dres_add else torch.empty(M, d, device=DEV)
    dres1 = dres0.clone()
    _, dyt0 = K.ln_bwd(xh, rs, g, bt, grads[0], grads[1], dout=dout, lens=lt, seq_len=T, p_in=p,
                       seed=5, site_in=3, dres=dres0, dres_add=dres_add, copy=torch.bfloat16,
                       dbias_in=grads[2])
    dyt1, _ = K.conv_gemm_ln_bwd(x, wf, M, T, cin, d, 1, 0, xh, rs, g, grads[3], grads[4], aux=aux,
                                 lens=lt, p_in=p, seed=5, site_in=3, dres=dres1,
                                 dres_add=dres_add, dbias_in=grads[5])
    live = (torch.ones(M, dtype=torch.bool, device=DEV) if lt is None else
            (torch.arange(T, device=DEV)[None] < lt[:, None]).reshape(-1))
    a1, a0 = dyt1.float(), dyt0.float()
    assert bool(((a1 - a0).abs() <= a0.abs() * 2.0 ** -7).all()), "bf16 dy copies differ by > 1 ulp"
    close(dres1[live], dres0[live], 1e-6)
    assert torch.equal(dres1[~live], dres0[~live])
    for a_, b_ in zip(grads[3:], grads[:3]):
        close(a_, b_, 1e-5)


def test_conv_gemm_bf16_padding_tiles():
    """lens: all-padding 128-row tiles are written as zero rows (bias dropped) / aux, the
    rest exactly as without lens; the weight gradient with zero dy at padded rows is
    bitwise the same with and without skipping."""
    B, T, cin, cout, k = 6, 512, 256, 1024, 9
    lens = torch.tensor([512, 300, 129, 128, 1, 400], device=DEV)
    pad_rows = (torch.arange(T, device=DEV)[None] >= lens[:, None]).reshape(-1)
    x = bf(rnd(B * T, cin, seed=31)) * (~pad_rows)[:, None]
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=32)).float()
    b = rnd(cout, seed=33)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    y0 = K.conv_gemm(x, wf, B * T, T, cin, cout, k, 4, bias=b)
    y1 = K.conv_gemm(x, wf, B * T, T, cin, cout, k, 4, bias=b, lens=lens)
    tile_pad = pad_rows.view(-1, 128).all(1).repeat_interleave(128)
    assert tile_pad.sum() > 0
    assert torch.equal(y1[~tile_pad], y0[~tile_pad])
    assert torch.equal(y1[tile_pad], torch.zeros_like(y1[tile_pad]))
    aux = rnd(B * T, cin, seed=34)
    dy = bf(rnd(B * T, cout, seed=35)) * (~pad_rows)[:, None]
    d0 = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, 4, flags=K.EPI_ADD_AUX, aux=aux)
    d1 = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, 4, flags=K.EPI_ADD_AUX, aux=aux, lens=lens)
    assert torch.equal(d1[~tile_pad], d0[~tile_pad]) and torch.equal(d1[tile_pad], aux[tile_pad])
    # weight gradient: the split-K kernels (FS2_TUNE_WGRAD_HALO = 1, both tap-major tile widths)
    # skip all-padding k-tiles at no change (bitwise); the band kernel (default) deals the bands
    # that hold a real row over its waves in rank order, so skipping re-deals them: equal to
    # fp32 rounding
    for halo, tile in ((1, 64), (1, 128), (0, 0)):
        K.lib.fs2_set_tuning(7, halo)
        K.lib.fs2_set_tuning(2, tile)
        try:
            dw0, db0 = torch.zeros_like(w), torch.zeros(cout, device=DEV)
            dw1, db1 = torch.zeros_like(w), torch.zeros(cout, device=DEV)
            K.conv_wgrad(dy, x, dw0, B * T, T, cin, cout, k, 4, db=db0)
            K.conv_wgrad(dy, x, dw1, B * T, T, cin, cout, k, 4, db=db1, lens=lens)
        finally:
            K.lib.fs2_set_tuning(2, 0)
            K.lib.fs2_set_tuning(7, 0)
        if halo:
            assert torch.equal(dw0, dw1) and torch.equal(db0, db1)
        else:
            close(dw1, dw0, 1e-6)
            close(db1, db0, 1e-6)


@pytest.mark.parametrize("act,res", [(True, False), (False, True)])
def test_batchnorm_eval(act, res):
    """Eval-mode BatchNorm1d (running statistics, no update) vs F.batch_norm(training=False)."""
    M, c = 333, 80 if res else 512
    z = rnd(M, c, seed=11) * 2 - 0.5
    g, b = 1 + 0.1 * rnd(c, seed=12), 0.1 * rnd(c, seed=13)
    rm, rv = 0.2 * rnd(c, seed=14), 0.5 + rnd(c, seed=15).abs()
    rm0, rv0 = rm.clone(), rv.clone()
    r = rnd(M, c, seed=16) if res else None
    out, out_t = K.bn_eval_fwd(z, g, b, rm, rv, act, res=r, copy=torch.bfloat16)
    ref = F.batch_norm(z, rm.clone(), rv.clone(), g, b, training=False, eps=1e-5)
    if act:
        ref = torch.tanh(ref)
    if res:
        ref = ref + r
    close(out, ref, 2e-6)
    close(out_t.float(), ref, 1e-2)
    assert torch.equal(rm, rm0) and torch.equal(rv, rv0)


def test_duration_round_golden():
    """Inference durations (modules.py:132-135) bit-exact vs the reference (G2) and vs
    torch on random log-durations, incl. control scaling and the clamp."""
    g = load_golden("g2_round.npz")
    got = K.duration_round(torch.from_numpy(g["log_d"]).to(DEV))
    np.testing.assert_array_equal(got.cpu().numpy(), g["rounded"])
    x = rnd(4097, scale=1.5, seed=21)
    for c in (1.0, 1.3, 0.5):
        want = torch.clamp(torch.round(torch.exp(x) - 1) * c, min=0)
        got = K.duration_round(x, c)
        # exp may differ by an ulp between libraries; only exact .5 ties could flip
        assert (got != want).sum().item() <= 1


@pytest.mark.parametrize("B,T,cin,cout,k", [(48, 128, 256, 1024, 9), (6, 512, 1024, 256, 9),
                                            (4, 256, 512, 512, 5), (2, 64, 256, 256, 3),
                                            (3, 128, 512, 80, 5), (8, 64, 1024, 256, 9)])
def test_conv_gemm_bf16_halo(B, T, cin, cout, k):
    """The channel-block-major halo kernel (Conv1d taps > 1, T a tile multiple) against fp32
    math on the same bf16 data and against the tap-major kernel, at every tile width
    (auto, forced 128-wide), with and without utterance lengths (padding skipped)."""
    pad = (k - 1) // 2
    x = bf(rnd(B * T, cin, seed=41))
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=42)).float()
    b = rnd(cout, seed=43)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    ref = ref_conv(x.float(), w, b, B, T, pad)
    lens = torch.tensor([T - (7 * u) % T for u in range(B)], device=DEV)
    lens[-1] = 1
    try:
        K.lib.fs2_set_tuning(15, -1)  # FS2_TUNE_TAPREG off: these are the halo kernels' checks
        K.lib.fs2_set_tuning(6, -1)  # FS2_TUNE_NT_HALO off: tap-major kernel
        y_tm = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b)
        for mode in (0, 1, 2):  # 0: the 8-wave (one block per CU) tiles where eligible
            K.lib.fs2_set_tuning(6, mode)
            y = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b)
            close(y, ref, 1e-5)
            close(y, y_tm, 1e-5)
            # with lens, input rows past each utterance's length are taken as zero (they are
            # zero in the step: Layers.py:25,28 / zero upstream gradients) and all-padding
            # tiles / half tiles are not computed: the valid rows equal the conv of the
            # masked input
            valid = (torch.arange(T, device=DEV)[None] < lens[:, None]).reshape(-1)
            yl = K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b, lens=lens)
            ref_l = ref_conv(x.float() * valid[:, None], w, b, B, T, pad)
            close(yl[valid], ref_l[valid], 1e-5)
            assert torch.isfinite(yl).all()
            if cout % 8 == 0:
                dy = bf(rnd(B * T, cout, seed=44))
                xr, wr = x.float().clone().requires_grad_(), w.clone().requires_grad_()
                ref_conv(xr, wr, b, B, T, pad).backward(dy.float())
                aux = rnd(B * T, cin, seed=45)
                dx = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX, aux=aux)
                close(dx, xr.grad + aux, 1e-5)
                dxl = K.conv_gemm(dy, wb, B * T, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX,
                                  aux=aux, lens=lens)
                assert torch.isfinite(dxl).all()
    finally:
        K.lib.fs2_set_tuning(6, 0)
        K.lib.fs2_set_tuning(15, 0)


@pytest.mark.parametrize("mode", [0, 1, 3])
def test_conv_gemm_bf16_tapreg_ragged_rows(mode):
    """A row count that is not a whole number of utterances (here not a multiple of the 128-row
    tile either): the tap-register kernel is not eligible (rows % seq_len, rows % 128) and the
    launch falls back to a kernel that computes every row -- rows past the matrix read as zero,
    as in a reference whose input is zero there."""
    B, T, cin, cout, k = 4, 512, 256, 1024, 9
    M = B * T - 96
    pad = (k - 1) // 2
    xf = bf(rnd(B * T, cin, seed=81))
    xf[M:] = 0
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=82)).float()
    b = rnd(cout, seed=83)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    K.lib.fs2_set_tuning(15, mode)  # FS2_TUNE_TAPREG
    try:
        y = K.conv_gemm(xf[:M].contiguous(), wf, M, T, cin, cout, k, pad, bias=b, flags=K.EPI_RELU)
    finally:
        K.lib.fs2_set_tuning(15, 0)
    ref = F.relu(ref_conv(xf.float(), w, b, B, T, pad))[:M]
    assert y.shape == (M, cout) and torch.isfinite(y).all()
    close(y, ref, 1e-5)


@pytest.mark.parametrize("B,T,cin,cout,k,mode", [
    (4, 512, 256, 1024, 9, 0), (4, 512, 256, 1024, 9, 1), (6, 512, 1024, 256, 9, 1),
    (2, 256, 512, 512, 5, 3), (3, 128, 512, 512, 5, 1), (3, 128, 256, 320, 9, 1),
    (2, 256, 256, 200, 9, 3), (6, 512, 1024, 256, 9, 0), (4, 512, 256, 1024, 9, 3),
    (3, 128, 512, 512, 5, 3)])
def test_conv_gemm_bf16_tapreg(B, T, cin, cout, k, mode):
    """The tap-register halo kernel (FS2_TUNE_TAPREG = 0: automatic, 1: 4-wave 128 x 64 tiles,
    3: 4-wave 128 x 128 tiles at two blocks per CU) against fp32 math
    on the same bf16 data, forward (bias + ReLU) and data
    gradient (+ residual), and bitwise against the halo kernels (knob -1): the same MFMAs per
    output in the same (channel block, tap, k-half) order.  With lens only the valid rows are
    compared: a wave whose 64-row band lies past the length computes nothing (epilogue of 0),
    the halo kernel skips at 16-row granularity."""
    pad = (k - 1) // 2
    x = bf(rnd(B * T, cin, seed=61))
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=62)).float()
    b = rnd(cout, seed=63)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    lens = torch.tensor([T - (11 * u) % T for u in range(B)], device=DEV)
    lens[-1] = 1
    valid = (torch.arange(T, device=DEV)[None] < lens[:, None]).reshape(-1)
    dy = bf(rnd(B * T, cout, seed=64))
    aux = rnd(B * T, cin, seed=65)
    M = B * T

    def run(v):
        K.lib.fs2_set_tuning(15, v)
        K.lib.fs2_set_tuning(8, -1)  # halo reference unsplit (a split sums in another order)
        try:
            return (K.conv_gemm(x, wf, M, T, cin, cout, k, pad, bias=b, flags=K.EPI_RELU),
                    K.conv_gemm(x, wf, M, T, cin, cout, k, pad, bias=b, flags=K.EPI_RELU,
                                out_dtype=torch.bfloat16, lens=lens),
                    K.conv_gemm(dy, wb, M, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX, aux=aux),
                    K.conv_gemm(dy, wb, M, T, cout, cin, k, pad, flags=K.EPI_ADD_AUX, aux=aux,
                                lens=lens))
        finally:
            K.lib.fs2_set_tuning(15, 0)
            K.lib.fs2_set_tuning(8, 0)
    t, h = run(mode), run(-1)
    close(t[0], F.relu(ref_conv(x.float(), w, b, B, T, pad)), 1e-5)
    xm = x.float() * valid[:, None]
    close(t[1].float()[valid], F.relu(ref_conv(xm, w, b, B, T, pad))[valid], 8e-3)
    xr = x.float().clone().requires_grad_()
    ref_conv(xr, w, b, B, T, pad).backward(dy.float())
    close(t[2], xr.grad + aux, 1e-5)
    if cout % 64 == 0:  # the data gradient runs on the halo kernels (zero rows past the length)
        xr2 = xm.clone().requires_grad_()
        ref_conv(xr2, w, b, B, T, pad).backward(dy.float() * valid[:, None])
        close(t[3][valid], (xr2.grad + aux)[valid], 1e-5)
    for a_, b_ in zip(t, h):
        assert torch.isfinite(a_.float()).all()
    assert torch.equal(t[0], h[0]) and torch.equal(t[2], h[2])
    assert torch.equal(t[1][valid], h[1][valid]) and torch.equal(t[3][valid], h[3][valid])


@pytest.mark.parametrize("B,T,cin,cout,k,flags", [
    (48, 128, 1024, 256, 9, "add_aux"), (48, 128, 1024, 256, 9, "bias_relu_bf16"),
    (8, 64, 512, 256, 5, "relu_mask_bf16")])
def test_conv_gemm_bf16_halo_splitk(B, T, cin, cout, k, flags):
    """Split-K 64x64 halo launch (channel blocks split over the grid, fp32 partials summed by
    halo_splitk_reduce) against the unsplit launch (FS2_TUNE_HALO_SPLITK = -1) on the encoder
    data-gradient shape, with lens: the epilogue (bias only on computed tiles, aux add, ReLU /
    ReLU mask, bf16 cast) must match on the valid rows; sums differ only by the split's
    rounding.  Padded rows are compared only when the tiling is the same: a 128-row tile that
    holds a valid frame computes padded rows a skipped 64-row tile leaves at the epilogue of 0."""
    pad = (k - 1) // 2
    x = bf(rnd(B * T, cin, seed=51))
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=52)).float()
    b = rnd(cout, seed=53)
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    wb = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, wb)
    lens = torch.tensor([T - (5 * u) % T for u in range(B)], device=DEV)
    lens[-1] = 1
    aux = rnd(B * T, cout, seed=54)

    def run():
        if flags == "add_aux":
            return K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, flags=K.EPI_ADD_AUX, aux=aux,
                               lens=lens)
        if flags == "bias_relu_bf16":
            return K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, bias=b, flags=K.EPI_RELU,
                               out_dtype=torch.bfloat16, lens=lens)
        return K.conv_gemm(x, wf, B * T, T, cin, cout, k, pad, flags=K.EPI_RELU_MASK_AUX,
                           aux=bf(aux), out_dtype=torch.bfloat16, lens=lens)
    valid = (torch.arange(T, device=DEV)[None] < lens[:, None]).reshape(-1)
    try:
        K.lib.fs2_set_tuning(8, -1)
        want = run().float()
        for kz in (0, 2, 4, -2):  # -2: 64x64 tiles only
            K.lib.fs2_set_tuning(8, kz)
            got = run().float()
            tol = 1e-5 if flags == "add_aux" else 8e-3
            close(got[valid], want[valid], tol)
            if kz == -2:  # same 64-row tiling as the unsplit launch: padded rows too
                close(got, want, tol)
    finally:
        K.lib.fs2_set_tuning(8, 0)


def test_conv_gemm_bf16_halo_splitk_streams():
    """The split-K launches share one partials buffer: a launch on another stream is ordered
    behind the previous user's reduce on the device (an event of the library's), and the split
    decomposition -- hence the fp32 summation order -- does not depend on which streams ran
    before or whether they still exist: the default-stream result is bitwise the same before
    and after split launches on other, since released, streams."""
    B, T, cin, cout, k = 48, 128, 1024, 256, 9
    x = bf(rnd(B * T, cin, seed=61))
    w = bf(rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=62)).float()
    wf = torch.empty(cout * cin * k, device=DEV, dtype=torch.bfloat16)
    K.weight_prep(w, cout, cin, k, wf, None)
    run = lambda: K.conv_gemm(x, wf, B * T, T, cin, cout, k, 4)
    want = run()
    for _ in range(3):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            other = run()
        s.synchronize()
        assert torch.equal(other, want)
        del s
        assert torch.equal(run(), want)
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,c", [(333, 8), (97, 24), (65, 4096), (32, 512), (2, 80)])
def test_batchnorm_widths(M, c):
    """BatchNorm forward/backward at the edges of the backward partials' lane layout (c / 8
    column lanes x up to 32 row lanes of a 32-row block: one column group, a non-power-of-two
    count, 512 groups with one row lane, exactly one block, two rows) against autograd."""
    z = rnd(M, c, seed=21) * 2 + 0.3
    g, b = 1 + 0.1 * rnd(c, seed=22), 0.1 * rnd(c, seed=23)
    out, _, mean, rstd = K.bn_fwd(z, g, b, None, None, True, 0.0, 1, 2)
    zr, gr, br = z.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    ref = torch.tanh(F.batch_norm(zr, None, None, gr, br, training=True, eps=1e-5))
    close(out, ref, 2e-5)
    dout = rnd(M, c, seed=24)
    ref.backward(dout)
    dg, db = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)
    dz, _ = K.bn_bwd(dout, z, mean, rstd, g, b, dg, db, True, 0.0, 1, 2)
    close(dz, zr.grad)
    close(dg, gr.grad)
    close(db, br.grad)


def test_batchnorm_tanh_relative_near_zero():
    """The PostNet's tanh (BatchNorm epilogue) in RELATIVE terms near 0, where an absolute
    error of ~3e-7 would be a large relative one: gamma spreads the normalised values over
    |y| in [1e-9, 2] on a log scale, against torch.tanh of the same fp32 pre-activation."""
    M, c = 4096, 64
    z = rnd(M, c, seed=31)
    g = torch.logspace(-9, 0.3, c, device=DEV)
    b = torch.zeros(c, device=DEV)
    out, _, mean, rstd = K.bn_fwd(z, g, b, None, None, True, 0.0, 1, 2)
    y = (z - mean) * rstd * g  # the kernel's own statistics: only the tanh is under test
    ref = torch.tanh(y.double())
    rel = ((out.double() - ref).abs() / ref.abs().clamp_min(1e-30))
    big = y.abs() >= 1e-12  # below that the pre-activation itself is at fp32's denormal edge
    assert rel[big].max().item() <= 5e-6, f"max relative error {rel[big].max().item():.3e}"


@pytest.mark.parametrize("c,act", [(512, True), (80, False)])
def test_batchnorm_dropout(c, act):
    """PostNet BatchNorm with dropout (p = 0.5): keep-rate of the 16-bit Philox draws, and the
    backward against autograd on the mask recovered from the forward output."""
    M, p = 1000, 0.5
    z = rnd(M, c, seed=11) * 2 + 0.5
    g, b = 1 + 0.1 * rnd(c, seed=12), 0.1 * rnd(c, seed=13)
    out, _, mean, rstd = K.bn_fwd(z, g, b, None, None, act, p, 7, 3)
    keep = out != 0
    frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01, frac
    zr, gr, br = z.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    ref = F.batch_norm(zr, None, None, gr, br, training=True, eps=1e-5)
    if act:
        ref = torch.tanh(ref)
    ref = ref * keep / (1 - p)
    close(out, ref, 2e-5)
    dout = rnd(M, c, seed=14)
    ref.backward(dout)
    dg, db = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)
    dz, _ = K.bn_bwd(dout, z, mean, rstd, g, b, dg, db, act, p, 7, 3)
    close(dz, zr.grad)
    close(dg, gr.grad)
    close(db, br.grad)


@pytest.mark.parametrize("B,T,C,k,d", [(2, 192, 256, 3, 5), (2, 192, 256, 7, 3),
                                       (1, 300, 256, 11, 5), (2, 128, 64, 11, 5),
                                       (3, 100, 32, 7, 5),
                                       # 64 x odd rows per utterance (the vocoder's 64-rows-
                                       # per-frame stage): 64-row halo tiles, wide grid
                                       (2, 64 * 513, 128, 11, 5), (3, 64 * 91, 128, 7, 3)])
def test_conv_gemm_ex_dilated_epilogues(B, T, C, k, d):
    """fs2_conv_gemm_ex (vocoder convs): dilated taps on the halo and tap-major kernels (bf16)
    and the fp32 kernel, with the LRELU / ADD_AUX / ACC_Y / Y2 epilogue, against torch."""
    pad = d * (k - 1) // 2
    xs = rnd(B * T, C, seed=51)
    w = bf(rnd(C, C, k, scale=1 / math.sqrt(C * k), seed=52)).float()
    b = rnd(C, seed=53) * 0.1
    aux, y_old = rnd(B * T, C, seed=54), rnd(B * T, C, seed=55)
    conv = F.conv1d(bf(xs).float().view(B, T, C).transpose(1, 2), w, b, padding=pad,
                    dilation=d).transpose(1, 2).reshape(B * T, C)
    v = (conv + aux + y_old) * (1 / 3)
    want_y = torch.where(v >= 0, v, 0.1 * v)
    want_y2 = torch.where(want_y >= 0, want_y, 0.01 * want_y)
    flags = K.EPI_LRELU | K.EPI_ADD_AUX | K.EPI_ACC_Y
    for dt, tol in ((torch.bfloat16, 1e-5), (torch.float32, 1e-5)):
        x = bf(xs) if dt == torch.bfloat16 else bf(xs).float()
        wf = torch.empty(C * C * k, dtype=dt, device=DEV)
        K.weight_prep(w, C, C, k, w_fwd=wf)
        for mode in ((0, -1) if dt == torch.bfloat16 else (0,)):
            K.lib.fs2_set_tuning(6, mode)
            try:
                y = y_old.clone()
                y2 = torch.empty(B * T, C, dtype=dt, device=DEV)
                K.conv_gemm_ex(x, wf, B * T, T, C, C, k, pad, dilation=d, bias=b, flags=flags,
                               aux=aux, out=y, y2=y2, alpha=0.1, scale=1 / 3, alpha2=0.01)
            finally:
                K.lib.fs2_set_tuning(6, 0)
            close(y, want_y, tol)
            close(y2.float(), want_y2, 8e-3 if dt == torch.bfloat16 else tol)


def test_convT_as_phase_conv():
    """ConvTranspose1d(k = 2s, stride s, pad s/2) == the 3-tap phase conv of
    fs2_convT_weight_prep, whose (rows, s*c_out) output is the (rows*s, c_out) signal."""
    for s, cin, cout, B, T in ((8, 128, 64, 2, 20), (2, 64, 32, 3, 33)):
        w = rnd(cin, cout, 2 * s, scale=0.1, seed=61)
        b = rnd(cout, seed=62)
        x = rnd(B * T, cin, seed=63)
        want = F.conv_transpose1d(x.view(B, T, cin).transpose(1, 2), w, b, stride=s,
                                  padding=s // 2).transpose(1, 2).reshape(B * T * s, cout)
        wc, bc = K.convT_weight_prep(w, b, s)
        wf = torch.empty(s * cout * cin * 3, dtype=torch.float32, device=DEV)
        K.weight_prep(wc, s * cout, cin, 3, w_fwd=wf)
        y = torch.empty(B * T * s, cout, device=DEV)
        K.conv_gemm_ex(x, wf, B * T, T, cin, s * cout, 3, 1, bias=bc, out=y.view(B * T, s * cout))
        close(y, want, 1e-5)


@pytest.mark.parametrize("B,T,cin,cout,k", [(6, 512, 256, 1024, 9), (4, 128, 256, 256, 3),
                                            (3, 256, 512, 512, 5), (48, 128, 256, 1024, 9),
                                            (2, 64, 1024, 256, 9), (3, 64, 200, 1024, 9),
                                            (2, 128, 256, 1000, 5), (3, 128, 256, 1024, 3),
                                            (2, 128, 80, 512, 5), (2, 128, 512, 80, 5)])
def test_conv_wgrad_halo(B, T, cin, cout, k):
    """The Conv1d (taps 3/5/9) weight gradient with its fused bias gradient against fp32
    autograd on the same bf16 data, every kernel: (FS2_TUNE_WGRAD_HALO, FS2_TUNE_WGRAD_WIDE)
    (0, 0) = the default choice, (0, 1) = the wide-tile kernel wherever eligible (64 x 64 x taps
    tiles, row splits + in-order reduce; T % 64 == 0), (0, -1) = the slab-free band kernel where
    its 32 x 32 tiles fill the chip (else the split-K halo kernel), (0, 3) = the wide kernel with
    3 forced splits, (1, 0) = the split-K
    halo kernel (C_in % 64 == 0, else tap-major), (-1, 0) = the tap-major kernel.  Partial
    o / c tiles, determinism, accumulation into dw, and the padding-band skip under lens."""
    pad = (k - 1) // 2
    x = bf(rnd(B * T, cin, seed=71))
    dy = bf(rnd(B * T, cout, seed=72))
    w = rnd(cout, cin, k, scale=1 / math.sqrt(cin * k), seed=73)
    xr, wr = x.float().clone().requires_grad_(), w.clone().requires_grad_()
    ref_conv(xr, wr, None, B, T, pad).backward(dy.float())
    out = {}
    try:
        for mode in ((0, 0), (0, 1), (0, -1), (0, 3), (1, 0), (-1, 0)):
            K.lib.fs2_set_tuning(7, mode[0])  # FS2_TUNE_WGRAD_HALO
            K.lib.fs2_set_tuning(19, mode[1])  # FS2_TUNE_WGRAD_WIDE
            dw, db = torch.zeros_like(w), torch.zeros(cout, device=DEV)
            K.conv_wgrad(dy, x, dw, B * T, T, cin, cout, k, pad, db=db)
            out[mode] = (dw, db)
            close(dw, wr.grad, 1e-5)
            close(db, dy.float().sum(0), 1e-5)
    finally:
        K.lib.fs2_set_tuning(7, 0)
        K.lib.fs2_set_tuning(19, 0)
    # fixed reduction order: a second run is bitwise equal; dw / db accumulate
    dw2, db2 = out[(0, 0)][0].clone(), out[(0, 0)][1].clone()
    K.conv_wgrad(dy, x, dw2, B * T, T, cin, cout, k, pad, db=db2)
    dw3, db3 = torch.zeros_like(w), torch.zeros(cout, device=DEV)
    K.conv_wgrad(dy, x, dw3, B * T, T, cin, cout, k, pad, db=db3)
    assert torch.equal(dw3, out[(0, 0)][0]) and torch.equal(db3, out[(0, 0)][1])
    close(dw2, 2 * wr.grad, 1e-5)
    close(db2, 2 * dy.float().sum(0), 1e-5)
    # lens: zero dy rows past each length; the all-padding bands / k-tiles are skipped.  That
    # changes which split / wave sums which rows, so the result equals the lens-free one to fp32
    # rounding, not bitwise (reproducible per lens: fs2hip.h)
    lens = torch.tensor([T - (13 * u) % T for u in range(B)], device=DEV)
    padr = (torch.arange(T, device=DEV)[None] >= lens[:, None]).reshape(-1)
    dyz = dy * (~padr)[:, None]
    dw0, db0 = torch.zeros_like(w), torch.zeros(cout, device=DEV)
    dw1, db1 = torch.zeros_like(w), torch.zeros(cout, device=DEV)
    K.conv_wgrad(dyz, x, dw0, B * T, T, cin, cout, k, pad, db=db0)
    K.conv_wgrad(dyz, x, dw1, B * T, T, cin, cout, k, pad, db=db1, lens=lens)
    close(dw1, dw0, 1e-6)
    close(db1, db0, 1e-6)


@pytest.mark.parametrize("B,T,lens_on", [(48, 512, True), (48, 128, False), (3, 64, True),
                                         (2, 128, False)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_wgrad_k1_multi(B, T, lens_on, dt):
    """The grouped k = 1 weight gradient (the FFT block's QKV + bias, fc and w_2 products in one
    launch: wgrad_k1_multi + one split reduce) against fp32 references on the same data, with
    accumulation into dw / db, a partial 128-wide tile (80 outputs), determinism, and the
    padding k-tile skip under lens."""
    M = B * T
    shapes = [(256, 768, True), (256, 256, False), (1024, 256, False), (256, 80, True)]
    lens = None
    valid = torch.ones(M, dtype=torch.bool, device=DEV)
    if lens_on:
        lens = torch.tensor([T - (37 * u) % T for u in range(B)], device=DEV)
        valid = (torch.arange(T, device=DEV)[None] < lens[:, None]).reshape(-1)
    jobs, refs = [], []
    for i, (cin, cout, bias) in enumerate(shapes):
        x = rnd(M, cin, seed=90 + i).to(dt)
        dy = (rnd(M, cout, seed=95 + i) * valid[:, None]).to(dt)
        dw = rnd(cout, cin, scale=0.1, seed=99 + i)
        db = rnd(cout, scale=0.1, seed=103 + i) if bias else None
        refs.append((dw + dy.float().t() @ x.float(), None if db is None else db + dy.float().sum(0)))
        jobs.append((dy, x, dw, db, cin, cout))
    snap = [(j[2].clone(), None if j[3] is None else j[3].clone()) for j in jobs]
    K.conv_wgrad_k1_multi(jobs, M, T, lens=lens)
    tol = 1e-5 if dt == torch.bfloat16 else 1e-4
    for (dy, x, dw, db, cin, cout), (rw, rb) in zip(jobs, refs):
        close(dw, rw, tol)
        if db is not None:
            close(db, rb, tol)
    # a second run from the same starting point is bitwise equal
    first = [(j[2].clone(), None if j[3] is None else j[3].clone()) for j in jobs]
    for j, (w0, b0) in zip(jobs, snap):
        j[2].copy_(w0)
        if j[3] is not None:
            j[3].copy_(b0)
    K.conv_wgrad_k1_multi(jobs, M, T, lens=lens)
    for j, (w1, b1) in zip(jobs, first):
        assert torch.equal(j[2], w1)
        if j[3] is not None:
            assert torch.equal(j[3], b1)


@pytest.mark.gpu
def test_lds_dma_out_of_range_lanes_land_zeros():
    """The padding-row contract of every LDS-DMA kernel (conv_wgrad_band, the halo / tap-register
    GEMMs, attention): a buffer LDS-DMA at an out-of-range offset writes zeros into LDS rather
    than leaving what was there (the LDS is pre-filled with 0xAB bytes, lanes 32-63 out of
    range).  If it left the old bytes, padded rows would carry whatever the CU's previous kernel
    left in LDS -- a result that depends on process history."""
    src = torch.arange(64 * 4, dtype=torch.float32, device=DEV) + 1.0
    out = torch.empty(64 * 4, dtype=torch.int32, device=DEV)
    K.lib.fs2_debug_lds_dma_oob(src.data_ptr(), out.data_ptr(), K.stream())
    got = out.cpu()
    assert torch.equal(got[:128], src[:128].cpu().view(torch.int32))
    assert int((got[128:] != 0).sum()) == 0, got[128:].tolist()[:8]
