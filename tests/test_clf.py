"""The --use_clf language discriminator against the reference's own
outputs (g10): the GE2E SpeechEmbedder + GE2ELoss BCE on seeded weights, and two full
use_clf training steps at SYN-3x48 (fp32, dropout off, fixed speaker shuffle)."""
import importlib

import numpy as np
import pytest
import torch

from conftest import load_golden

PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
G = importlib.import_module("mid-attribute-speaker-generation_amd.ge2e")


def _keys(g):
    return {k: tuple(int(x) for x in s.split(",")) for k, s in zip(g["disc.keys"], g["disc.shapes"])}


def test_discriminator_state_dict_matches_reference():
    g = load_golden("g10_clf.npz")
    d = G.SpeechEmbedder(device="meta")
    assert {k: tuple(v.shape) for k, v in d.state_dict().items()} == _keys(g)


def test_da_coefficient_and_chunk_count():
    assert G.da_coefficient(0, 10) == 0.0
    assert abs(G.da_coefficient(4, 10) - (2 / (1 + np.exp(-4.0)) - 1)) < 1e-12
    # train.py:180: T // 150 + 1 chunks (a full zero chunk when T is a multiple of 150)
    assert [t // 150 + 1 for t in (149, 150, 151, 300)] == [1, 2, 2, 3]


def _disc(dev="cuda"):
    d = G.SpeechEmbedder(device=dev)
    PKG.seeded.load_seeded_(d)
    d.da_dropout = 0.0  # the fixtures ran with dropout patched off
    return d


@pytest.mark.gpu
def test_discriminator_matches_reference():
    g = load_golden("g10_clf.npz")
    d, dl = _disc(), G.GE2ELoss("cuda")
    x = torch.from_numpy(g["d.x"]).cuda().requires_grad_()
    langs = torch.from_numpy(g["d.langs"]).cuda()
    out = d(x)
    tot, ge2e, da = dl(out["embeddings"].view(6, 1, -1), out["da_lang_logits"], langs,
                       reduction="sum")
    assert torch.isnan(ge2e) and torch.isnan(tot)  # M = 1: exclude-self centroid / 0
    np.testing.assert_allclose(out["embeddings"].detach().cpu().numpy(), g["d.emb"], atol=2e-5)
    np.testing.assert_allclose(out["da_lang_logits"].detach().cpu().numpy(), g["d.logits"],
                               rtol=1e-4, atol=1e-5)
    assert abs(da.item() - float(g["d.da"])) <= 1e-4 * abs(float(g["d.da"]))
    (da * 0.37).backward()
    dx, ref = x.grad.cpu().numpy(), g["d.dx"]
    assert np.abs(dx - ref).max() <= 1e-4 * np.abs(ref).max()
    # only the last frame of each sequence reaches the classifier: a zero-padded tail still
    # back-propagates through the recurrence
    assert np.abs(dx[4:, 100:]).max() > 0


@pytest.mark.gpu
def test_discriminator_dropout_keeps_forward_backward_consistent():
    """Classifier dropout (p = 0.2, train mode): the backward regenerates the forward's
    masks -- the input gradient matches a finite difference of the same call's key."""
    d = G.SpeechEmbedder(device="cuda")
    PKG.seeded.load_seeded_(d)
    g = load_golden("g10_clf.npz")
    x = torch.from_numpy(g["d.x"]).cuda().requires_grad_()
    out = d(x)
    assert d.da_dropout == 0.2
    out["da_lang_logits"].sum().backward()
    assert torch.isfinite(x.grad).all() and x.grad.abs().max() > 0


@pytest.mark.gpu
def test_use_clf_training_steps_match_reference():
    g = load_golden("g10_clf.npz")
    M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
    TR = importlib.import_module("mid-attribute-speaker-generation_amd.train")
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device="cuda", compute_dtype=torch.float32)
    PKG.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    tr = TR.Trainer(model, pp, mc, tc)
    clf = (_disc(), G.GE2ELoss("cuda"))
    batch = PKG.data.to_device(PKG.data.syn_batch(3, 48, seed=3), "cuda")
    perm = [int(i) for i in g["perm"]]
    for it, step in enumerate((4, 5)):
        out = TR.train_step(model, tr.opt, tr.Loss, tr.eLoss, batch, tr.clip, clf=clf,
                            clf_args=(perm, step, 10, 1.0))
        losses, eloss, gnorm, _, (dloss, cross, n_chunks) = out
        assert n_chunks == 3 * int(g[f"s{it}.max_len_r"])
        got = np.array([float(l) for l in losses] + [float(eloss), float(dloss), float(gnorm)])
        want = np.concatenate([g[f"s{it}.losses"],
                               [g[f"s{it}.eloss"], g[f"s{it}.dloss"], g[f"s{it}.gnorm"]]])
        err = np.abs(got - want) / np.maximum(np.abs(want), 1e-6)
        assert err.max() < 1e-4, (it, got, want)


@pytest.mark.gpu
def test_lstm_layer_matches_torch_lstm():
    """One LSTM layer through the C-ABI (f32 MFMA recurrence, split-K step kernels) against
    torch.nn.LSTM in fp32: ragged sequence count (37: partial 16-sequence tiles), c_in 80,
    outputs h within 2e-5 and the input gradient within 1e-4 of its peak."""
    K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
    lib = importlib.import_module("mid-attribute-speaker-generation_amd._lib").lib
    N, T, H, D = 37, 23, 256, 80
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(N * T, D, generator=gen).cuda()
    w_ih = (torch.randn(4 * H, D, generator=gen) * 0.1).cuda()
    w_hh = (torch.randn(4 * H, H, generator=gen) * 0.1).cuda()
    b = (torch.randn(4 * H, generator=gen) * 0.1).cuda()
    dh = (torch.randn(N * T, H, generator=gen) * 0.1).cuda()
    gx, act, dg = (torch.empty(N * T, 4 * H, device="cuda") for _ in range(3))
    h, c = torch.empty(N * T, H, device="cuda"), torch.empty(N * T, H, device="cuda")
    dc, dx = torch.empty(2 * N * H, device="cuda"), torch.empty(N * T, D, device="cuda")
    P = lambda t: t.data_ptr()
    assert lib.fs2_lstm_layer_fwd(P(x), N, T, D, H, P(w_ih), P(b), P(w_hh), P(gx), P(h), P(c),
                                  P(act), K.stream()) == 0
    w_ih_t, w_hh_t = w_ih.t().contiguous(), w_hh.t().contiguous()
    assert lib.fs2_lstm_layer_bwd(P(dh), N, T, D, H, P(w_ih_t), P(w_hh_t), P(act), P(c), P(dg),
                                  P(dc), P(dx), K.stream()) == 0
    torch.cuda.synchronize()
    ref = torch.nn.LSTM(D, H, batch_first=True).cuda()
    with torch.no_grad():
        ref.weight_ih_l0.copy_(w_ih)
        ref.weight_hh_l0.copy_(w_hh)
        ref.bias_ih_l0.copy_(b)
        ref.bias_hh_l0.zero_()
    xr = x.view(N, T, D).clone().requires_grad_()
    out, _ = ref(xr)
    out.backward(dh.view(N, T, H))
    assert (h.view(N, T, H) - out.detach()).abs().max().item() < 2e-5
    assert (dx.view(N, T, D) - xr.grad).abs().max().item() < 1e-4 * xr.grad.abs().max().item()


@pytest.mark.gpu
def test_lstm_stack_wavefront_matches_torch_lstm():
    """The 3-layer stack as one wavefront (fs2_lstm_stack_fwd/bwd: launch s runs layer l at
    step s - l, inter-layer products inside the step kernels) against torch.nn.LSTM(
    num_layers=3) in fp32 on a ragged sequence count: every layer's h within 2e-5, the input
    gradient within 1e-4 of its peak."""
    K = importlib.import_module("mid-attribute-speaker-generation_amd.kernels")
    lib = importlib.import_module("mid-attribute-speaker-generation_amd._lib").lib
    N, T, H, D, L = 21, 17, 256, 80, 3
    ref = torch.nn.LSTM(D, H, num_layers=L, batch_first=True).cuda()
    gen = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for prm in ref.parameters():
            prm.copy_(torch.randn(prm.shape, generator=gen) * 0.1)
    W = lambda n: getattr(ref, n).detach().contiguous()
    w_ih = [W(f"weight_ih_l{l}") for l in range(L)]
    w_hh = torch.stack([W(f"weight_hh_l{l}") for l in range(L)])
    bias = torch.stack([W(f"bias_ih_l{l}") + W(f"bias_hh_l{l}") for l in range(L)])
    w_ih_up = torch.stack(w_ih[1:])
    x = torch.randn(N * T, D, generator=gen).cuda()
    dh = (torch.randn(N * T, H, generator=gen) * 0.1).cuda()
    rows = N * T
    gx = torch.empty(rows, 4 * H, device="cuda")
    h, c = (torch.empty(L, rows, H, device="cuda") for _ in range(2))
    act, dg = (torch.empty(L, rows, 4 * H, device="cuda") for _ in range(2))
    dc, dx = torch.empty(L * 2 * N * H, device="cuda"), torch.empty(rows, D, device="cuda")
    P = lambda t: t.data_ptr()
    assert lib.fs2_lstm_stack_fwd(P(x), N, T, D, H, L, P(w_ih[0]), P(w_ih_up), P(w_hh), P(bias),
                                  P(gx), P(h), P(c), P(act), K.stream()) == 0
    tr = lambda t: t.transpose(-1, -2).contiguous()
    w_ih0_t, w_ih_up_t, w_hh_t = tr(w_ih[0]), tr(w_ih_up), tr(w_hh)
    assert lib.fs2_lstm_stack_bwd(P(dh), N, T, D, H, L, P(w_ih0_t), P(w_ih_up_t), P(w_hh_t),
                                  P(act), P(c), P(dg), P(dc), P(dx), K.stream()) == 0
    torch.cuda.synchronize()
    xr = x.view(N, T, D).clone().requires_grad_()
    out, (hn, _) = ref(xr)
    out.backward(dh.view(N, T, H))
    assert (h[L - 1].view(N, T, H) - out.detach()).abs().max().item() < 2e-5
    for l in range(L):  # last step of every layer
        assert (h[l].view(N, T, H)[:, -1] - hn[l].detach()).abs().max().item() < 2e-5
    assert (dx.view(N, T, D) - xr.grad).abs().max().item() < 1e-4 * xr.grad.abs().max().item()
