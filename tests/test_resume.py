"""Checkpoint save / resume (``train.py:271-285``, ``utils/model.py:15-28``) and gradient
accumulation (``train.py:112,159,165,200``) of the HIP training step.

* A run interrupted after k steps -- ``{"model", "optimizer"}`` saved with ``torch.save``,
  reloaded into a fresh model through ``load_state_dict`` and ``ScheduledOptim(...,
  restore_step)`` + ``load_state_dict`` -- continues bitwise-equal to an uninterrupted run.
* A checkpoint written by ``torch.optim.Adam`` (the CPU oracle's optimiser, the reference's
  format) loads, and the next step matches the oracle's next step (fp32, 1e-4 relative).
* ``grad_acc_step = 2``: two identical half-scaled micro-batches equal one full step
  bitwise; two different micro-batches match the oracle running ``train.py``'s
  accumulation (losses / grad_acc_step, step every grad_acc_step batches).
"""
import copy
import importlib
import io

import numpy as np
import pytest
import torch

from oracle import fs2_cpu

pytestmark = pytest.mark.gpu
PKG = importlib.import_module("mid-attribute-speaker-generation_amd")
M = importlib.import_module("mid-attribute-speaker-generation_amd.model")
T = importlib.import_module("mid-attribute-speaker-generation_amd.train")
DEV = "cuda"


def _model(dtype=torch.float32):
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    model = M.FastSpeech2(pp, mc, path, device=DEV, compute_dtype=dtype)
    PKG.seeded.load_seeded_(model)
    model.dropout = False
    model.train()
    return model, (pp, mc, tc)


def _batch(B, Ts, seed, dev=DEV):
    return PKG.data.to_device(PKG.data.syn_batch(B, Ts, seed=seed), dev)


def _roundtrip(obj):
    buf = io.BytesIO()
    torch.save(obj, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resume_continues_bitwise(dtype):
    batches = [_batch(4, 24, seed=s) for s in (1, 2, 3, 4)]
    # uninterrupted: 4 steps
    model, (pp, mc, tc) = _model(dtype)
    tr = T.Trainer(model, pp, mc, tc)
    for b in batches:
        tr.step(b)
    torch.cuda.synchronize()
    want = (model.arena().flat.clone(), tr.opt.m.clone(), tr.opt.v.clone(),
            tr.opt._optimizer.param_groups[0]["lr"])
    # interrupted after 2 steps: save exactly as train.py:276-285 does
    model, _ = _model(dtype)
    tr = T.Trainer(model, pp, mc, tc)
    for b in batches[:2]:
        tr.step(b)
    ckpt = _roundtrip({"model": model.state_dict(), "optimizer": tr.opt._optimizer.state_dict()})
    assert len(ckpt["model"]) == 242
    del model, tr
    # resume as utils/model.py:15-28 does (restore_step = 2)
    model2, _ = _model(dtype)
    with torch.no_grad():
        for p in model2.parameters():
            p.add_(1.0)  # make sure the weights really come from the checkpoint
    model2.load_state_dict(ckpt["model"])
    tr2 = T.Trainer(model2, pp, mc, tc, current_step=2)
    tr2.opt.load_state_dict(ckpt["optimizer"])
    assert tr2.opt.adam_steps == 2 and tr2.opt.current_step == 2
    for b in batches[2:]:
        tr2.step(b)
    torch.cuda.synchronize()
    got = (model2.arena().flat, tr2.opt.m, tr2.opt.v)
    for a, b, name in zip(got, want[:3], ("weights", "exp_avg", "exp_avg_sq")):
        assert torch.equal(a, b), name
    assert tr2.opt._optimizer.param_groups[0]["lr"] == want[3]


def test_resume_from_torch_adam_checkpoint():
    """The reference's checkpoint format, written by torch.optim.Adam (CPU oracle, 2 steps),
    loads into the HIP model + ScheduledOptim; step 3 matches the oracle's step 3."""
    B, Ts = 3, 16
    fs2_cpu.DROPOUT["enabled"] = False
    ref, _ = fs2_cpu.build("JVS-VCTK")
    ref.train()
    opt = fs2_cpu.make_opt(ref)
    cb = _batch(B, Ts, seed=0, dev="cpu")
    for _ in range(2):
        fs2_cpu.train_step(ref, opt, cb)
    ckpt = _roundtrip({"model": ref.state_dict(), "optimizer": opt["adam"].state_dict()})
    rl, re_, rg, _ = fs2_cpu.train_step(ref, opt, cb)  # the oracle's step 3

    model, (pp, mc, tc) = _model()
    model.load_state_dict(ckpt["model"])
    tr = T.Trainer(model, pp, mc, tc, current_step=2)
    tr.opt.load_state_dict(ckpt["optimizer"])
    losses, eloss, gnorm, _ = tr.step(_batch(B, Ts, seed=0))
    got = [float(l) for l in losses] + [float(eloss), float(gnorm)]
    assert _rel(got, rl + [re_, rg]) <= 1e-4, (got, rl + [re_, rg])
    # weights and Adam moments after the step
    ours = dict(model.named_parameters())
    st = opt["adam"].state
    for name, p in ref.named_parameters():
        if not p.requires_grad:
            continue
        assert _rel(ours[name].detach().cpu(), p.detach()) <= 1e-4, name
        off = tr.opt.arena.offsets[[id(q) for q in tr.opt.arena.params].index(id(ours[name]))]
        m = tr.opt.m[off:off + p.numel()].cpu()
        assert _rel(m, st[p]["exp_avg"].reshape(-1)) <= 2e-4, name + " exp_avg"


def _tc_acc(tc, n):
    tc = copy.deepcopy(tc)
    tc["optimizer"]["grad_acc_step"] = n
    return tc


def test_grad_accumulation_identical_microbatches_bitwise():
    """grad_acc_step = 2 over (b, b): each micro-batch back-propagates loss / 2 (a power of
    two, so every gradient is exactly half) and the accumulated gradient is exactly the
    grad_acc_step = 1 gradient of b; weights and moments after the update are bitwise equal."""
    b = _batch(4, 24, seed=7)
    model, (pp, mc, tc) = _model()
    tr = T.Trainer(model, pp, mc, tc)
    tr.step(b)
    torch.cuda.synchronize()
    want = (model.arena().flat.clone(), tr.opt.m.clone(), tr.opt.v.clone())

    model2, _ = _model()
    tr2 = T.Trainer(model2, pp, mc, _tc_acc(tc, 2))
    out1 = tr2.step(b)
    assert out1[2] is None and tr2.opt.adam_steps == 0  # batch 1: accumulate only
    out2 = tr2.step(b)
    assert out2[2] is not None and tr2.opt.adam_steps == 1
    torch.cuda.synchronize()
    for a, w, name in zip((model2.arena().flat, tr2.opt.m, tr2.opt.v), want,
                          ("weights", "exp_avg", "exp_avg_sq")):
        assert torch.equal(a, w), name


def test_grad_accumulation_matches_oracle():
    """grad_acc_step = 2 over four different batches (two optimiser steps) against the CPU
    oracle running train.py:159-206's accumulation."""
    bs = [(3, 16, s) for s in (11, 12, 13, 14)]
    model, (pp, mc, tc) = _model()
    tr = T.Trainer(model, pp, mc, _tc_acc(tc, 2))
    got = []
    for (B, Ts, s) in bs:
        losses, eloss, gnorm, _ = tr.step(_batch(B, Ts, s))
        got.append([float(l) for l in losses] + [float(eloss)] +
                   ([float(gnorm)] if gnorm is not None else []))

    fs2_cpu.DROPOUT["enabled"] = False
    ref, _ = fs2_cpu.build("JVS-VCTK")
    ref.train()
    opt = fs2_cpu.make_opt(ref)
    want = []
    for i, (B, Ts, s) in enumerate(bs, start=1):
        cb = _batch(B, Ts, s, dev="cpu")
        out = ref(*cb[2:12], accents=cb[13], speaker_meta=cb[12])
        losses = fs2_cpu.fs2_loss(cb[:12], out[:-2])
        (losses[0] / 2).backward()
        eloss = fs2_cpu.speaker_enc_loss(out[-1], out[-2])
        (-eloss / 2).backward()
        row = [float(l) for l in losses] + [float(eloss)]
        if i % 2 == 0:
            row.append(float(torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)))
            opt["step"] += 1
            for g in opt["adam"].param_groups:
                g["lr"] = fs2_cpu.lr_at(opt["step"])
            opt["adam"].step()
            opt["adam"].zero_grad()
        want.append(row)
    for i, (a, w) in enumerate(zip(got, want)):
        assert len(a) == len(w) and _rel(a, w) <= 1e-4, (i, a, w)
    assert tr.opt.adam_steps == 2 and tr.opt.current_step == 2
