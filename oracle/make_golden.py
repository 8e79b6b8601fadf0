"""ORACLE — TEST INFRASTRUCTURE ONLY.  Captures golden vectors from the *reference itself*.

Run in the build container (``python oracle/make_golden.py``): it imports the reference
hot path from ``/root/reference`` (read-only; offline stubs for the three import-time-only
modules ``ot``/``unidecode``/``inflect`` and a bypass of ``model/__init__.py``, per
SURVEY.md §8c), runs it on CPU in fp32 with dropout disabled, and writes small ``.npz``
fixtures to ``tests/golden/``.  Only data leaves this script; the reference never travels
to the GPU box.

Fixtures:
  g1_lr.npz        LengthRegulator known-answer tests (int and float durations, cropping)
  g2_round.npz     inference duration rounding (half-to-even)
  g3_bucket.npz    bucketize KATs and the 255-entry pitch/energy bins
  g4_ops.npz       per-module fwd outputs / input grads / weight-grad checksums
  g5_step_*.npz    3-step training trajectories (losses, eloss, grad norm, lr, output sums)
  g6_infer.npz     eval-mode forward (synthesize.py / evaluate.py): predicted durations with
                   controls, teacher-forced eval, synthesize_from_speaker_emb, and a decoder
                   longer than max_seq_len (fresh position table)
  g7_gmm_ops.npz   mid-attribute GMM operations (model/distributions.py): InterpolateGMM
                   cost / OT plan / mixture at two rates, BarycenterGMM at two rate vectors.
                   POT is absent: ``ot.emd`` is stubbed by the same LP solved with scipy's
                   HiGHS (unique optimum); BarycenterGMM's ``_print`` TypeError is bypassed
                   by letting ``_barycenter_gaussians`` accept and ignore the kwarg.
  g8_data.npz      data pipeline (dataset.py, utils/tools.py pad_1D/pad_2D): the reference's
                   Dataset + ConcatDataset + collate_fn over the seeded synthetic corpora of
                   tests/synth_corpus.py (one corpus with accent files, one without): two
                   sorted/drop-last draws through the concatenation (14-tuples) and the
                   accent-free corpus alone unsorted with its tail kept (13-tuples)
  g9_hifigan.npz   HiFi-GAN generator (hifigan/models.py, config.json V1) after
                   remove_weight_norm with name-seeded weights: waveform and the int16 PCM of
                   vocoder_infer for a seeded (2, 80, 24) mel, and one utterance of 37 frames
  g10_clf.npz      the --use_clf language discriminator (train.py:168-197): the GE2E
                   SpeechEmbedder (3-layer LSTM 80->256, projection 64, DA classifier) and
                   GE2ELoss's BCE term on seeded weights -- embeddings, logits, da_loss and the
                   input gradient of a weighted da_loss -- and 2 training steps of the full
                   use_clf step at SYN-3x48 (the hparam file path and librosa are stubbed: the
                   module reads /path/to/.../config.yaml at import, values from its own
                   config/config.yaml)
"""
import importlib
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)


def import_reference():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    for n in ("ot", "unidecode", "inflect"):
        sys.modules.setdefault(n, types.ModuleType(n))
    sys.modules["unidecode"].unidecode = lambda s: s
    sys.modules["inflect"].engine = lambda: None
    pkg = types.ModuleType("model")
    pkg.__path__ = [os.path.join(REF, "model")]
    sys.modules["model"] = pkg
    fs2 = importlib.import_module("model.fastspeech2")
    loss = importlib.import_module("model.loss")
    mods = importlib.import_module("model.modules")
    layers = importlib.import_module("transformer.Layers")
    return fs2, loss, mods, layers


def no_dropout():
    torch.nn.functional.dropout = lambda x, p=0.5, training=True, inplace=False: x


PKG = importlib.import_module("mid-attribute-speaker-generation_amd")


def seeded(module, prefix=""):
    sd = module.state_dict()
    new = PKG.seeded.seeded_state_dict((prefix + k, v.shape) for k, v in sd.items())
    with torch.no_grad():
        for k, v in sd.items():
            if prefix + k in new:
                v.copy_(torch.from_numpy(new[prefix + k]))
    return module


def probe_idx(n, k=16, seed=0):
    return np.random.default_rng(seed + n).integers(0, n, size=k)


def grad_summary(module, prefix):
    out = {}
    for name, p in module.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().reshape(-1).double().numpy()
        idx = probe_idx(g.size)
        out[f"{prefix}{name}.gsum"] = np.array([g.sum(), np.abs(g).sum()])
        out[f"{prefix}{name}.gprobe"] = g[idx].astype(np.float32)
    return out


def g1_g2_g3(mods):
    LR = mods.LengthRegulator()
    x = torch.arange(24, dtype=torch.float32).view(2, 4, 3)
    res = {"x": x.numpy()}
    d_int = torch.tensor([[1, 0, 2, 3], [2, 2, 0, 0]])
    d_flt = torch.tensor([[1.7, -1.0, 2.2, 0.0], [0.49, 2.5, 3.0, 1.0]])
    for name, d, ml in (("int", d_int, None), ("flt", d_flt, None), ("crop", d_int, 4),
                        ("pad", d_int, 9)):
        o, ln = LR(x, d, ml)
        res[f"d_{name}"] = d.numpy()
        res[f"out_{name}"] = o.numpy()
        res[f"len_{name}"] = ln.numpy()
        res[f"maxlen_{name}"] = np.array(-1 if ml is None else ml)
    rng = np.random.default_rng(1)
    d_rand = rng.integers(-2, 6, size=(5, 11))
    xr = torch.from_numpy(rng.standard_normal((5, 11, 7)).astype(np.float32))
    o, ln = LR(xr, torch.from_numpy(d_rand), None)
    res.update(d_rand=d_rand, x_rand=xr.numpy(), out_rand=o.numpy(), len_rand=ln.numpy())
    np.savez_compressed(os.path.join(OUT, "g1_lr.npz"), **res)

    # G2: exp(log(d+1)) - 1 -> round (half to even) -> clamp at 0 (modules.py:132-135)
    d = torch.tensor([1.5, 2.5, 3.5, 0.2, 0.5, -0.7, 7.49])
    logd = torch.log(d + 1)
    r = torch.clamp(torch.round(torch.exp(logd) - 1) * 1.0, min=0)
    np.savez_compressed(os.path.join(OUT, "g2_round.npz"), log_d=logd.numpy(), rounded=r.numpy())

    # G3: bucketize (modules.py:84,96) incl. bins built from stats.json
    cfg = PKG.config.config_dir("JVS-VCTK")
    pp, mc, tc, path = PKG.config.load_configs(cfg)
    va = mods.VarianceAdaptor(pp, mc, path)
    v = torch.tensor([-2.0, -1.0, -0.5, 0.0, 1.0, 2.0])
    bins = torch.tensor([-1.0, 0.0, 1.0])
    vr = torch.from_numpy(np.random.default_rng(3).standard_normal(4096).astype(np.float32) * 4)
    edge = va.pitch_bins.detach()[::17].clone()
    np.savez_compressed(
        os.path.join(OUT, "g3_bucket.npz"), v=v.numpy(), bins=bins.numpy(),
        idx=torch.bucketize(v, bins).numpy(),
        pitch_bins=va.pitch_bins.detach().numpy(), energy_bins=va.energy_bins.detach().numpy(),
        v_rand=vr.numpy(), pitch_idx=torch.bucketize(vr, va.pitch_bins).numpy(),
        energy_idx=torch.bucketize(vr, va.energy_bins).numpy(),
        v_edge=edge.numpy(), edge_idx=torch.bucketize(edge, va.pitch_bins).numpy())


def g4(fs2, loss_mod, mods, layers):
    torch.manual_seed(0)
    rng = np.random.default_rng(4)
    res = {}
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")

    # FFT block (decoder-sized), B=3 T=24, lengths 24/17/9
    blk = seeded(layers.FFTBlock(256, 2, 128, 128, 1024, [9, 1], dropout=0.2), "fft.")
    B, T = 3, 24
    lens = torch.tensor([24, 17, 9])
    pad = torch.arange(T)[None] >= lens[:, None]
    x = torch.from_numpy(rng.standard_normal((B, T, 256)).astype(np.float32)).requires_grad_()
    y, _ = blk(x, mask=pad, slf_attn_mask=pad[:, None, :].expand(-1, T, -1))
    gy = torch.from_numpy(rng.standard_normal((B, T, 256)).astype(np.float32))
    y.backward(gy)
    res.update({"fft.x": x.detach().numpy(), "fft.lens": lens.numpy(), "fft.y": y.detach().numpy(),
                "fft.gy": gy.numpy(), "fft.gx": x.grad.numpy()})
    res.update(grad_summary(blk, "fft."))

    # Variance predictor, B=3 T=20 (padding rows nonzero on purpose)
    vp = seeded(mods.VariancePredictor(mc), "vp.")
    B, T = 3, 20
    lens = torch.tensor([20, 13, 5])
    pad = torch.arange(T)[None] >= lens[:, None]
    x = torch.from_numpy(rng.standard_normal((B, T, 256)).astype(np.float32)).requires_grad_()
    y = vp(x, pad)
    gy = torch.from_numpy(rng.standard_normal((B, T)).astype(np.float32))
    y.backward(gy)
    res.update({"vp.x": x.detach().numpy(), "vp.lens": lens.numpy(), "vp.y": y.detach().numpy(),
                "vp.gy": gy.numpy(), "vp.gx": x.grad.numpy()})
    res.update(grad_summary(vp, "vp."))

    # PostNet (train mode: batch statistics), B=2 T=40
    pn = seeded(layers.PostNet(), "pn.")
    pn.train()
    x = torch.from_numpy(rng.standard_normal((2, 40, 80)).astype(np.float32)).requires_grad_()
    y = pn(x)
    gy = torch.from_numpy(rng.standard_normal((2, 40, 80)).astype(np.float32))
    y.backward(gy)
    res.update({"pn.x": x.detach().numpy(), "pn.y": y.detach().numpy(), "pn.gy": gy.numpy(),
                "pn.gx": x.grad.numpy()})
    res.update(grad_summary(pn, "pn."))
    for i in range(5):
        res[f"pn.running_mean{i}"] = pn.convolutions[i][1].running_mean.numpy()
        res[f"pn.running_var{i}"] = pn.convolutions[i][1].running_var.numpy()

    # GMM head + SpeakerMetaEncLoss, B=6
    enc = seeded(fs2.SpeakerMetaEncoder(pp, mc), "senc.")
    meta = torch.from_numpy(np.concatenate([np.eye(2)[[0, 1, 1, 0, 0, 1]],
                                            np.eye(2)[[1, 1, 0, 0, 1, 0]]], 1).astype(np.float32))
    e = torch.from_numpy(rng.standard_normal((6, 256)).astype(np.float32) * 0.5)
    gmm = enc(meta)
    el = loss_mod.SpeakerMetaEncLoss(pp, mc)(e, gmm)
    (-el).backward()
    res.update({"gmm.meta": meta.numpy(), "gmm.e": e.numpy(), "gmm.eloss": np.array(float(el)),
                "gmm.logp": gmm.log_prob(e).detach().numpy(),
                "gmm.pi": gmm.mixture_distribution.probs.detach().numpy(),
                "gmm.mu": gmm.component_distribution.base_dist.loc.detach().numpy(),
                "gmm.sigma": gmm.component_distribution.base_dist.scale.detach().numpy()})
    for name, p in enc.named_parameters():
        res[f"gmm.{name}.grad"] = p.grad.numpy()
    np.savez_compressed(os.path.join(OUT, "g4_ops.npz"), **res)


def g5(fs2, loss_mod, B, Ts, steps=3, seed=0, config="JVS-VCTK", name=None, curve_only=False):
    """3-step trajectories (``g5_step_*``); with ``curve_only`` a long run that stores only
    the per-step scalars (``g11_curve_*``: the loss curve the bf16 path is checked against)."""
    from model.optimizer import ScheduledOptim
    pp, mc, tc, path = PKG.config.load_configs(config)
    torch.manual_seed(0)
    model = fs2.FastSpeech2(pp, mc, path)
    seeded(model)
    model.train()
    opt = ScheduledOptim(model, tc, mc, 0)
    Loss = loss_mod.FastSpeech2Loss(pp, mc)
    eLoss = loss_mod.SpeakerMetaEncLoss(pp, mc)
    res = {"B": np.array(B), "Ts": np.array(Ts), "seed": np.array(seed),
           "config": np.array(config)}
    batch = PKG.data.to_device(PKG.data.syn_batch_for(config, B, Ts, seed=seed), "cpu")
    res["pos_enc_probe"] = model.encoder.position_enc.detach()[0, ::97, ::31].numpy()
    if curve_only:
        curve = []
        for s in range(steps):
            output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
            losses = Loss(batch[:12], output[:-2])
            losses[0].backward()
            eloss = eLoss(output[-1], output[-2])
            (-eloss).backward()
            gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step_and_update_lr()
            opt.zero_grad()
            curve.append([float(l) for l in losses] + [float(eloss), float(gn)])
        res["curve"] = np.array(curve)
        np.savez_compressed(os.path.join(OUT, name), **res)
        print(name, res["curve"][0], res["curve"][-1])
        return
    for s in range(steps):
        output = model(*(batch[2:12]), accents=batch[13], speaker_meta=batch[12])
        losses = Loss(batch[:12], output[:-2])
        losses[0].backward()
        eloss = eLoss(output[-1], output[-2])
        (-eloss).backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step_and_update_lr()
        opt.zero_grad()
        res[f"s{s}.losses"] = np.array([float(l) for l in losses])
        res[f"s{s}.eloss"] = np.array(float(eloss))
        res[f"s{s}.gnorm"] = np.array(float(gn))
        res[f"s{s}.lr"] = np.array(opt._optimizer.param_groups[0]["lr"])
        o, po = output[0].detach().double(), output[1].detach().double()
        res[f"s{s}.out_sum"] = np.array([o.sum(), o.abs().sum(), po.sum(), po.abs().sum()])
        res[f"s{s}.out_probe"] = output[1].detach()[:, ::37, ::7].numpy()
        res[f"s{s}.pred_probe"] = np.stack([output[2].detach().numpy(), output[3].detach().numpy(),
                                            output[4].detach().numpy()])
        res[f"s{s}.mel_lens"] = output[9].numpy()
    res["final_probe"] = torch.cat([p.detach().reshape(-1)[:64] for p in model.parameters()
                                    if p.requires_grad]).numpy()
    name = name or f"g5_step_b{B}_t{Ts}.npz"
    np.savez_compressed(os.path.join(OUT, name), **res)
    print(name, res["s0.losses"], res["s2.losses"])


def infer_overrides(model_prefix=""):
    """Fixture-only weight overrides for the eval-mode cases (applied identically to every
    implementation under test): a duration-head bias so predicted durations are a few
    frames per phoneme instead of ~0, and non-trivial PostNet BatchNorm running stats."""
    rng = np.random.default_rng(6)
    ov = {model_prefix + "variance_adaptor.duration_predictor.linear_layer.bias":
          np.array([np.log(4.0)], np.float32)}
    chans = [512, 512, 512, 512, 80]
    for i, c in enumerate(chans):
        ov[f"{model_prefix}postnet.convolutions.{i}.1.running_mean"] = \
            (0.1 * rng.standard_normal(c)).astype(np.float32)
        ov[f"{model_prefix}postnet.convolutions.{i}.1.running_var"] = \
            (0.5 + rng.random(c)).astype(np.float32)
    return ov


def _apply(model, ov):
    sd = model.state_dict()
    with torch.no_grad():
        for k, v in ov.items():
            sd[k].copy_(torch.from_numpy(v))


def g6(fs2, loss_mod):
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    torch.manual_seed(0)
    model = fs2.FastSpeech2(pp, mc, path)
    seeded(model)
    ov = infer_overrides()
    _apply(model, ov)
    model.eval()
    res = {"ov." + k: v for k, v in ov.items()}

    def record(tag, out):
        for i, name in enumerate(("out", "post", "p", "e", "log_d", "d_r")):
            res[f"{tag}.{name}"] = out[i].detach().float().numpy()
        res[f"{tag}.mel_mask"] = out[7].numpy()
        res[f"{tag}.mel_lens"] = out[9].numpy()

    b = PKG.data.to_device(PKG.data.syn_batch(3, 16, seed=0), "cpu")
    with torch.no_grad():
        # A: synthesize.py -- no targets, unit controls
        record("A", model(b[2], b[3], b[4], b[5], accents=b[13], speaker_meta=b[12]))
        # B: controls (energy follows p_control: modules.py:124)
        record("B", model(b[2], b[3], b[4], b[5], p_control=1.3, e_control=0.7, d_control=1.2,
                          accents=b[13], speaker_meta=b[12]))
        # C: evaluate.py -- teacher-forced forward in eval mode, plus the loss 6-tuple
        out = model(*(b[2:12]), accents=b[13], speaker_meta=b[12])
        record("C", out)
        losses = loss_mod.FastSpeech2Loss(pp, mc)(b[:12], out[:-2])
        res["C.losses"] = np.array([float(l) for l in losses])
        # D: examples_gen_distri.py -- given speaker embedding, B = 1
        b1 = PKG.data.to_device(PKG.data.syn_batch(1, 20, seed=5), "cpu")
        emb = torch.from_numpy(np.random.default_rng(7).standard_normal((1, 256))
                               .astype(np.float32) * 0.5)
        res["D.emb"] = emb.numpy()
        record("D", model.synthesize_from_speaker_emb(None, b1[3], b1[4], b1[5], accents=b1[13],
                                                      speaker_emb=emb))
        # E: decoder longer than max_seq_len (eval: fresh position table, no truncation)
        bl = PKG.data.to_device(PKG.data.syn_batch(1, 128, seed=9), "cpu")
        model.variance_adaptor.duration_predictor.linear_layer.bias.fill_(float(np.log(9.5)))
        out = model(bl[2], bl[3], bl[4], bl[5], accents=bl[13], speaker_meta=bl[12])
        res["E.dur_bias"] = np.array([np.log(9.5)], np.float32)
        res["E.mel_lens"] = out[9].numpy()
        res["E.d_r"] = out[5].numpy()
        res["E.post_probe"] = out[1][:, ::13, ::5].numpy()
        res["E.post_sum"] = np.array([out[1].double().sum(), out[1].double().abs().sum()])
        print("g6: mel lens A", res["A.mel_lens"], "B", res["B.mel_lens"], "D",
              res["D.mel_lens"], "E", res["E.mel_lens"])
    np.savez_compressed(os.path.join(OUT, "g6_infer.npz"), **res)


def g7(fs2):
    from oracle import gmm_ops
    sys.modules["ot"].emd = lambda a, b, M: gmm_ops.emd(a, b, np.asarray(M, np.float64))
    sys.modules["model"].FastSpeech2 = fs2.FastSpeech2
    dist = importlib.import_module("model.distributions")
    orig = dist.BarycenterGMM._barycenter_gaussians
    dist.BarycenterGMM._barycenter_gaussians = lambda self, _print=True: orig(self)
    pp, mc, tc, path = PKG.config.load_configs("JVS-VCTK")
    torch.manual_seed(0)
    model = fs2.FastSpeech2(pp, mc, path)
    seeded(model)
    # spread the per-metadata mixtures apart (fixture-only: seeded heads give near-equal ones)
    rng = np.random.default_rng(7)
    ov = {}
    with torch.no_grad():
        for name in ("pi_linear.0.weight", "sigma_linear.0.weight", "mu_linear.weight"):
            p_ = dict(model.speaker_enc.named_parameters())[name]
            scale = {"pi": 1.5, "sigma": 0.6, "mu": 1.0}[name.split("_")[0]]
            p_.add_(torch.from_numpy((scale * rng.standard_normal(tuple(p_.shape)))
                                     .astype(np.float32)))
            ov["speaker_enc." + name] = p_.detach().numpy().copy()
    model.eval()
    res = {"ov." + k: v for k, v in ov.items()}

    def params(g):
        return (g.mixture_distribution.probs.detach().numpy(),
                g.component_distribution.base_dist.loc.detach().numpy(),
                g.component_distribution.base_dist.scale.detach().numpy())

    meta_a = torch.tensor([[1.0, 0.0, 1.0, 0.0]])
    meta_b = torch.tensor([[0.0, 1.0, 0.0, 1.0]])
    ga, gb = model.speaker_distribution(meta_a), model.speaker_distribution(meta_b)
    res["I.meta_a"], res["I.meta_b"] = meta_a.numpy(), meta_b.numpy()
    for tag, g in (("a", ga), ("b", gb)):
        res[f"I.pi_{tag}"], res[f"I.mu_{tag}"], res[f"I.sd_{tag}"] = params(g)
    ig = dist.InterpolateGMM(ga, gb)
    res["I.cost"] = np.array(ig.ot_Cost, np.float64)
    res["I.plan"] = np.asarray(ig.ot_Matrix, np.float64)
    for t in (0.5, 0.3):
        if t != 0.5:
            ig.interpolate_rate(t)
        pi, mu, sd = params(ig)
        res[f"I.t{t}.pi"] = pi.astype(np.float64)
        res[f"I.t{t}.mu"] = mu.astype(np.float32)
        res[f"I.t{t}.sd"] = sd.astype(np.float64)
    bg = dist.BarycenterGMM(model)
    for tag, rate in (("u", None), ("w", [0.5, 0.25, 0.125, 0.125])):
        if rate is not None:
            bg.barycenter_rate(rate, _print=False)
        pi, mu, sd = params(bg)
        res[f"G.{tag}.pi"], res[f"G.{tag}.mu"], res[f"G.{tag}.sd"] = pi, mu, sd
        res[f"G.{tag}.rate"] = np.array(bg.rate, np.float64)
    res["G.metas"] = np.stack([m.numpy()[0] for m in bg.original_distri.keys()])
    print("g7: plan", res["I.plan"].round(4).tolist(), "barycenter comps",
          res["G.u.pi"].shape, res["G.w.pi"].shape)
    np.savez_compressed(os.path.join(OUT, "g7_gmm_ops.npz"), **res)


BATCH_FIELDS = ("ids", "raw_texts", "speakers", "texts", "src_lens", "max_src_len", "mels",
                "mel_lens", "max_mel_len", "pitches", "energies", "durations", "speaker_meta",
                "accents")


def g8():
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from synth_corpus import make_corpora
    ds_mod = importlib.import_module("dataset")  # the reference's dataset.py
    res = {}
    with tempfile.TemporaryDirectory() as root:
        cfg_dir, corpora, pp, tc = make_corpora(root, seed=0)
        dsets = []
        for corpus in corpora:  # train.py:36-47
            cfg = dict(corpus)
            cfg["preprocessing"] = dict(pp, text=corpus["text"], accent=corpus["accent"])
            dsets.append(ds_mod.Dataset("train.txt", cfg, tc, sort=True, drop_last=True))
        concat = ds_mod.ConcatDataset(cfg_dir, dsets)
        order = np.random.default_rng(1).permutation(len(concat))
        res["order"] = order
        draws = [order[:16], order[16:]]  # a loader batch of batch_size * 4, then the rest
        cfg = dict(corpora[1])
        cfg["preprocessing"] = dict(pp, text=corpora[1]["text"], accent=corpora[1]["accent"])
        plain = ds_mod.Dataset("train.txt", cfg, tc, sort=False, drop_last=False)
        runs = [("c0", concat, draws[0]), ("c1", concat, draws[1]),
                ("p0", plain, np.arange(len(plain)))]
        for tag, ds, idx in runs:
            batches = ds.collate_fn([ds[int(i)] for i in idx])
            res[f"{tag}.n"] = np.int64(len(batches))
            for j, b in enumerate(batches):
                for name, v in zip(BATCH_FIELDS, b):
                    res[f"{tag}.{j}.{name}"] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, "g8_data.npz"), **res)
    print("g8:", {k: v for k, v in res.items() if k.endswith(".n")})


def g9():
    import json
    hf = importlib.import_module("hifigan")
    with open(os.path.join(REF, "hifigan", "config.json")) as f:
        h = hf.AttrDict(json.load(f))
    gen = hf.Generator(h)
    gen.eval()
    gen.remove_weight_norm()
    seeded(gen)
    sd = gen.state_dict()
    res = {"keys": np.array(list(sd.keys())),
           "shapes": np.array([",".join(map(str, v.shape)) for v in sd.values()])}
    rng = np.random.default_rng(9)
    for tag, (B, T) in (("a", (2, 24)), ("b", (1, 37))):
        mel = torch.from_numpy((rng.standard_normal((B, 80, T)) * 2 - 5).astype(np.float32))
        with torch.no_grad():
            wav = gen(mel).squeeze(1)
        res[f"{tag}.mel"] = mel.numpy()
        res[f"{tag}.wav"] = wav.numpy()
        res[f"{tag}.pcm"] = (wav.numpy() * 32768.0).astype("int16")  # utils/model.py:84-88
    np.savez_compressed(os.path.join(OUT, "g9_hifigan.npz"), **res)
    print("g9:", {k: v.shape for k, v in res.items()})


def import_discriminator():
    """The reference's SpeechEmbedder / GE2ELoss package, with its import-time hparam file
    (an absolute placeholder path) read from the package's own config/config.yaml and
    librosa (absent, used only by data utilities) stubbed."""
    pkg_dir = os.path.join(REF, "Multilingual-Speaker-Encoder-with-Domain-Adaptation")
    name = "Multilingual-Speaker-Encoder-with-Domain-Adaptation"
    sys.modules.setdefault("librosa", types.ModuleType("librosa"))
    pkg = types.ModuleType(name)
    pkg.__path__ = [pkg_dir]
    sys.modules[name] = pkg
    hmod = types.ModuleType(name + ".hparam")
    src = open(os.path.join(pkg_dir, "hparam.py")).read()
    src = src.replace("hparam = Hparam()", "")
    exec(compile(src, os.path.join(pkg_dir, "hparam.py"), "exec"), hmod.__dict__)
    hmod.hparam = hmod.Hparam(os.path.join(pkg_dir, "config", "config.yaml"))
    sys.modules[name + ".hparam"] = hmod
    return importlib.import_module(name + ".speech_embedder_net")


CLF_PERM = {"B3": [2, 0, 1]}


def g10(fs2, loss_mod):
    import math
    sen = import_discriminator()
    torch.manual_seed(0)
    disc = sen.SpeechEmbedder()
    seeded(disc)
    dl = sen.GE2ELoss("cpu")
    res = {"disc.keys": np.array(list(disc.state_dict().keys())),
           "disc.shapes": np.array([",".join(map(str, v.shape)) for v in disc.state_dict().values()])}
    rng = np.random.default_rng(10)
    x = torch.from_numpy((rng.standard_normal((6, 150, 80)) * 2 - 3).astype(np.float32))
    x[4:, 100:] = 0.0  # zero-padded tail, as the chunked mel has
    langs = torch.tensor([1., 0., 1., 1., 0., 0.])
    xr = x.clone().requires_grad_()
    out = disc(xr)
    _, _, da = dl(out["embeddings"].view(6, 1, -1), out["da_lang_logits"], langs, reduction="sum")
    (da * 0.37).backward()
    res.update({"d.x": x.numpy(), "d.langs": langs.numpy(),
                "d.emb": out["embeddings"].detach().numpy(),
                "d.logits": out["da_lang_logits"].detach().numpy(),
                "d.da": np.float64(da.item()), "d.dx": xr.grad.numpy()})
    # full use_clf steps (train.py:142-206) at SYN-3x48, dropout off, fixed speaker shuffle
    cfg = "/root/reference/config/JVS-VCTK_langemb_configs/JVS-VCTK_1"
    import yaml
    pp = yaml.safe_load(open(cfg + "/preprocess.yaml"))
    mc = yaml.safe_load(open(cfg + "/model.yaml"))
    tc = yaml.safe_load(open(cfg + "/train.yaml"))
    model = fs2.FastSpeech2(pp, mc, cfg)
    seeded(model)
    model.train()
    opt_mod = importlib.import_module("model.optimizer")
    optim = opt_mod.ScheduledOptim(model, tc, mc, 0)
    Loss = loss_mod.FastSpeech2Loss(pp, mc)
    eLoss = loss_mod.SpeakerMetaEncLoss(pp, mc)
    b = PKG.data.syn_batch(3, 48, seed=3)
    batch = PKG.data.to_device(b, "cpu")
    perm = CLF_PERM["B3"]
    step_of, total = 4, 10  # the DA coefficient 2/(1+e^{-10 p})-1 at p = 0.4 (0.96)
    for it in range(2):
        accents, speaker_meta = batch[13], batch[12]
        bb = batch[:12]
        output = model(*(bb[2:]), accents=accents, speaker_meta=speaker_meta)
        losses = Loss(bb, output[:-2])
        losses[0].backward()
        eloss = eLoss(output[-1], output[-2])
        (-eloss).backward()
        speakers = torch.stack([bb[2][perm[i]] for i in range(3)])
        sm = torch.stack([speaker_meta[perm[i]] for i in range(3)])
        bb2 = bb[:2] + (speakers,) + bb[3:]
        output = model(*(bb2[2:]), accents=accents, speaker_meta=sm)
        max_len = output[0].shape[1]
        max_len_r = max_len // 150 + 1
        n_mels = output[0].shape[2]
        batch_r_m = torch.cat([output[0], torch.zeros(3, max_len_r * 150 - max_len, n_mels)],
                              dim=1).view(3 * max_len_r, 150, n_mels)
        langs = sm[:, 2].view(-1, 1).repeat(1, max_len_r).view(-1)
        output_r = disc(batch_r_m)
        _, _, dloss = dl(output_r.get("embeddings").view(3 * max_len_r, 1, -1),
                         output_r.get("da_lang_logits"), langs, reduction="sum")
        coef = 2 / (1 + math.exp(-10 * (step_of / total))) - 1
        (dloss * coef / len(langs) * 1.0).backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        optim.step_and_update_lr()
        optim.zero_grad()
        res[f"s{it}.losses"] = np.array([l.item() for l in losses])
        res[f"s{it}.eloss"] = np.float64(eloss.item())
        res[f"s{it}.dloss"] = np.float64(dloss.item())
        res[f"s{it}.gnorm"] = np.float64(gn.item())
        res[f"s{it}.max_len_r"] = np.int64(max_len_r)
        step_of += 1
    res["perm"] = np.array(perm)
    np.savez_compressed(os.path.join(OUT, "g10_clf.npz"), **res)
    print("g10:", {k: v for k, v in res.items() if k.startswith(("s0", "s1", "d.da"))})


def main():
    os.makedirs(OUT, exist_ok=True)
    if "--only-g10" in sys.argv:
        fs2, loss_mod, mods, layers = import_reference()
        no_dropout()
        torch.set_num_threads(8)
        g10(fs2, loss_mod)
        return
    if "--only-g9" in sys.argv:
        sys.path.insert(0, REF)
        sys.dont_write_bytecode = True
        torch.set_num_threads(8)
        g9()
        return
    if "--only-g8" in sys.argv:
        sys.path.insert(0, REF)
        sys.dont_write_bytecode = True
        for n in ("unidecode", "inflect"):
            sys.modules.setdefault(n, types.ModuleType(n))
        sys.modules["unidecode"].unidecode = lambda s: s
        sys.modules["inflect"].engine = lambda: None
        g8()
        return
    fs2, loss_mod, mods, layers = import_reference()
    no_dropout()
    torch.set_num_threads(8)
    if "--only-g6" in sys.argv:
        g6(fs2, loss_mod)
        return
    if "--only-g7" in sys.argv:
        g7(fs2)
        return
    if "--only-r2" in sys.argv:  # round-2 fixtures: JSUT (BASELINE config 1), loss curve
        r2_fixtures(fs2, loss_mod)
        return
    g1_g2_g3(mods)
    g4(fs2, loss_mod, mods, layers)
    g6(fs2, loss_mod)
    g7(fs2)
    g8()
    g9()
    g10(fs2, loss_mod)
    sizes = [(3, 16), (8, 32)] + ([(48, 128)] if "--full" in sys.argv else [])
    for B, Ts in sizes:
        g5(fs2, loss_mod, B, Ts)
    r2_fixtures(fs2, loss_mod)


def r2_fixtures(fs2, loss_mod):
    """g5_step_jsut_b4_t128: BASELINE config 1 (config/JSUT/model.yaml: K = 1 GMM component,
    1 speaker, gender-only metadata of width 2) at batch 4, 128 phonemes x 512 frames, 3 steps.
    g11_curve_b8_t32: 100 steps at SYN-8x32 (per-step losses, eloss, grad norm).
    g5_step_b2_t264_trunc: 3 steps with 1,056 mel frames (decoder truncation to 1,000)."""
    g5(fs2, loss_mod, 4, 128, config="JSUT", name="g5_step_jsut_b4_t128.npz")
    g5(fs2, loss_mod, 8, 32, steps=100, name="g11_curve_b8_t32.npz", curve_only=True)
    # training-mode decoder truncation (transformer/Models.py:166-174): 4 x 264 = 1,056 frames
    # > max_seq_len 1,000, so the decoder, its mask and the mel loss see 1,000 frames while
    # mel_lens stay uncropped
    g5(fs2, loss_mod, 2, 264, name="g5_step_b2_t264_trunc.npz")


if __name__ == "__main__":
    main()
