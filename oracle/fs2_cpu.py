"""ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference FastSpeech2 +
TacoSpawn training step, used by ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg as the *checker*.  The product path
(``mid-attribute-speaker-generation_amd``) never imports anything under ``oracle/``.

Pinning: ``tests/test_oracle_golden.py`` checks this restatement against golden vectors
captured from the reference itself (``oracle/make_golden.py`` imports
``/root/reference`` in the build container and writes ``tests/golden/*.npz``).

The restatement runs plain ATen ops on the CPU in fp32 with the reference's module tree and
state-dict names, so that ``load_state_dict`` moves weights between the
reference, this oracle and the HIP path.  Every block cites the reference line it follows.
Integer index math (LengthRegulator source-row maps, bucketize) is restated separately in
numpy in ``oracle/index_math.py``.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------------------


def mask_from_lengths(lengths, max_len=None):
    """True = padding.  ``utils/tools.py:155-163``."""
    if max_len is None:
        max_len = int(lengths.max())
    return torch.arange(max_len, device=lengths.device)[None, :] >= lengths[:, None]


def sinusoid_table(n_position, d_hid):
    """``transformer/Models.py:10-30``: angle = pos / 10000^(2*(i//2)/d), sin on even,
    cos on odd columns, evaluated in float64 and stored as float32."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    i = np.arange(d_hid)
    denom = np.array([np.power(10000, 2 * (j // 2) / d_hid) for j in i], dtype=np.float64)
    ang = pos / denom[None, :]
    tab = np.empty_like(ang)
    tab[:, 0::2] = np.sin(ang[:, 0::2])
    tab[:, 1::2] = np.cos(ang[:, 1::2])
    return torch.from_numpy(tab.astype(np.float32))


DROPOUT = {"enabled": True}


def _drop(x, p, training):
    if DROPOUT["enabled"]:
        return F.dropout(x, p, training)
    return x


# ---------------------------------------------------------------------------------------
# FFT block (transformer/Layers.py:11-30, SubLayers.py:8-93, Modules.py:6-25)
# ---------------------------------------------------------------------------------------


class MultiHeadAttention(nn.Module):
    def __init__(self, n_head, d_model, d_k, dropout):
        super().__init__()
        self.n_head, self.d_k, self.p = n_head, d_k, dropout
        self.w_qs = nn.Linear(d_model, n_head * d_k)
        self.w_ks = nn.Linear(d_model, n_head * d_k)
        self.w_vs = nn.Linear(d_model, n_head * d_k)
        self.layer_norm = nn.LayerNorm(d_model)
        self.fc = nn.Linear(n_head * d_k, d_model)

    def forward(self, x, key_pad):
        B, T, _ = x.shape
        h, dk = self.n_head, self.d_k
        # SubLayers.py:39-44 — (h*B, T, dk) head-major layout, index = head*B + b
        heads = lambda y: y.view(B, T, h, dk).permute(2, 0, 1, 3).reshape(h * B, T, dk)
        q, k, v = heads(self.w_qs(x)), heads(self.w_ks(x)), heads(self.w_vs(x))
        # Modules.py:16-23 — scores divided by sqrt(d_k); key padding -> -inf
        s = torch.bmm(q, k.transpose(1, 2)) / np.power(dk, 0.5)
        s = s.masked_fill(key_pad.repeat(h, 1)[:, None, :], -np.inf)
        o = torch.bmm(torch.softmax(s, dim=2), v)
        o = o.view(h, B, T, dk).permute(1, 2, 0, 3).reshape(B, T, h * dk)
        # SubLayers.py:54-55 — dropout(fc) + residual, post-LN
        return self.layer_norm(_drop(self.fc(o), self.p, self.training) + x)


class PositionwiseFeedForward(nn.Module):
    def __init__(self, d_in, d_hid, kernel_size, dropout):
        super().__init__()
        self.p = dropout
        self.w_1 = nn.Conv1d(d_in, d_hid, kernel_size[0], padding=(kernel_size[0] - 1) // 2)
        self.w_2 = nn.Conv1d(d_hid, d_in, kernel_size[1], padding=(kernel_size[1] - 1) // 2)
        self.layer_norm = nn.LayerNorm(d_in)

    def forward(self, x):
        # SubLayers.py:85-93
        y = self.w_2(F.relu(self.w_1(x.transpose(1, 2)))).transpose(1, 2)
        return self.layer_norm(_drop(y, self.p, self.training) + x)


class FFTBlock(nn.Module):
    def __init__(self, d_model, n_head, d_inner, kernel_size, dropout):
        super().__init__()
        self.slf_attn = MultiHeadAttention(n_head, d_model, d_model // n_head, dropout)
        self.pos_ffn = PositionwiseFeedForward(d_model, d_inner, kernel_size, dropout)

    def forward(self, x, pad):
        # Layers.py:21-30 — padded rows zeroed after each sub-layer
        x = self.slf_attn(x, pad).masked_fill(pad[..., None], 0)
        return self.pos_ffn(x).masked_fill(pad[..., None], 0)


def _stack_cfg(config, side):
    t = config["transformer"]
    return dict(d_model=t[f"{side}_hidden"], n_head=t[f"{side}_head"],
                d_inner=t["conv_filter_size"], kernel_size=t["conv_kernel_size"],
                dropout=t[f"{side}_dropout"])


class Encoder(nn.Module):
    """``transformer/Models.py:33-112`` (training branch)."""

    def __init__(self, config):
        super().__init__()
        c = _stack_cfg(config, "encoder")
        self.max_seq_len = config["max_seq_len"]
        self.src_word_emb = nn.Embedding(429, c["d_model"], padding_idx=0)
        self.src_accent_emb = nn.Embedding(5, c["d_model"], padding_idx=0)
        self.position_enc = nn.Parameter(
            sinusoid_table(config["max_seq_len"] + 1, c["d_model"])[None], requires_grad=False)
        self.layer_stack = nn.ModuleList(
            FFTBlock(c["d_model"], c["n_head"], c["d_inner"], c["kernel_size"], c["dropout"])
            for _ in range(config["transformer"]["encoder_layer"]))

    def forward(self, texts, pad, accents):
        T = texts.shape[1]
        x = self.src_word_emb(texts) + self.src_accent_emb(accents) + self.position_enc[:, :T]
        for layer in self.layer_stack:
            x = layer(x, pad)
        return x


class Decoder(nn.Module):
    """``transformer/Models.py:115-183`` (truncate to max_seq_len, except in eval mode)."""

    def __init__(self, config):
        super().__init__()
        c = _stack_cfg(config, "decoder")
        self.max_seq_len = config["max_seq_len"]
        self.position_enc = nn.Parameter(
            sinusoid_table(config["max_seq_len"] + 1, c["d_model"])[None], requires_grad=False)
        self.layer_stack = nn.ModuleList(
            FFTBlock(c["d_model"], c["n_head"], c["d_inner"], c["kernel_size"], c["dropout"])
            for _ in range(config["transformer"]["decoder_layer"]))

    def forward(self, x, pad):
        if not self.training and x.shape[1] > self.max_seq_len:
            # Models.py:160-165: eval past max_seq_len, fresh table, no truncation
            T = x.shape[1]
            x = x + sinusoid_table(T, x.shape[2])[None, :T]
            for layer in self.layer_stack:
                x = layer(x, pad)
            return x, pad
        T = min(x.shape[1], self.max_seq_len)
        x = x[:, :T] + self.position_enc[:, :T]
        pad = pad[:, :T]
        for layer in self.layer_stack:
            x = layer(x, pad)
        return x, pad


# ---------------------------------------------------------------------------------------
# Variance adaptor (model/modules.py:17-296)
# ---------------------------------------------------------------------------------------


class _Conv(nn.Module):
    """``model/modules.py:253-296``: Conv1d over the time axis of a (B, T, C) tensor."""

    def __init__(self, c_in, c_out, k, padding):
        super().__init__()
        self.conv = nn.Conv1d(c_in, c_out, k, padding=padding)

    def forward(self, x):
        return self.conv(x.transpose(1, 2)).transpose(1, 2)


class VariancePredictor(nn.Module):
    """``model/modules.py:197-250``.  Padded rows are *not* zeroed between the convs."""

    def __init__(self, config):
        super().__init__()
        d = config["transformer"]["encoder_hidden"]
        f = config["variance_predictor"]["filter_size"]
        k = config["variance_predictor"]["kernel_size"]
        self.p = config["variance_predictor"]["dropout"]
        self.conv_layer = nn.Module()
        self.conv_layer.conv1d_1 = _Conv(d, f, k, (k - 1) // 2)
        self.conv_layer.layer_norm_1 = nn.LayerNorm(f)
        self.conv_layer.conv1d_2 = _Conv(f, f, k, 1)  # padding hard-coded to 1 (modules.py:230)
        self.conv_layer.layer_norm_2 = nn.LayerNorm(f)
        self.linear_layer = nn.Linear(f, 1)

    def forward(self, x, pad):
        c = self.conv_layer
        y = _drop(c.layer_norm_1(F.relu(c.conv1d_1(x))), self.p, self.training)
        y = _drop(c.layer_norm_2(F.relu(c.conv1d_2(y))), self.p, self.training)
        y = self.linear_layer(y).squeeze(-1)
        return y.masked_fill(pad, 0.0)


def length_regulate(x, durations, max_len):
    """``model/modules.py:161-194`` + ``utils/tools.py:363-381``: repeat phoneme row i
    ``max(int(d_i), 0)`` times (``int`` truncates toward zero), pad or crop to ``max_len``;
    ``mel_len`` is the uncropped length."""
    reps = torch.clamp(durations.to(torch.float64).trunc(), min=0).long()
    rows, lens = [], []
    for b in range(x.shape[0]):
        e = torch.repeat_interleave(x[b], reps[b], dim=0)
        rows.append(e)
        lens.append(e.shape[0])
    T = max_len if max_len is not None else max(lens)
    out = torch.stack([F.pad(e, (0, 0, 0, T - e.shape[0])) for e in rows])
    return out, torch.tensor(lens, dtype=torch.long)


class VarianceAdaptor(nn.Module):
    def __init__(self, preprocess_config, model_config, pitch_range, energy_range):
        super().__init__()
        n_bins = model_config["variance_embedding"]["n_bins"]
        d = model_config["transformer"]["encoder_hidden"]
        self.duration_predictor = VariancePredictor(model_config)
        self.pitch_predictor = VariancePredictor(model_config)
        self.energy_predictor = VariancePredictor(model_config)
        # modules.py:56-71 — linear quantisation bins from stats.json min/max
        self.pitch_bins = nn.Parameter(torch.linspace(*pitch_range, n_bins - 1),
                                       requires_grad=False)
        self.energy_bins = nn.Parameter(torch.linspace(*energy_range, n_bins - 1),
                                        requires_grad=False)
        self.pitch_embedding = nn.Embedding(n_bins, d)
        self.energy_embedding = nn.Embedding(n_bins, d)

    def forward(self, x, src_pad, mel_pad, max_len, p_t, e_t, d_t, p_c=1.0, e_c=1.0, d_c=1.0):
        # modules.py:102-158 (phoneme-level pitch and energy)
        log_d = self.duration_predictor(x, src_pad)
        p = self.pitch_predictor(x, src_pad)
        if p_t is not None:
            x = x + self.pitch_embedding(torch.bucketize(p_t, self.pitch_bins))
        else:
            p = p * p_c
            x = x + self.pitch_embedding(torch.bucketize(p, self.pitch_bins))
        e = self.energy_predictor(x, src_pad)
        if e_t is not None:
            x = x + self.energy_embedding(torch.bucketize(e_t, self.energy_bins))
        else:
            e = e * p_c  # the reference passes p_control to the energy branch (modules.py:124)
            x = x + self.energy_embedding(torch.bucketize(e, self.energy_bins))
        if d_t is not None:
            x, mel_len = length_regulate(x, d_t, max_len)
            d_r = d_t
        else:
            d_r = torch.clamp(torch.round(torch.exp(log_d) - 1) * d_c, min=0)
            x, mel_len = length_regulate(x, d_r, max_len)
            mel_pad = mask_from_lengths(mel_len)
        return x, p, e, log_d, d_r, mel_len, mel_pad


# ---------------------------------------------------------------------------------------
# PostNet (transformer/Layers.py:33-137)
# ---------------------------------------------------------------------------------------


class _ConvNorm(nn.Module):
    def __init__(self, c_in, c_out, k):
        super().__init__()
        self.conv = nn.Conv1d(c_in, c_out, k, padding=(k - 1) // 2)


class PostNet(nn.Module):
    def __init__(self, n_mel=80, dim=512, k=5, n=5):
        super().__init__()
        chans = [n_mel] + [dim] * (n - 1) + [n_mel]
        self.convolutions = nn.ModuleList(
            nn.Sequential(_ConvNorm(chans[i], chans[i + 1], k), nn.BatchNorm1d(chans[i + 1]))
            for i in range(n))

    def forward(self, x):
        y = x.transpose(1, 2)
        last = len(self.convolutions) - 1
        for i, layer in enumerate(self.convolutions):
            y = layer[1](layer[0].conv(y))
            if i < last:
                y = torch.tanh(y)
            y = _drop(y, 0.5, self.training)  # hard-coded F.dropout(0.5) (Layers.py:133-134)
        return y.transpose(1, 2)


# ---------------------------------------------------------------------------------------
# TacoSpawn GMM head and top level (model/fastspeech2.py:15-174, 306-341)
# ---------------------------------------------------------------------------------------


class GMMParams:
    """The mixture the reference wraps as ``MixtureSameFamily(Categorical(pi),
    Independent(Normal(mu, sigma), 1))``; ``log_prob`` follows torch.distributions."""

    def __init__(self, pi, mu, sigma):
        self.pi, self.mu, self.sigma = pi, mu, sigma

    def log_prob(self, e):
        probs = self.pi / self.pi.sum(-1, keepdim=True)
        eps = torch.finfo(probs.dtype).eps
        logits = torch.log(probs.clamp(min=eps, max=1 - eps))
        log_mix = torch.log_softmax(logits, dim=-1)
        x = e[:, None, :]
        comp = (-((x - self.mu) ** 2) / (2 * self.sigma ** 2) - torch.log(self.sigma)
                - math.log(math.sqrt(2 * math.pi))).sum(-1)
        return torch.logsumexp(comp + log_mix, dim=-1)


class SpeakerMetaEncoder(nn.Module):
    def __init__(self, in_dim, K, D):
        super().__init__()
        self.K, self.D = K, D
        self.pi_linear = nn.Sequential(nn.Linear(in_dim, K), nn.Softmax(dim=1))
        self.sigma_linear = nn.Sequential(nn.Linear(in_dim, K * D), nn.Softplus())
        self.mu_linear = nn.Linear(in_dim, K * D)

    def forward(self, m):
        return GMMParams(self.pi_linear(m).view(-1, self.K),
                         self.mu_linear(m).view(-1, self.K, self.D),
                         self.sigma_linear(m).view(-1, self.K, self.D))


class FastSpeech2(nn.Module):
    def __init__(self, preprocess_config, model_config, n_speaker, pitch_range, energy_range):
        super().__init__()
        d = model_config["transformer"]["encoder_hidden"]
        self.encoder = Encoder(model_config)
        self.variance_adaptor = VarianceAdaptor(preprocess_config, model_config, pitch_range,
                                                energy_range)
        self.decoder = Decoder(model_config)
        self.mel_linear = nn.Linear(model_config["transformer"]["decoder_hidden"],
                                    preprocess_config["mel"]["n_mel_channels"])
        self.postnet = PostNet()
        meta = preprocess_config["speaker_generation"]["metadata"]
        self.speaker_emb = nn.Embedding(n_speaker, d)
        self.speaker_enc = SpeakerMetaEncoder(sum(len(v) for v in meta.values()),
                                              model_config["speaker_generation"]["GMM_mixtures"], d)

    def forward(self, speakers, texts, src_lens, max_src_len, mels=None, mel_lens=None,
                max_mel_len=None, p_targets=None, e_targets=None, d_targets=None,
                p_control=1.0, e_control=1.0, d_control=1.0, accents=None, speaker_meta=None):
        src_pad = mask_from_lengths(src_lens, max_src_len)
        mel_pad = mask_from_lengths(mel_lens, max_mel_len) if mel_lens is not None else None
        x = self.encoder(texts, src_pad, accents)
        spk = self.speaker_emb(speakers)
        x = x + spk[:, None, :]
        gmm = self.speaker_enc(speaker_meta)
        x, p, e, log_d, d_r, mel_lens, mel_pad = self.variance_adaptor(
            x, src_pad, mel_pad, max_mel_len, p_targets, e_targets, d_targets,
            p_control, e_control, d_control)
        x, mel_pad = self.decoder(x, mel_pad)
        out = self.mel_linear(x)
        post = self.postnet(out) + out
        return (out, post, p, e, log_d, d_r, src_pad, mel_pad, src_lens, mel_lens, gmm, spk)

    def synthesize_from_speaker_emb(self, speakers, texts, src_lens, max_src_len, mels=None,
                                    mel_lens=None, max_mel_len=None, p_targets=None,
                                    e_targets=None, d_targets=None, p_control=1.0, e_control=1.0,
                                    d_control=1.0, accents=None, speaker_emb=None):
        # model/fastspeech2.py:186-303 (multi_speaker, no JDIT): 10-tuple
        src_pad = mask_from_lengths(src_lens, max_src_len)
        mel_pad = mask_from_lengths(mel_lens, max_mel_len) if mel_lens is not None else None
        x = self.encoder(texts, src_pad, accents)
        x = x + speaker_emb.unsqueeze(1).expand(-1, max_src_len, -1)
        x, p, e, log_d, d_r, mel_lens, mel_pad = self.variance_adaptor(
            x, src_pad, mel_pad, max_mel_len, p_targets, e_targets, d_targets,
            p_control, e_control, d_control)
        x, mel_pad = self.decoder(x, mel_pad)
        out = self.mel_linear(x)
        post = self.postnet(out) + out
        return (out, post, p, e, log_d, d_r, src_pad, mel_pad, src_lens, mel_lens)


# ---------------------------------------------------------------------------------------
# Losses, optimiser, step (model/loss.py, model/optimizer.py, train.py:138-206)
# ---------------------------------------------------------------------------------------


def fs2_loss(inputs, predictions):
    """``model/loss.py:19-92``: masked L1 on mels, masked MSE on phoneme-level variances."""
    mels, _, _, p_t, e_t, d_t = inputs[6:12]
    out, post, p, e, log_d, _, src_pad, mel_pad = predictions[:8]
    sv, mv = ~src_pad, ~mel_pad
    log_d_t = torch.log(d_t.float() + 1)
    mels = mels[:, : mv.shape[1]]
    mel_loss = F.l1_loss(out.masked_select(mv[..., None]), mels.masked_select(mv[..., None]))
    post_loss = F.l1_loss(post.masked_select(mv[..., None]), mels.masked_select(mv[..., None]))
    p_loss = F.mse_loss(p.masked_select(sv), p_t.masked_select(sv))
    e_loss = F.mse_loss(e.masked_select(sv), e_t.masked_select(sv))
    d_loss = F.mse_loss(log_d.masked_select(sv), log_d_t.masked_select(sv))
    total = mel_loss + post_loss + d_loss + p_loss + e_loss
    return total, mel_loss, post_loss, p_loss, e_loss, d_loss


def speaker_enc_loss(emb, gmm):
    """``model/loss.py:102-104``: mean log-likelihood of the detached speaker embedding."""
    lp = gmm.log_prob(emb.detach())
    return sum(lp) / lp.size()[0]


def lr_at(step, d_model=256, warmup=4000, anneal_steps=(300000, 400000, 500000),
          anneal_rate=0.3):
    """``model/optimizer.py:33-51`` for the 1-based step the update is taken at."""
    lr = min(step ** -0.5, warmup ** -1.5 * step)
    for s in anneal_steps:
        if step > s:
            lr *= anneal_rate
    return float(np.power(d_model, -0.5)) * lr


def build(config_name_or_dir, seeded=True):
    """Oracle model from a bundled config, name-seeded weights loaded."""
    import importlib
    pkg = importlib.import_module("mid-attribute-speaker-generation_amd")
    pp, mc, tc, path = pkg.config.load_configs(config_name_or_dir)
    pr = pkg.config.pitch_energy_range(path)
    m = FastSpeech2(pp, mc, pkg.config.n_speakers(path), pr[:2], pr[2:])
    if seeded:
        pkg.seeded.load_seeded_(m)
    return m, (pp, mc, tc)


def train_step(model, opt, batch, clip=1.0):
    """One optimiser step exactly as ``train.py:138-206`` (``use_clf`` off, grad_acc 1)."""
    out = model(*batch[2:12], accents=batch[13], speaker_meta=batch[12])
    losses = fs2_loss(batch[:12], out[:-2])
    losses[0].backward()
    eloss = speaker_enc_loss(out[-1], out[-2])
    (-eloss).backward()
    gn = torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
    opt["step"] += 1
    for g in opt["adam"].param_groups:
        g["lr"] = lr_at(opt["step"])
    opt["adam"].step()
    opt["adam"].zero_grad()
    return [float(l) for l in losses], float(eloss), float(gn), out


def make_opt(model, betas=(0.9, 0.98), eps=1e-9):
    return {"adam": torch.optim.Adam(model.parameters(), betas=betas, eps=eps, weight_decay=0.0),
            "step": 0}
