"""HiFi-GAN generator (V1/"universal" configuration) on the HIP path.

Drop-in for ``hifigan.Generator`` after ``remove_weight_norm()`` as ``utils/model.py:57-69``
uses it, and for ``vocoder_infer`` (``utils/model.py:74-90``):

* the same state-dict keys and shapes as the reference generator after weight-norm removal
  (``conv_pre``, ``ups.{i}`` ConvTranspose1d (c_in, c_out, k), ``resblocks.{n}.convs{1,2}.{m}``,
  ``conv_post``); ``load_state_dict`` also takes the checkpoint form with ``weight_g`` /
  ``weight_v`` (``torch.nn.utils.weight_norm``, dim 0) and folds it;
* ``forward(mels)`` with mels ``(B, 80, T)`` returns ``(B, 1, 256 T)`` as
  ``hifigan/models.py:155-171``; ``forward_rows(mel_rows, B, T)`` takes the FastSpeech2
  output in its native ``(B*T, 80)`` row layout (no transpose, used by ``synthesize``).

Every convolution is one ``fs2_conv_gemm_ex`` launch (bf16 MFMA implicit GEMM; fp32 mode for
parity) with the surrounding elementwise work fused into its epilogue:

* ``leaky_relu(x, 0.1)`` before each conv (``models.py:95,157``) is the second output (Y2)
  of the conv that produced ``x``; the one after ``c1`` (``models.py:97``) is its LRELU
  epilogue;
* the residual ``x = xt + x`` (``models.py:99``) is ADD_AUX of ``c2``, and the
  multi-receptive-field average ``(rb0 + rb1 + rb2) / 3`` (``models.py:160-166``) is ACC_Y of
  the last ``c2`` of each resblock into one running buffer (scale 1/3 on the third);
* ConvTranspose1d(k=2s, stride s, pad s/2) runs as a 3-tap conv producing the s output
  phases of each input frame as s*c_out columns -- its row-major output IS the upsampled
  ``(frames*s, c_out)`` activation (``fs2_convT_weight_prep``);
* ``conv_post`` + ``tanh`` (+ the int16 PCM of ``vocoder_infer``) is ``fs2_vocoder_post``.
"""
import json
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import kernels as K
from .config import CONFIG_ROOT

LRELU_SLOPE = 0.1  # hifigan/models.py:7


class AttrDict(dict):
    """``hifigan/__init__.py`` AttrDict: keys as attributes."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.__dict__ = self


def load_config(path=None):
    with open(path or os.path.join(CONFIG_ROOT, "hifigan.json")) as f:
        return AttrDict(json.load(f))


def get_padding(kernel_size, dilation=1):
    return int((kernel_size * dilation - dilation) / 2)  # hifigan/models.py:16-17


def _fold_weight_norm(sd):
    """``weight = g * v / ||v||`` (norm over every dim but 0), for ``*.weight_g/_v`` pairs."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".weight_v"):
            base = k[: -len("_v")]
            g = sd[base + "_g"]
            n = v.reshape(v.shape[0], -1).norm(dim=1).reshape(g.shape)
            out[base] = v * (g / n)
        elif not k.endswith(".weight_g"):
            out[k] = v
    return out


class Generator(nn.Module):
    """``hifigan/models.py:104-178`` (inference; weights are fp32 masters, never trained)."""

    def __init__(self, h, device="cuda", compute_dtype=torch.bfloat16):
        super().__init__()
        self.h = h
        self.num_kernels = len(h.resblock_kernel_sizes)
        self.num_upsamples = len(h.upsample_rates)
        self.compute_dtype = compute_dtype
        self.fused_resblocks = True  # bf16: narrow-stage resblocks as one fused launch each
        dev = torch.device(device)
        P = lambda *shape: nn.Parameter(torch.zeros(*shape, device=dev), requires_grad=False)
        ch0 = h.upsample_initial_channel
        self.conv_pre = nn.Module()
        self.conv_pre.weight, self.conv_pre.bias = P(ch0, 80, 7), P(ch0)  # models.py:113-115
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(h.upsample_rates, h.upsample_kernel_sizes)):
            if k != 2 * u or (k - u) // 2 != u // 2:
                raise ValueError(f"upsample {i}: kernel {k} / stride {u} is not k = 2s, pad s/2")
            m = nn.Module()
            m.weight, m.bias = P(ch0 // 2 ** i, ch0 // 2 ** (i + 1), k), P(ch0 // 2 ** (i + 1))
            self.ups.append(m)
        self.resblocks = nn.ModuleList()
        for i in range(self.num_upsamples):
            ch = ch0 // 2 ** (i + 1)
            for k, d in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes):
                rb = nn.Module()
                rb.kernel_size, rb.dilation = k, tuple(d)
                for name in ("convs1", "convs2"):
                    convs = nn.ModuleList()
                    for _ in range(3):
                        c = nn.Module()
                        c.weight, c.bias = P(ch, ch, k), P(ch)
                        convs.append(c)
                    setattr(rb, name, convs)
                self.resblocks.append(rb)
        self.conv_post = nn.Module()
        self.conv_post.weight, self.conv_post.bias = P(1, ch, 7), P(1)
        self._prepared = None

    # ---------------------------------------------------------------- weights
    def load_state_dict(self, state_dict, strict=True):
        sd = _fold_weight_norm(dict(state_dict))
        r = super().load_state_dict(sd, strict=strict)
        self._prepared = None
        return r

    def remove_weight_norm(self):
        """Weights are stored folded already (``models.py:172-178`` prints and folds)."""
        print("Removing weight norm...")

    def _prep(self):
        """Compute-layout weights (once per weight load): conv weights as
        ``w_fwd[o, j*c_in + c]`` in the compute dtype, transposed convs via their 3-tap
        phase form."""
        if self._prepared is not None:
            return self._prepared
        cdt = self.compute_dtype

        def conv(w):
            c_out, c_in, k = w.shape
            wf = torch.empty(c_out * c_in * k, dtype=cdt, device=w.device)
            K.weight_prep(w.contiguous(), c_out, c_in, k, w_fwd=wf)
            return wf

        prep = {"pre": conv(self.conv_pre.weight), "ups": [], "rb": []}
        for i, m in enumerate(self.ups):
            wc, bc = K.convT_weight_prep(m.weight.contiguous(), m.bias, self.h.upsample_rates[i])
            prep["ups"].append((conv(wc), bc))
        for rb in self.resblocks:
            prep["rb"].append(([conv(c.weight) for c in rb.convs1], [conv(c.weight) for c in rb.convs2]))
        prep["post_w"] = self.conv_post.weight.reshape(-1).contiguous()
        self._prepared = prep
        return prep

    # ---------------------------------------------------------------- forward
    def forward(self, x):
        """mels (B, 80, T) -> waveform (B, 1, T * prod(upsample_rates)) in [-1, 1]."""
        B, C, T = x.shape
        rows = x.transpose(1, 2).contiguous().reshape(B * T, C)  # API adapter: (B,C,T) -> rows
        wav, _ = self.forward_rows(rows, B, T, pcm=False)
        return wav.view(B, 1, -1)

    def receptive_frames(self):
        """Receptive radius of one output sample, in mel frames (rounded up): conv_pre, each
        upsample's 3-tap phase conv, each stage's widest resblock chain and conv_post, every
        radius divided by the rows per frame at its resolution."""
        h, res = self.h, 1
        r = 3.0  # conv_pre k=7
        for i, s in enumerate(h.upsample_rates):
            r += 1.0 / res  # phase conv (taps 3, pad 1) at the input resolution
            res *= s
            r += max(sum((k - 1) // 2 * d + (k - 1) // 2 for d in dil)
                     for k, dil in zip(h.resblock_kernel_sizes, h.resblock_dilation_sizes)) / res
        r += 3.0 / res  # conv_post k=7
        return int(math.ceil(r))

    def _stage_lens(self, lengths, B, T, dev):
        """Per-resolution row limits for length-aware launches: min(T, len + R) frames times
        the rows per frame (R = receptive_frames), so every kept sample is computed from
        exactly the rows the padded-batch pass uses; the last entry (samples) is len * up."""
        R = self.receptive_frames()
        if torch.is_tensor(lengths):  # device lengths (the model's mel_len): no host sync
            if lengths.numel() != B:
                raise ValueError(f"lengths must hold {B} frame counts")
            l = lengths.to(device=dev, dtype=torch.int64).reshape(B)
            ext = torch.clamp(l + R, max=T)
            res, out = 1, []
            for s in [1] + list(self.h.upsample_rates):
                res *= s
                out.append((ext * res).contiguous())
            out.append((torch.clamp(l, 0, T) * res).contiguous())
            return out
        lens = [int(l) for l in lengths]
        if len(lens) != B or min(lens) < 0 or max(lens) > T:
            raise ValueError(f"lengths must be {B} frame counts in [0, {T}]")
        res, table = 1, []
        for s in [1] + list(self.h.upsample_rates):
            res *= s
            table.append([min(T, l + R) * res for l in lens])
        table.append([l * res for l in lens])
        t = torch.tensor(table, dtype=torch.int64).to(dev, non_blocking=True)
        return [t[i] for i in range(len(table))]

    @torch.no_grad()
    def forward_rows(self, mel_rows, B, T, pcm=True, max_wav_value=32768.0, lengths=None):
        """mel_rows (B*T, 80) fp32 (the FastSpeech2 row layout) -> (wav (B*T*up,) fp32,
        pcm int16 or None).  ``lengths`` (mel frames per utterance, optional; a list or a
        device tensor such as the model's mel_len): row tiles past
        length + receptive radius are not computed and samples past length * up are 0; the
        samples before it are bitwise those of the full padded pass."""
        prep = self._prep()
        cdt, dev = self.compute_dtype, mel_rows.device
        sl = self._stage_lens(lengths, B, T, dev) if lengths is not None else None
        L = (lambda i: sl[i]) if sl is not None else (lambda i: None)
        # skipped tiles store nothing: rows past length + radius are never read for a kept
        # sample (a GEMM output row depends only on the input rows within its taps)
        NS = K.EPI_SKIP_NOSTORE if sl is not None else 0
        x_c = mel_rows.contiguous()
        if x_c.dtype != cdt:
            x_c = K.cast_bf16(x_c.float()) if cdt == torch.bfloat16 else x_c.float()
        rows, seq = B * T, T
        ch = self.h.upsample_initial_channel
        # conv_pre: only its leaky-ReLU'd copy is consumed (models.py:156-157)
        h_c = torch.empty(rows, ch, dtype=cdt, device=dev)
        K.conv_gemm_ex(x_c, prep["pre"], rows, seq, x_c.shape[1], ch, 7, 3,
                       bias=self.conv_pre.bias, y2=h_c, alpha2=LRELU_SLOPE, lens=L(0), flags=NS)
        nk = self.num_kernels
        for i in range(self.num_upsamples):
            s = self.h.upsample_rates[i]
            c_in, c_out = ch // 2 ** i, ch // 2 ** (i + 1)
            wk, bc = prep["ups"][i]
            # narrow stages (32 / 64 channels, bf16): each resblock is one fused launch on an
            # LDS-resident tile (fs2_resblock1_fused), which takes x and applies its own
            # leaky ReLU -- no bf16 copy of x needed
            fused = (self.fused_resblocks and cdt == torch.bfloat16 and all(
                K.resblock1_supported(c_out, seq * s, rb.kernel_size, rb.dilation)
                for rb in self.resblocks[i * nk:(i + 1) * nk]))
            x = torch.empty(rows * s, c_out, dtype=torch.float32, device=dev)
            xl = None if fused else torch.empty(rows * s, c_out, dtype=cdt, device=dev)
            # ConvTranspose1d as the 3-tap phase conv: (rows, s*c_out) == (rows*s, c_out)
            K.conv_gemm_ex(h_c, wk, rows, seq, c_in, s * c_out, 3, 1, bias=bc,
                           out=x.view(rows, s * c_out),
                           y2=None if fused else xl.view(rows, s * c_out),
                           alpha2=LRELU_SLOPE, lens=L(i), flags=NS)
            rows, seq = rows * s, seq * s
            xs = torch.empty(rows, c_out, dtype=torch.float32, device=dev)
            last_stage = i == self.num_upsamples - 1
            h_c = torch.empty(rows, c_out, dtype=cdt, device=dev)
            if fused:
                for j in range(nk):
                    rb = self.resblocks[i * nk + j]
                    w1, w2 = prep["rb"][i * nk + j]
                    fin = j == nk - 1
                    K.resblock1_fused(x, rows, seq, c_out, rb.kernel_size, rb.dilation, w1, w2,
                                      [c.bias for c in rb.convs1], [c.bias for c in rb.convs2],
                                      xs, acc=j > 0, scale=1.0 / nk if fin else 1.0,
                                      store_xs=not fin, hc=h_c if fin else None,
                                      alpha2=0.01 if last_stage else LRELU_SLOPE, lens=L(i + 1))
                continue
            for j in range(nk):
                rb = self.resblocks[i * nk + j]
                w1, w2 = prep["rb"][i * nk + j]
                k = rb.kernel_size
                cur, cur_l = x, xl
                for m, d in enumerate(rb.dilation):
                    t_c = torch.empty(rows, c_out, dtype=cdt, device=dev)
                    K.conv_gemm_ex(cur_l, w1[m], rows, seq, c_out, c_out, k, get_padding(k, d),
                                   dilation=d, bias=rb.convs1[m].bias, flags=K.EPI_LRELU | NS,
                                   alpha=LRELU_SLOPE, out=t_c, lens=L(i + 1))
                    if m < 2:
                        nxt = torch.empty(rows, c_out, dtype=torch.float32, device=dev)
                        nxt_l = torch.empty(rows, c_out, dtype=cdt, device=dev)
                        K.conv_gemm_ex(t_c, w2[m], rows, seq, c_out, c_out, k, get_padding(k, 1),
                                       bias=rb.convs2[m].bias, flags=K.EPI_ADD_AUX | NS, aux=cur,
                                       out=nxt, y2=nxt_l, alpha2=LRELU_SLOPE, lens=L(i + 1))
                        cur, cur_l = nxt, nxt_l
                    else:
                        # xs (+)= this resblock's output; the third also averages and emits the
                        # leaky-ReLU'd input of the next upsample / of conv_post (slope 0.01,
                        # F.leaky_relu's default, models.py:167)
                        flags = K.EPI_ADD_AUX | (K.EPI_ACC_Y if j > 0 else 0) | NS
                        fin = j == nk - 1
                        K.conv_gemm_ex(t_c, w2[m], rows, seq, c_out, c_out, k, get_padding(k, 1),
                                       bias=rb.convs2[m].bias, flags=flags, aux=cur, out=xs,
                                       y2=h_c if fin else None,
                                       scale=1.0 / nk if fin else 1.0,
                                       alpha2=0.01 if last_stage else LRELU_SLOPE,
                                       lens=L(i + 1))
        c_last = ch // 2 ** self.num_upsamples
        return K.vocoder_post(h_c, rows, seq, c_last, prep["post_w"], self.conv_post.bias,
                              max_wav_value, pcm=pcm, lens=L(self.num_upsamples + 1))


def get_vocoder(config=None, device="cuda", ckpt=None, compute_dtype=torch.bfloat16):
    """``utils/model.py:57-69`` for HiFi-GAN: bundled config; the checkpoint's
    ``"generator"`` state dict when given (else name-seeded weights: the reference's
    ``generator_*.pth.tar`` blobs are not shipped)."""
    from .seeded import load_seeded_
    h = load_config(config)
    g = Generator(h, device=device, compute_dtype=compute_dtype)
    if ckpt is not None:
        sd = torch.load(ckpt, map_location=device, weights_only=True)
        g.load_state_dict(sd["generator"] if "generator" in sd else sd)
    else:
        load_seeded_(g)
    g.eval()
    return g


def vocoder_infer(mels, vocoder, model_config, preprocess_config, lengths=None):
    """``utils/model.py:74-90`` (HiFi-GAN branch): mels (B, 80, T) -> list of int16 arrays,
    each cropped to ``lengths[i]`` samples when given."""
    B, C, T = mels.shape
    rows = mels.transpose(1, 2).contiguous().reshape(B * T, C)
    max_wav = preprocess_config["audio"]["max_wav_value"]  # utils/model.py:84-86
    # with lengths, only the frames that reach a kept sample are computed (length-aware
    # launches; the kept samples are identical to the padded pass)
    up = math.prod(vocoder.h.upsample_rates)
    frames = None if lengths is None else [min(T, -(-int(l) // up)) for l in lengths]
    _, pcm = vocoder.forward_rows(rows, B, T, pcm=True, max_wav_value=float(max_wav),
                                  lengths=frames)
    wavs = list(pcm.view(B, -1).cpu().numpy())
    if lengths is not None:
        wavs = [w[: lengths[i]] for i, w in enumerate(wavs)]
    return wavs
