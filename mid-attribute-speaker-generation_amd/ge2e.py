"""The ``--use_clf`` language discriminator on the HIP path.

Mirrors ``Multilingual-Speaker-Encoder-with-Domain-Adaptation/speech_embedder_net.py``:

* ``SpeechEmbedder()`` -- 3-layer ``nn.LSTM(80, 256, batch_first)`` (``LSTM_stack``), last
  frame, ``projection`` (LinearNorm 256 -> 64), L2 normalisation, and the domain classifier
  ``da_classifier.classifier`` (MultiLayerNN 64 -> [64, 64, 1], dropout 0.2, ReLU); same
  state-dict keys and shapes; ``forward(x)`` returns ``{'embeddings', 'da_lang_logits'}``
  (``speech_embedder_net.py:126-146``, config/config.yaml: hidden 256, 3 layers, proj 64,
  da on language).
* ``GE2ELoss(device)`` -- ``forward(embeddings, lang_logits, langs, **kw)`` returns
  ``(loss + da_loss, loss, da_loss)`` with ``da_loss = BCEWithLogitsLoss(reduction='sum')``
  (``speech_embedder_net.py:165-186``).  ``train.py:190`` only back-propagates ``da_loss``;
  the GE2E similarity term there has M = 1 utterance per "speaker", for which the
  reference's exclude-self centroid divides by M - 1 = 0 (``utils.py:36``) -- it is NaN and
  returned as NaN here as well (M > 1, the speaker-encoder pre-training loss, is outside
  the hot path and raises).

Kernels (``csrc/lstm.hip``): the 3-layer stack runs as a wavefront -- launch s computes
layer l at step s - l, all layers in one launch (T + 2 launches instead of 3T), with the
inputs of layers 1-2 folded into their step kernels; layer 0's input projection is one GEMM.
The backward is the same in reverse plus one GEMM for the input gradient.  The head (projection .. logit) is one kernel,
one wave per sequence, forward and backward.  The discriminator's own weight gradients are
not formed: ``train.py`` never steps it (its parameters are set ``requires_grad`` but no
optimiser holds them), so only the gradient into FastSpeech2's mel output is computed.
"""
import math

import torch
import torch.nn as nn

from . import kernels as K
from ._lib import lib

HIDDEN, LAYERS, PROJ, NMELS, CHUNK = 256, 3, 64, 80, 150  # config/config.yaml
DA_DROPOUT = 0.2  # module.py:24 via speech_embedder_net.py:152


def _p(t):
    return t.data_ptr()


class _EmbedderFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, emb_mod, seed):
        N, T, D = x.shape
        dev = x.device
        w = emb_mod._prep()
        st, rows = w["stack"], N * T
        gx = torch.empty(rows, 4 * HIDDEN, device=dev)
        h = torch.empty(LAYERS, rows, HIDDEN, device=dev)
        c = torch.empty(LAYERS, rows, HIDDEN, device=dev)
        act = torch.empty(LAYERS, rows, 4 * HIDDEN, device=dev)
        xc = x.contiguous()
        lib.fs2_lstm_stack_fwd(_p(xc), N, T, D, HIDDEN, LAYERS, _p(st["w_ih0"]),
                               _p(st["w_ih_up"]), _p(st["w_hh"]), _p(st["bias"]), _p(gx), _p(h),
                               _p(c), _p(act), K.stream())
        del gx
        saved, inp = (c, act), h[LAYERS - 1]
        emb = torch.empty(N, PROJ, device=dev)
        logit = torch.empty(N, device=dev)
        hd = w["head"]
        p = emb_mod.da_dropout if emb_mod.training else 0.0
        last = _p(inp) + (T - 1) * HIDDEN * 4  # h[n*T + T-1], row stride T*H
        lib.fs2_clf_head(last, T * HIDDEN, N, *hd, p, _p(seed) if p > 0 else None,
                         emb_mod.site, _p(emb), _p(logit), None, None, None, 0, K.stream())
        fctx.emb_mod, fctx.saved, fctx.h_top, fctx.seed = emb_mod, saved, inp, seed
        fctx.shape, fctx.p = (N, T, D), p
        return emb, logit

    @staticmethod
    def backward(fctx, demb, dlogit):
        N, T, D = fctx.shape
        dev = fctx.h_top.device
        w = fctx.emb_mod._prep()
        dh = K.zeros((N * T, HIDDEN), dev)
        last_in = _p(fctx.h_top) + (T - 1) * HIDDEN * 4
        last_out = _p(dh) + (T - 1) * HIDDEN * 4
        demb = demb.contiguous() if demb is not None else None
        dlogit = dlogit.contiguous() if dlogit is not None else None
        lib.fs2_clf_head(last_in, T * HIDDEN, N, *w["head"], fctx.p,
                         _p(fctx.seed) if fctx.p > 0 else None, fctx.emb_mod.site, None, None,
                         _p(demb) if demb is not None else None,
                         _p(dlogit) if dlogit is not None else None, last_out, T * HIDDEN,
                         K.stream())
        c, act = fctx.saved
        st = w["stack"]
        dgates = torch.empty(LAYERS, N * T, 4 * HIDDEN, device=dev)
        dc = torch.empty(LAYERS * 2 * N * HIDDEN, device=dev)
        dx = torch.empty(N * T, D, device=dev)
        lib.fs2_lstm_stack_bwd(_p(dh), N, T, D, HIDDEN, LAYERS, _p(st["w_ih0_t"]),
                               _p(st["w_ih_up_t"]), _p(st["w_hh_t"]), _p(act), _p(c), _p(dgates),
                               _p(dc), _p(dx), K.stream())
        dh = dx
        return dh.view(N, T, D), None, None


class _Module(nn.Module):
    pass


def _linear_norm(in_dim, out_dim, dev):
    m = _Module()
    m.linear_layer = nn.Linear(in_dim, out_dim, device=dev)
    return m


class SpeechEmbedder(nn.Module):
    """``speech_embedder_net.py:65-146`` (LSTM architecture, language DA head)."""

    def __init__(self, device="cuda"):
        super().__init__()
        dev = torch.device(device)
        self.LSTM_stack = nn.LSTM(NMELS, HIDDEN, num_layers=LAYERS, batch_first=True, device=dev)
        self.projection = _linear_norm(HIDDEN, PROJ, dev)
        self.da_classifier = _Module()
        self.da_classifier.classifier = _Module()
        self.da_classifier.classifier.layer = nn.Sequential()
        for i, o in enumerate((PROJ, PROJ, 1)):
            self.da_classifier.classifier.layer.add_module(f"linear_{i}", _linear_norm(PROJ, o, dev))
        self.da_dropout = DA_DROPOUT
        self.site = 0x5E2E  # dropout stream of the classifier
        self._key = None
        self._seed_state = None
        self.seed(0x6E2E)

    def seed(self, s):
        """Classifier dropout stream: call k draws key splitmix64(s, k) on the device."""
        self._seed_base = int(s) & (2 ** 63 - 1)
        self._seed_state = None

    def _prep(self):
        """Kernel-layout weights: combined LSTM biases, transposes (fs2_conv_weight_prep's
        w_bwd of a taps = 1 weight is its transpose); rebuilt when a weight changes."""
        key = tuple(p._version for p in self.parameters())
        if self._key == key:
            return self._cache
        dev = self.LSTM_stack.weight_ih_l0.device

        def t(w):  # (out, in) -> (in, out)
            o, i = w.shape
            wt = torch.empty(i, o, device=dev)
            K.weight_prep(w.detach().contiguous(), o, i, 1, w_bwd=wt)
            return wt

        lstm = []
        for l in range(LAYERS):
            w_ih = getattr(self.LSTM_stack, f"weight_ih_l{l}").detach().contiguous()
            w_hh = getattr(self.LSTM_stack, f"weight_hh_l{l}").detach().contiguous()
            bias = K.add(getattr(self.LSTM_stack, f"bias_ih_l{l}").detach().contiguous(),
                         getattr(self.LSTM_stack, f"bias_hh_l{l}").detach().contiguous())
            lstm.append({"w_ih": w_ih, "w_ih_t": t(w_ih), "w_hh": w_hh, "w_hh_t": t(w_hh),
                         "bias": bias})
        stack = {
            "w_ih0": lstm[0]["w_ih"], "w_ih0_t": lstm[0]["w_ih_t"],
            "w_ih_up": torch.stack([lstm[l]["w_ih"] for l in range(1, LAYERS)]),
            "w_ih_up_t": torch.stack([lstm[l]["w_ih_t"] for l in range(1, LAYERS)]),
            "w_hh": torch.stack([lstm[l]["w_hh"] for l in range(LAYERS)]),
            "w_hh_t": torch.stack([lstm[l]["w_hh_t"] for l in range(LAYERS)]),
            "bias": torch.stack([lstm[l]["bias"] for l in range(LAYERS)]),
        }
        L = [self.projection.linear_layer] + [
            getattr(self.da_classifier.classifier.layer, f"linear_{i}").linear_layer
            for i in range(3)]
        wts = [l.weight.detach().contiguous() for l in L]
        bs = [l.bias.detach().contiguous() for l in L]
        keep = (wts[0], t(wts[0]), bs[0], wts[1], t(wts[1]), bs[1], wts[2], t(wts[2]), bs[2],
                wts[3], bs[3])
        head = tuple(_p(a) for a in keep)
        self._cache = {"lstm": lstm, "stack": stack, "head": head, "keep": keep}
        self._key = key
        return self._cache

    def forward(self, x, detach=False):
        """x (N, 150, 80) fp32 on the GPU -> {'embeddings': (N, 64), 'da_lang_logits': (N,)}."""
        if self._seed_state is None:
            self._seed_state = torch.tensor([self._seed_base, 0, 0], dtype=torch.int64,
                                            device=x.device)
        if self.training and self.da_dropout > 0:
            K.seed_next(self._seed_state)  # a fresh classifier dropout key per call
        seed = self._seed_state[2:3].clone()  # this call's key (the backward re-reads it)
        emb, logit = _EmbedderFn.apply(x.float(), self, seed)
        if detach:
            emb = emb.detach()
        return {"embeddings": emb, "da_lang_logits": logit}


class _BCESumFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, logit, y):
        n = logit.shape[0]
        rows = torch.empty(n, 1, device=logit.device)
        lib.fs2_bce_logits(_p(logit), _p(y), n, _p(rows), None, 1.0, None, K.stream())
        out = torch.zeros(1, device=logit.device)
        K.colsum(rows, n, 1, out)  # fixed-order sum (reduction='sum')
        fctx.save_for_backward(logit, y)
        return out.view(())

    @staticmethod
    def backward(fctx, g):
        logit, y = fctx.saved_tensors
        d = torch.empty_like(logit)
        lib.fs2_bce_logits(_p(logit), _p(y), logit.shape[0], None, _p(g.contiguous().view(1)),
                           1.0, _p(d), K.stream())
        return d, None


class GE2ELoss(nn.Module):
    """``speech_embedder_net.py:165-186`` (softmax GE2E + BCE domain loss)."""

    def __init__(self, device="cuda"):
        super().__init__()
        self.w = nn.Parameter(torch.tensor(10.0, device=device))
        self.b = nn.Parameter(torch.tensor(-5.0, device=device))

    def forward(self, embeddings, lang_logits, langs, **kwargs):
        N, M, _ = embeddings.shape
        if M != 1:
            raise NotImplementedError("GE2E similarity loss for M > 1 (speaker-encoder "
                                      "pre-training) is outside the hot path")
        loss = torch.full((), float("nan"), device=embeddings.device)  # utils.py:36, M - 1 = 0
        da = _BCESumFn.apply(lang_logits.contiguous(), langs.contiguous().float()) \
            if lang_logits is not None else torch.zeros((), device=embeddings.device)
        return loss + da, loss, da


class _RepadFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, t_dst):
        B, T, C = x.shape
        y = torch.empty(B, t_dst, C, device=x.device)
        lib.fs2_rows_repad(_p(x.contiguous()), B, T, t_dst, C, _p(y), K.stream())
        fctx.shape = (B, T, C, t_dst)
        return y

    @staticmethod
    def backward(fctx, dy):
        B, T, C, t_dst = fctx.shape
        dx = torch.empty(B, T, C, device=dy.device)
        lib.fs2_rows_repad(_p(dy.contiguous()), B, t_dst, T, C, _p(dx), K.stream())
        return dx, None


def chunk_mels(mel, chunk=CHUNK):
    """``train.py:178-183``: (B, T, 80) -> (B * (T // chunk + 1), chunk, 80), zero-padded
    (a full zero chunk when T is a multiple of ``chunk``, as the reference's ``// + 1``)."""
    B, T, C = mel.shape
    r = T // chunk + 1
    return _RepadFn.apply(mel, r * chunk).view(B * r, chunk, C), r


def chunk_langs(speaker_meta, rep, col=2):
    """``train.py:184``: ``speaker_meta[:, 2]`` repeated once per chunk."""
    B, ld = speaker_meta.shape
    y = torch.empty(B * rep, device=speaker_meta.device)
    m = speaker_meta.contiguous().float()
    lib.fs2_repeat_col(_p(m), B, ld, col, rep, _p(y), K.stream())
    return y


def da_coefficient(step, total_step):
    """``train.py:194``: 2 / (1 + exp(-10 p)) - 1 at p = step / total_step."""
    return 2 / (1 + math.exp(-10 * (step / total_step))) - 1
