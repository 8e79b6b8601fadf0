"""Losses of the training step and the TacoSpawn GMM prior object.

Drop-ins for ``model/loss.py``: ``FastSpeech2Loss(preprocess_config, model_config)`` returns
the same 6-tuple (total, mel, postnet, pitch, energy, duration) and ``SpeakerMetaEncLoss``
the same mean log-likelihood; both are single HIP launches (plus a finaliser) with
device-side valid counts, so no ``masked_select`` host sync remains.
"""
import torch
import torch.nn as nn

from . import kernels as K


class FS2LossFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, mel_out, post_out, p, e, log_d, mels, p_t, e_t, d_t, src_pad, mel_pad, denoms,
                g6buf):
        fctx.set_materialize_grads(False)  # unused outputs' gradients stay None (no fills)
        fctx.g6buf = g6buf
        T = mel_out.shape[1]
        args = (mel_out.contiguous(), post_out.contiguous(), mels.contiguous(), p.contiguous(),
                e.contiguous(), log_d.contiguous(), p_t.contiguous().float(),
                e_t.contiguous().float(), d_t.contiguous(), src_pad.contiguous(),
                mel_pad[:, :T].contiguous())
        losses, ws = K.fs2loss_fwd(*args, denoms=denoms)
        fctx.args, fctx.ws = args, ws
        return tuple(losses[i] for i in range(6))

    @staticmethod
    def backward(fctx, *g):
        dev = fctx.ws.device
        buf = fctx.g6buf
        if g[0] is not None and all(x is None for x in g[1:]) and buf is not None:
            # the usual case (only the total loss back-propagated): one copy into a persistent
            # [g, 0, 0, 0, 0, 0] buffer instead of five zero fills and a stack
            buf[0:1].copy_(g[0].reshape(1))
            g6 = buf
        else:
            g6 = torch.stack([x.reshape(()) if x is not None else torch.zeros((), device=dev)
                              for x in g])
        a = fctx.args
        d_mel, d_post, d_p, d_e, d_d = K.fs2loss_bwd(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7],
                                                     a[8], a[9], a[10], fctx.ws, g6.float().contiguous())
        fctx.args = fctx.g6buf = None
        return (d_mel, d_post, d_p, d_e, d_d) + (None,) * 8


class FastSpeech2Loss(nn.Module):
    """``model/loss.py:5-92`` (phoneme-level pitch/energy)."""

    def __init__(self, preprocess_config, model_config):
        super().__init__()
        for key in ("pitch", "energy"):
            assert preprocess_config[key]["feature"] == "phoneme_level", \
                "frame-level variance losses are not built"
        self.denoms = None  # data-parallel: device [mel elements, phonemes] of the global batch
        self._g6 = None  # persistent upstream-gradient vector (entries 1-5 stay zero)

    def forward(self, inputs, predictions):
        mels, _, _, p_t, e_t, d_t = inputs[6:12]
        (mel_out, post_out, p, e, log_d, _, src_masks, mel_masks, _, _) = predictions[:10]
        if self._g6 is None or self._g6.device != mel_out.device:
            self._g6 = torch.zeros(6, dtype=torch.float32, device=mel_out.device)
        return FS2LossFn.apply(mel_out, post_out, p, e, log_d, mels, p_t, e_t, d_t, src_masks,
                               mel_masks, self.denoms, self._g6)


class GMMMeanLogProbFn(torch.autograd.Function):
    """scale * mean_b log p(e_b); backward into the head's weight gradients
    (fastspeech2.py:322-341, loss.py:102-104)."""

    @staticmethod
    def forward(fctx, token, e, gmm, denom):
        e = e.detach().contiguous().float()
        _, resp, mean = K.gmm_logprob(e, gmm.pi, gmm.mu, gmm.sigma, want_mean=True, denom=denom)
        fctx.saved = (e, resp, gmm, denom)
        return mean

    @staticmethod
    def backward(fctx, g):
        e, resp, gmm, denom = fctx.saved
        B = e.shape[0]
        gl = torch.empty(B, dtype=torch.float32, device=e.device)
        # d mean / d logp_b = 1 / (global) batch
        K.lib.fs2_fill_from(K.ptr(gl), B, K.ptr(g.contiguous()), 1.0 if denom is not None else 1.0 / B,
                            K.ptr(denom), K.stream())
        K.gmm_head_bwd(gmm.meta, e, gmm.pi, gmm.mu, gmm.sigma, gmm.sigma_pre, resp, gl,
                       gmm.head.grads())
        hooks = getattr(gmm.head, "_model_hooks", None)
        if hooks is not None and hooks["grad"] is not None:
            hooks["grad"](gmm.head.params())
        fctx.saved = None
        return None, None, None, None


class _Mix:
    def __init__(self, pi):
        self.probs = pi


class _Normal:
    def __init__(self, mu, sigma):
        self.loc = self.mean = mu
        self.scale = self.stddev = sigma

    @property
    def variance(self):
        return self.scale.pow(2)


class _Comp:
    def __init__(self, mu, sigma):
        self.base_dist = _Normal(mu, sigma)


class GMMPrior:
    """The reference's ``MixtureSameFamily(Categorical(pi), Independent(Normal(mu, sigma), 1))``
    (``model/fastspeech2.py:336-341``) as device tensors, with HIP log_prob / sample."""

    def __init__(self, pi, mu, sigma, sigma_pre=None, meta=None, head=None):
        self.pi, self.mu, self.sigma = pi, mu, sigma
        self.sigma_pre, self.meta, self.head = sigma_pre, meta, head

    # torch.distributions-shaped read access used by the reference's callers
    # (model/distributions.py:14-19, 88-90): .mixture_distribution.probs,
    # .component_distribution.base_dist.{loc, scale, mean, stddev, variance}
    @property
    def mixture_distribution(self):
        return _Mix(self.pi)

    @property
    def component_distribution(self):
        return _Comp(self.mu, self.sigma)

    def log_prob(self, e):
        logp, _, _ = K.gmm_logprob(e.detach().contiguous().float(), self.pi, self.mu, self.sigma)
        return logp

    def mean_log_prob(self, e, denom=None):
        """sum_b log p(e_b) / B, or / denom[0] (device; the global batch when data parallel)."""
        token = getattr(self.head, "_tok", None)
        if token is None:
            logp, _, mean = K.gmm_logprob(e.detach().contiguous().float(), self.pi, self.mu,
                                          self.sigma, want_mean=True, denom=denom)
            return mean
        return GMMMeanLogProbFn.apply(token, e, self, denom)

    def sample(self, seed=None, offset=0):
        import numpy as np
        if seed is None:
            seed = int(np.random.default_rng().integers(0, 2 ** 62))
        out, _ = K.gmm_sample(self.pi, self.mu, self.sigma, int(seed), int(offset))
        return out


class SpeakerMetaEncLoss(nn.Module):
    """``model/loss.py:94-105``: sum_b log p(e_b) / B (the caller backprops its negative)."""

    def __init__(self, preprocess_config, model_config):
        super().__init__()
        self.K = model_config["speaker_generation"]["GMM_mixtures"]
        self.denom = None  # data-parallel: device [global batch]

    def forward(self, input, prediction):
        return prediction.mean_log_prob(input, self.denom)
