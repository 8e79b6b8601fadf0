"""Mid-attribute speaker priors: ``model/distributions.py`` on the HIP kernels.

``InterpolateGMM(distri_a, distri_b)`` (distributions.py:12-77) and ``BarycenterGMM(model)``
(79-192) build a new attribute prior from the TacoSpawn GMMs of ``speaker_distribution``;
the result is a ``GMMPrior`` (``sample`` / ``log_prob`` on the device, and the
``mixture_distribution`` / ``component_distribution`` read accessors the reference's
callers use), so ``model.synthesize_from_speaker_emb(..., speaker_emb=g.sample())`` runs
the examples_gen_distri.py flow end to end on the GPU.

Every arithmetic step is a kernel of ``csrc/gmm_ops.hip`` (costs, OT plan, interpolated
components, barycenters, nearest-barycenter weights); the host only builds the metadata
one-hots and reads back the OT solver status and the number of barycenter components.

Reference behaviour kept: the elementwise-diagonal "W2" cost, the variance-as-scale of the
interpolated components, and the transposed weight/component pairing of InterpolateGMM
(see ``oracle/gmm_ops.py``).  Deliberate fix: ``BarycenterGMM.__init__`` raises TypeError
as shipped (it passes ``_print=False`` to ``_barycenter_gaussians``, which has no such
parameter); here the constructor works, with the result the reference gives when that
kwarg is ignored.  ``ot.emd`` (POT, absent here) is replaced by ``fs2_ot_emd``.
"""
import itertools

import numpy as np
import torch

from . import kernels as K
from .loss import GMMPrior


def _rows(g, b=0):
    """(pi (k,), mu (k, d), sd (k, d)) of row ``b`` of a GMMPrior."""
    k = g.pi.shape[-1]
    d = g.mu.shape[-1]
    return (g.pi.reshape(-1, k)[b].contiguous(), g.mu.reshape(-1, k, d)[b].contiguous(),
            g.sigma.reshape(-1, k, d)[b].contiguous())


class InterpolateGMM(GMMPrior):
    """Component-wise interpolation of two speaker GMMs along their optimal-transport plan
    (``distributions.py:12-77``); ``interpolate_rate(t)`` moves along the path, t = 0.5
    initially."""

    def __init__(self, distri_a, distri_b, max_iter=10000):
        self.distri_a = _rows(distri_a)
        self.distri_b = _rows(distri_b)
        pa, ma, sa = self.distri_a
        pb, mb, sb = self.distri_b
        self.t = 0.5
        self.ot_Cost = K.gmm_w2_cost(ma, sa, mb, sb)
        self.ot_Matrix, status = K.ot_emd(pa, pb, self.ot_Cost, max_iter)
        if int(status.item()) < 0:
            raise RuntimeError("fs2_ot_emd: transport simplex did not converge")
        self._build()

    def _build(self):
        pa, ma, sa = self.distri_a
        pb, mb, sb = self.distri_b
        pi, mu, sd = K.gmm_interpolate(self.ot_Matrix, ma, sa, mb, sb, self.t)
        GMMPrior.__init__(self, pi[None], mu[None], sd[None])

    def interpolate_rate(self, t):
        self.t = t
        self._build()


def meta_product(metadata_list):
    """One-hot metadata vectors of every attribute combination, in ``_product`` order
    (``distributions.py:83-84, 102-108``)."""
    pools = [[np.eye(len(v))[i] for i in v.values()] for v in metadata_list.values()]
    return np.stack([np.concatenate(p) for p in itertools.product(*pools)]).astype(np.float32)


class BarycenterGMM(GMMPrior):
    """Wasserstein-barycenter prior of the GMMs of every metadata combination
    (``distributions.py:79-192``): a barycenter per choice of one component from each
    mixture (K^M of them), each original component assigned to its nearest barycenter,
    barycenter weight = sum of rate_i * pi_ij assigned to it.  ``barycenter_rate(rate)``
    reweights the mixtures (``rate`` sums to 1)."""

    ITERS = 60  # fixed-point iterations (distributions.py:154)

    def __init__(self, model, device=None):
        self.metadata_list = model.speaker_enc.metadata_list
        dev = model.encoder.position_enc.device if device is None else torch.device(device)
        self.device = dev
        metas = torch.from_numpy(meta_product(self.metadata_list)).to(dev)
        g = model.speaker_distribution(metas)
        m = metas.shape[0]
        k = g.pi.shape[-1]
        d = g.mu.shape[-1]
        self._pi = g.pi.reshape(m, k).contiguous()
        self._mu = g.mu.reshape(m, k, d).contiguous()
        self._sd = g.sigma.reshape(m, k, d).contiguous()
        self.original_distri = {
            tuple(metas[i].tolist()): {"probs": self._pi[i:i + 1],
                                       "distributes": (self._mu[i:i + 1], self._sd[i:i + 1])}
            for i in range(m)}
        self.rate = [1 / m for _ in range(m)]
        self._update()

    def _update(self):
        m, k, _ = self._mu.shape
        r32 = torch.tensor(self.rate, dtype=torch.float32).to(self.device)
        r64 = torch.tensor(self.rate, dtype=torch.float64).to(self.device)
        self.bary_mean, self.bary_std = K.gmm_barycenter(self._mu, self._sd, r32, self.ITERS)
        n_used, used, pi, mu, sd = K.gmm_bary_mix(self._pi, self._mu, self._sd, r64,
                                                  self.bary_mean, self.bary_std)
        n = int(n_used.item())
        idx = used[:n].tolist()
        self.positions = [tuple(p) for p in
                          (list(itertools.product(range(k), repeat=m))[i] for i in idx)]
        GMMPrior.__init__(self, pi[:n][None], mu[:n][None], sd[:n][None])

    def barycenter_rate(self, rate, _print=True):
        assert hasattr(rate, "__len__") and len(rate) == len(self.original_distri)
        assert sum(rate) == 1
        self.rate = rate
        if _print:
            print("rate: ", rate)
            for i, meta in enumerate(self.original_distri):
                print("distribution " + str(i + 1) + "(rate: " + str(rate[i]) + ")")
                point = 0
                for name, values in self.metadata_list.items():
                    print(" " + name + ":")
                    for v in values:
                        print("     " + v + ": " + str(meta[point]))
                        point += 1
        self._update()
