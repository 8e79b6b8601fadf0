"""ORACLE — TEST INFRASTRUCTURE ONLY.  numpy restatement of the mid-attribute GMM operations
of ``model/distributions.py`` (InterpolateGMM, BarycenterGMM), the checker for
``fs2_gmm_*`` / ``fs2_ot_emd`` (csrc/gmm_ops.hip).  Pinned to fixtures captured from the
reference itself (oracle/make_golden.py -> tests/golden/g7_gmm_ops.npz); see
``tests/test_oracle_golden.py::test_g7_*``.

Third-party algorithm: ``ot.emd`` (POT, not pinned in requirements.txt and absent here) is the
exact optimal-transport plan between the two mixtures' weights.  It is restated as the
linear program min <C, G> s.t. G 1 = a, G^T 1 = b, G >= 0, with b rescaled to a's mass first
(POT's ``emd`` does ``b = b * a.sum() / b.sum()``), solved by scipy's HiGHS; for costs with
a unique optimum every exact solver returns the same vertex.

Reference quirks kept (all verified against the fixtures):
* ``InterpolateGMM._w2sq`` (64-77) multiplies diagonal matrices *elementwise*, so its
  "W2" is ||mu_a - mu_b||^2 + sum(var_a + var_b - 2 sd_a^3 sd_b), not the Gaussian W2;
* ``_cal_comp_sigma`` (45-62) likewise yields ((1-t) sd_a + t sd_b)^2 -- a variance -- and
  the reference passes it to ``Normal`` as the *scale*;
* the mixture weights are ``ot_Matrix.flatten()`` (row-major: i * Kb + j) while the
  components are stacked with j outer (index j * Ka + i) (23-25): weight n and component
  n belong to different (i, j) pairs when Ka = Kb > 1;
* ``BarycenterGMM.__init__`` calls ``_barycenter_gaussians(_print=False)`` on a method
  without that parameter (TypeError as shipped); the fixtures were captured with the kwarg
  ignored, which is the behaviour restated here.
"""
import itertools

import numpy as np


# ------------------------------------------------------------------ InterpolateGMM
def interp_cost(mu_a, sd_a, mu_b, sd_b):
    """(Ka, Kb) cost matrix of ``InterpolateGMM._w2sq`` (distributions.py:64-77), float64."""
    ka, kb = mu_a.shape[0], mu_b.shape[0]
    var_a = (sd_a.astype(np.float32) ** 2).astype(np.float64)
    var_b = (sd_b.astype(np.float32) ** 2).astype(np.float64)
    c = np.empty((ka, kb))
    for i in range(ka):
        for j in range(kb):
            sa, sb = np.sqrt(var_a[i]), np.sqrt(var_b[j])
            dm = mu_a[i].astype(np.float64) - mu_b[j].astype(np.float64)
            c[i, j] = dm @ dm + np.sum(var_a[i] + var_b[j] - 2.0 * sa ** 3 * sb)
    return c


def emd(a, b, cost):
    """Exact OT plan (``ot.emd`` restated as an LP; module docstring)."""
    from scipy.optimize import linprog
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    b = b * a.sum() / b.sum()
    ka, kb = len(a), len(b)
    a_eq = np.zeros((ka + kb, ka * kb))
    for i in range(ka):
        a_eq[i, i * kb:(i + 1) * kb] = 1.0
    for j in range(kb):
        a_eq[ka + j, j::kb] = 1.0
    r = linprog(np.asarray(cost, np.float64).reshape(-1), A_eq=a_eq,
                b_eq=np.concatenate([a, b]), bounds=(0, None), method="highs")
    assert r.success, r.message
    return r.x.reshape(ka, kb)


def interp_mixture(plan, mu_a, sd_a, mu_b, sd_b, t):
    """(pi, mu, sd) of the interpolated mixture at rate t (distributions.py:23-62)."""
    ka, kb = plan.shape
    w = plan.reshape(-1)
    pi = (w / w.sum()).astype(np.float32)
    t32, u32 = np.float32(t), np.float32(1.0 - t)
    mu = np.empty((ka * kb, mu_a.shape[1]), np.float32)
    sd = np.empty_like(mu)
    var_a = (sd_a.astype(np.float32) ** 2).astype(np.float64)
    var_b = (sd_b.astype(np.float32) ** 2).astype(np.float64)
    for j in range(kb):
        for i in range(ka):
            n = j * ka + i
            mu[n] = u32 * mu_a[i] + t32 * mu_b[j]
            s = (1.0 - t) * np.sqrt(var_a[i]) + t * np.sqrt(var_b[j])
            sd[n] = (s * s).astype(np.float32)
    return pi, mu, sd


# ------------------------------------------------------------------ BarycenterGMM
def meta_product(metadata):
    """One-hot metadata vectors in ``BarycenterGMM._product`` order (102-108)."""
    pools = [[np.eye(len(v))[i] for i in v.values()] for v in metadata.values()]
    return np.stack([np.concatenate(p) for p in itertools.product(*pools)]).astype(np.float32)


def barycenters(mu, sd, rate, iters=60):
    """Every position in product(range(K), repeat=M) (distributions.py:136-163), float32
    with the reference's operation order: mean = sum_i r_i mu_i, and 60 fixed-point steps
    std <- (1/std) * sum_j (r_j * std) * sd_j."""
    m, k, d = mu.shape
    r32 = np.asarray(rate, np.float64).astype(np.float32)
    pos = list(itertools.product(range(k), repeat=m))
    bm = np.empty((len(pos), d), np.float32)
    bs = np.empty_like(bm)
    for n, p in enumerate(pos):
        acc = np.zeros(d, np.float32)
        for i in range(m):
            acc = acc + r32[i] * mu[i, p[i]]
        bm[n] = acc
        s = sd[0, p[0]].astype(np.float32).copy()
        for _ in range(iters):
            acc = np.zeros(d, np.float32)
            for j in range(m):
                acc = acc + (r32[j] * s) * sd[j, p[j]]
            s = (np.float32(1.0) / s) * acc
        bs[n] = s
    return pos, bm, bs


def determine_pi(pi, mu, sd, rate, bm, bs):
    """``_determine_pi`` (165-184): each original component goes to its nearest barycenter
    (||dmu||^2 + ||dsd||^2, first minimum in position order); weights rate_i * pi_ij summed
    per barycenter in first-use order.  Returns (used position indices, probs float64)."""
    m, k, _ = mu.shape
    used, probs = [], []
    for i in range(m):
        for j in range(k):
            dm = bm.astype(np.float64) - mu[i, j].astype(np.float64)
            ds = bs.astype(np.float64) - sd[i, j].astype(np.float64)
            dist = (dm * dm).sum(1) + (ds * ds).sum(1)
            best = int(np.argmin(dist))  # first minimum
            w = float(rate[i]) * float(pi[i, j])
            if best in used:
                probs[used.index(best)] += w
            else:
                used.append(best)
                probs.append(w)
    return np.array(used), np.array(probs)


def barycenter_mixture(pi, mu, sd, rate, iters=60):
    """(used positions, pi f32 normalised as Categorical does, mean, std)."""
    _, bm, bs = barycenters(mu, sd, rate, iters)
    used, probs = determine_pi(pi, mu, sd, rate, bm, bs)
    p32 = probs.astype(np.float32)
    return used, p32 / p32.sum(), bm[used], bs[used]
