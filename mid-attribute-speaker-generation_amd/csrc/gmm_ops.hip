// Mid-attribute speaker-prior operations (model/distributions.py): InterpolateGMM's
// component cost, exact OT plan and interpolated mixture; BarycenterGMM's per-position
// barycenters and nearest-barycenter weights.  Off the training step (SURVEY.md §8a row
// 22, §8f f4): the shapes are tiny (K <= 16 components of D = 256, K^M <= 4096 barycenter
// positions), so every kernel is launch-bound; the point is that the whole construction
// stays on the device (the reference runs it in numpy/scipy with one 256 x 256 sqrtm per
// diagonal covariance) and reproduces the reference's arithmetic:
//
//  * costs / distances: fixed-order double reductions;
//  * barycenters: float32 with the reference's operation order and no contraction
//    (no contraction, IEEE division), so they match torch's CPU result bitwise;
//  * the OT plan: a transportation simplex (north-west-corner start, MODI potentials,
//    most-negative reduced cost, cycle through the basis tree) in one thread, double.
#include "common.hpp"

// The reference's float32 sums of products must not become FMAs (hipcc contracts by
// default, and HIP's __fmul_rn / __fadd_rn are plain operators defined in a header whose
// operations keep that default): the products and sums below are written here, where
// contraction is off.
#pragma clang fp contract(off)

namespace fs2 {

FS2_DEV float mul_rn(float a, float b) { return a * b; }
FS2_DEV float add_rn(float a, float b) { return a + b; }
FS2_DEV float rcp_rn(float a) { return 1.f / a; }  // IEEE division (correctly rounded)

constexpr int GMM_MAXK = 16;      // components per mixture (InterpolateGMM)
constexpr int GMM_MAXPOS = 4096;  // barycenter positions K^M
constexpr int GMM_MAXSRC = 64;    // original components M*K (BarycenterGMM)

// block-wide fixed-order double sum (256 threads)
FS2_DEV double block_sum_d(double v, double* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
#pragma unroll
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

// InterpolateGMM._w2sq (distributions.py:64-77) with its elementwise products of diagonal
// matrices: ||mu_a - mu_b||^2 + sum_d (va + vb - 2 sa^3 sb), va = fl32(sd_a^2), sa = sqrt(va)
__global__ __launch_bounds__(256) void gmm_w2_cost(const float* mu_a, const float* sd_a, int kb,
                                                   const float* mu_b, const float* sd_b, int d,
                                                   double* cost) {
  __shared__ double red[256];
  const int i = blockIdx.x / kb, j = blockIdx.x % kb;
  double acc = 0.0;
  for (int c = threadIdx.x; c < d; c += 256) {
    const double dm = (double)mu_a[i * d + c] - (double)mu_b[j * d + c];
    const float fa = sd_a[i * d + c], fb = sd_b[j * d + c];
    const double va = (double)mul_rn(fa, fa), vb = (double)mul_rn(fb, fb);
    const double sa = sqrt(va), sb = sqrt(vb);
    acc += dm * dm + (va + vb - 2.0 * sa * sa * sa * sb);
  }
  const double s = block_sum_d(acc, red);
  if (threadIdx.x == 0) cost[blockIdx.x] = s;
}

// Exact transport plan between a (ka) and b (kb, rescaled to a's mass as ot.emd does).
// status[0] = simplex iterations (>= 0) or -1 when max_iter was hit.
__global__ void ot_emd_kernel(const float* a_in, const float* b_in, const double* cost, int ka,
                              int kb, int max_iter, double* plan, int* status) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double sa[GMM_MAXK], sb[GMM_MAXK], x[GMM_MAXK * GMM_MAXK];
  bool basic[GMM_MAXK * GMM_MAXK];
  double suma = 0.0, sumb = 0.0;
  for (int i = 0; i < ka; ++i) suma += (double)a_in[i];
  for (int j = 0; j < kb; ++j) sumb += (double)b_in[j];
  for (int i = 0; i < ka; ++i) sa[i] = (double)a_in[i];
  for (int j = 0; j < kb; ++j) sb[j] = (double)b_in[j] * suma / sumb;
  for (int n = 0; n < ka * kb; ++n) {
    x[n] = 0.0;
    basic[n] = false;
  }
  // north-west corner: exactly ka + kb - 1 basic cells (one index advances per cell)
  {
    int i = 0, j = 0;
    while (true) {
      const double q = sa[i] < sb[j] ? sa[i] : sb[j];
      x[i * kb + j] = q;
      basic[i * kb + j] = true;
      sa[i] -= q;
      sb[j] -= q;
      if (i == ka - 1 && j == kb - 1) break;
      if (j == kb - 1 || (i < ka - 1 && sa[i] <= sb[j])) ++i;
      else ++j;
    }
  }
  double scale = 0.0;
  for (int n = 0; n < ka * kb; ++n) scale = fmax(scale, fabs(cost[n]));
  const double tol = 1e-12 * (scale > 0.0 ? scale : 1.0);
  int it = 0;
  for (; it < max_iter; ++it) {
    // potentials u_i + v_j = c_ij on the basis tree (u_0 = 0)
    double u[GMM_MAXK], v[GMM_MAXK];
    bool hu[GMM_MAXK], hv[GMM_MAXK];
    for (int i = 0; i < ka; ++i) hu[i] = false;
    for (int j = 0; j < kb; ++j) hv[j] = false;
    u[0] = 0.0;
    hu[0] = true;
    for (int pass = 0; pass < ka + kb; ++pass) {
      bool changed = false;
      for (int i = 0; i < ka; ++i)
        for (int j = 0; j < kb; ++j) {
          if (!basic[i * kb + j]) continue;
          if (hu[i] && !hv[j]) {
            v[j] = cost[i * kb + j] - u[i];
            hv[j] = changed = true;
          } else if (hv[j] && !hu[i]) {
            u[i] = cost[i * kb + j] - v[j];
            hu[i] = changed = true;
          }
        }
      if (!changed) break;
    }
    // entering cell: most negative reduced cost (first in row-major order on ties)
    int ei = -1, ej = -1;
    double best = -tol;
    for (int i = 0; i < ka; ++i)
      for (int j = 0; j < kb; ++j) {
        if (basic[i * kb + j]) continue;
        const double r = cost[i * kb + j] - u[i] - v[j];
        if (r < best) {
          best = r;
          ei = i;
          ej = j;
        }
      }
    if (ei < 0) break;  // optimal
    // path column ej -> row ei in the basis tree (BFS over ka + kb nodes; rows 0..ka-1,
    // columns ka..ka+kb-1), then the cycle alternates - / + starting at the column end
    int par[2 * GMM_MAXK], q[2 * GMM_MAXK];
    for (int n = 0; n < ka + kb; ++n) par[n] = -2;
    int qh = 0, qt = 0;
    q[qt++] = ka + ej;
    par[ka + ej] = -1;
    while (qh < qt && par[ei] == -2) {
      const int n = q[qh++];
      if (n < ka) {
        for (int j = 0; j < kb; ++j)
          if (basic[n * kb + j] && par[ka + j] == -2) {
            par[ka + j] = n;
            q[qt++] = ka + j;
          }
      } else {
        const int j = n - ka;
        for (int i = 0; i < ka; ++i)
          if (basic[i * kb + j] && par[i] == -2) {
            par[i] = n;
            q[qt++] = i;
          }
      }
    }
    // the cycle is (ei,ej)+ followed by the tree path back from column ej to row ei with
    // alternating signs: the edge at ej's end is -, the next +, ... (odd length, so the
    // edge at ei's end is - as well).  Collect the path walking up from ei.
    int cells[2 * GMM_MAXK];
    int nc = 0;
    for (int n = ei; par[n] != -1; n = par[n]) {
      const int p = par[n];
      const int r = n < ka ? n : p, c = n < ka ? p - ka : n - ka;
      cells[nc++] = r * kb + c;
    }
    // cells[nc-1] touches column ej: sign -, cells[nc-2] +, ..., cells[0] (touches ei) -
    double theta = 1e300;
    int leave = -1;
    for (int k = nc - 1; k >= 0; k -= 2) {
      if (x[cells[k]] < theta) {
        theta = x[cells[k]];
        leave = cells[k];
      }
    }
    for (int k = 0; k < nc; ++k) {
      const bool minus = ((nc - 1 - k) % 2) == 0;
      x[cells[k]] += minus ? -theta : theta;
    }
    x[ei * kb + ej] = theta;
    basic[ei * kb + ej] = true;
    basic[leave] = false;
    x[leave] = 0.0;
  }
  for (int n = 0; n < ka * kb; ++n) plan[n] = x[n] > 0.0 ? x[n] : 0.0;
  status[0] = it < max_iter ? it : -1;
}

// Interpolated mixture (distributions.py:23-62): weight n = plan.flatten()[n] / sum (row-major
// i * kb + j); component n = j * ka + i: mu = (1-t) mu_a[i] + t mu_b[j] (fp32),
// sd = ((1-t) sa + t sb)^2 (the variance the reference passes as the scale).
__global__ void gmm_interp(const double* plan, const float* mu_a, const float* sd_a, int ka,
                           const float* mu_b, const float* sd_b, int kb, int d, double t,
                           float* pi, float* mu, float* sd) {
  const int n = blockIdx.x;
  const int i = n % ka, j = n / ka;
  const float t32 = (float)t, u32 = (float)(1.0 - t);
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    mu[(int64_t)n * d + c] = add_rn(mul_rn(u32, mu_a[i * d + c]), mul_rn(t32, mu_b[j * d + c]));
    const float fa = sd_a[i * d + c], fb = sd_b[j * d + c];
    const double s = (1.0 - t) * sqrt((double)mul_rn(fa, fa)) + t * sqrt((double)mul_rn(fb, fb));
    sd[(int64_t)n * d + c] = (float)(s * s);
  }
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int k = 0; k < ka * kb; ++k) tot += plan[k];
    pi[n] = (float)(plan[n] / tot);
  }
}

// One barycenter per position p (itertools.product(range(k), repeat=m): last index fastest),
// distributions.py:144-163, fp32 in the reference's order:
//   mean = ((0 + r0 mu_0) + r1 mu_1) + ...
//   std <- (1/std) * (((0 + (r0 std) sd_0) + (r1 std) sd_1) + ...), iters times, from sd_0
__global__ void gmm_barycenter(const float* mu, const float* sd, int m, int k, int d,
                               const float* rate, int iters, float* bmean, float* bstd) {
  const int p = blockIdx.x;
  int pos[GMM_MAXSRC];
  int rem = p;
  for (int i = m - 1; i >= 0; --i) {
    pos[i] = rem % k;
    rem /= k;
  }
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float acc = 0.f;
    for (int i = 0; i < m; ++i)
      acc = add_rn(acc, mul_rn(rate[i], mu[((int64_t)i * k + pos[i]) * d + c]));
    bmean[(int64_t)p * d + c] = acc;
    float s = sd[(int64_t)pos[0] * d + c];
    for (int it = 0; it < iters; ++it) {
      float a2 = 0.f;
      for (int j = 0; j < m; ++j)
        a2 = add_rn(a2, mul_rn(mul_rn(rate[j], s), sd[((int64_t)j * k + pos[j]) * d + c]));
      s = mul_rn(rcp_rn(s), a2);
    }
    bstd[(int64_t)p * d + c] = s;
  }
}

// dist[src][p] = ||bmean_p - mu_src||^2 + ||bstd_p - sd_src||^2 (BarycenterGMM._w2sq, 186-192)
__global__ __launch_bounds__(256) void gmm_bary_dist(const float* mu, const float* sd, int d,
                                                     const float* bmean, const float* bstd,
                                                     int n_pos, double* dist) {
  __shared__ double red[256];
  const int src = blockIdx.y, p = blockIdx.x;
  double acc = 0.0;
  for (int c = threadIdx.x; c < d; c += 256) {
    const double dm = (double)bmean[(int64_t)p * d + c] - (double)mu[(int64_t)src * d + c];
    const double ds = (double)bstd[(int64_t)p * d + c] - (double)sd[(int64_t)src * d + c];
    acc += dm * dm + ds * ds;
  }
  const double s = block_sum_d(acc, red);
  if (threadIdx.x == 0) dist[(int64_t)src * n_pos + p] = s;
}

// _determine_pi (165-184): first minimum per original component (row-major over (i, j)),
// weights rate_i * pi_ij accumulated in double per barycenter in first-use order; then the
// Categorical normalisation in fp32.  n_used[0], used[], pi_out[] (capacity m * k).
__global__ void gmm_bary_assign(const double* dist, const float* pi, const double* rate, int m,
                                int k, int n_pos, int* n_used, int* used, float* pi_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double probs[GMM_MAXSRC];
  int nu = 0;
  for (int src = 0; src < m * k; ++src) {
    const double* row = dist + (int64_t)src * n_pos;
    int best = 0;
    for (int p = 1; p < n_pos; ++p)
      if (row[p] < row[best]) best = p;
    const double w = rate[src / k] * (double)pi[src];
    int u = 0;
    while (u < nu && used[u] != best) ++u;
    if (u == nu) {
      used[nu] = best;
      probs[nu++] = w;
    } else {
      probs[u] += w;
    }
  }
  float tot = 0.f;
  for (int u = 0; u < nu; ++u) tot += (float)probs[u];
  for (int u = 0; u < nu; ++u) pi_out[u] = (float)probs[u] / tot;
  n_used[0] = nu;
}

__global__ void gmm_bary_gather(const float* bmean, const float* bstd, const int* n_used,
                                const int* used, int d, float* mu_out, float* sd_out) {
  const int u = blockIdx.x;
  if (u >= n_used[0]) return;
  const int64_t p = used[u];
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    mu_out[(int64_t)u * d + c] = bmean[p * d + c];
    sd_out[(int64_t)u * d + c] = bstd[p * d + c];
  }
}

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_gmm_w2_cost(const float* mu_a, const float* sd_a, int ka, const float* mu_b,
                    const float* sd_b, int kb, int d, double* cost, void* stream) {
  FS2_CHECK_ARG(ka > 0 && kb > 0 && ka <= GMM_MAXK && kb <= GMM_MAXK && d > 0,
                "fs2_gmm_w2_cost: 1 <= ka, kb <= %d components, d > 0", GMM_MAXK);
  gmm_w2_cost<<<(unsigned)(ka * kb), 256, 0, as_stream(stream)>>>(mu_a, sd_a, kb, mu_b, sd_b, d,
                                                                  cost);
  return launch_status("fs2_gmm_w2_cost");
}

int fs2_ot_emd(const float* a, const float* b, const double* cost, int ka, int kb,
               int max_iter, double* plan, int* status, void* stream) {
  FS2_CHECK_ARG(ka > 0 && kb > 0 && ka <= GMM_MAXK && kb <= GMM_MAXK && max_iter > 0,
                "fs2_ot_emd: 1 <= ka, kb <= %d, max_iter > 0", GMM_MAXK);
  ot_emd_kernel<<<1, 64, 0, as_stream(stream)>>>(a, b, cost, ka, kb, max_iter, plan, status);
  return launch_status("fs2_ot_emd");
}

int fs2_gmm_interpolate(const double* plan, const float* mu_a, const float* sd_a, int ka,
                        const float* mu_b, const float* sd_b, int kb, int d, double t, float* pi,
                        float* mu, float* sd, void* stream) {
  FS2_CHECK_ARG(ka > 0 && kb > 0 && ka <= GMM_MAXK && kb <= GMM_MAXK && d > 0,
                "fs2_gmm_interpolate: bad shape");
  gmm_interp<<<(unsigned)(ka * kb), 256, 0, as_stream(stream)>>>(plan, mu_a, sd_a, ka, mu_b, sd_b,
                                                                 kb, d, t, pi, mu, sd);
  return launch_status("fs2_gmm_interpolate");
}

int64_t fs2_gmm_barycenter_positions(int m, int k) {
  if (m <= 0 || k <= 0) return -1;
  int64_t n = 1;
  for (int i = 0; i < m; ++i) {
    n *= k;
    if (n > GMM_MAXPOS) return -1;
  }
  return n;
}

int fs2_gmm_barycenter(const float* mu, const float* sd, int m, int k, int d, const float* rate,
                       int iters, float* bmean, float* bstd, void* stream) {
  const int64_t n_pos = fs2_gmm_barycenter_positions(m, k);
  FS2_CHECK_ARG(n_pos > 0 && m * k <= GMM_MAXSRC && d > 0 && iters >= 0,
                "fs2_gmm_barycenter: need k^m <= %d positions and m*k <= %d", GMM_MAXPOS,
                GMM_MAXSRC);
  gmm_barycenter<<<(unsigned)n_pos, 256, 0, as_stream(stream)>>>(mu, sd, m, k, d, rate, iters,
                                                                 bmean, bstd);
  return launch_status("fs2_gmm_barycenter");
}

int64_t fs2_gmm_bary_mix_ws_bytes(int m, int k) {
  const int64_t n_pos = fs2_gmm_barycenter_positions(m, k);
  return n_pos > 0 ? (int64_t)m * k * n_pos * (int64_t)sizeof(double) : -1;
}

int fs2_gmm_bary_mix(const float* pi, const float* mu, const float* sd, int m, int k, int d,
                     const double* rate, const float* bmean, const float* bstd, int* n_used,
                     int* used, float* pi_out, float* mu_out, float* sd_out, double* ws,
                     int64_t ws_bytes, void* stream) {
  const int64_t n_pos = fs2_gmm_barycenter_positions(m, k);
  FS2_CHECK_ARG(n_pos > 0 && m * k <= GMM_MAXSRC && d > 0, "fs2_gmm_bary_mix: bad shape");
  FS2_CHECK_ARG(ws_bytes >= fs2_gmm_bary_mix_ws_bytes(m, k), "fs2_gmm_bary_mix: workspace too small");
  hipStream_t st = as_stream(stream);
  gmm_bary_dist<<<dim3((unsigned)n_pos, (unsigned)(m * k)), 256, 0, st>>>(mu, sd, d, bmean, bstd,
                                                                          (int)n_pos, ws);
  gmm_bary_assign<<<1, 64, 0, st>>>(ws, pi, rate, m, k, (int)n_pos, n_used, used, pi_out);
  gmm_bary_gather<<<(unsigned)(m * k), 256, 0, st>>>(bmean, bstd, n_used, used, d, mu_out, sd_out);
  return launch_status("fs2_gmm_bary_mix");
}

}  // extern "C"
