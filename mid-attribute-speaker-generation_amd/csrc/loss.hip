// Losses and the TacoSpawn GMM speaker prior.
//
// FastSpeech2Loss (model/loss.py:19-92) is computed without masked_select: each block sums
// |pred - target| (mel, postnet), (pred - target)^2 (pitch, energy, log-duration vs
// log(d + 1)) and the valid counts over its share of the padded tensors; a one-block
// finaliser adds the block partials in a fixed order (double accumulation) and divides.
// The backward writes sign/2x-residual gradients scaled by the upstream grads.
//
// The GMM head (model/fastspeech2.py:306-341) and SpeakerMetaEncLoss
// (model/loss.py:94-105) follow torch.distributions exactly: Categorical normalises pi
// and takes log(clamp(p, eps, 1 - eps)), MixtureSameFamily adds log_softmax of those
// logits to the Independent(Normal) component log-densities and logsumexps.
#include <math.h>

#include "common.hpp"

namespace fs2 {

constexpr int LOSS_FR = 64;  // frames per mel block

// partial layout per block: [mel_abs, post_abs, p_sq, e_sq, d_sq, mel_frames, src_count, 0]
__global__ void fs2loss_partial(const float* mel_out, const float* post_out, const float* mel_tgt,
                                int64_t tgt_len, const float* p_pred, const float* e_pred,
                                const float* logd_pred, const float* p_tgt, const float* e_tgt,
                                const int64_t* d_tgt, const uint8_t* src_pad, const uint8_t* mel_pad,
                                int64_t B, int64_t Ts, int64_t Tm, int n_mel, int64_t n_mel_blocks,
                                float* part) {
  __shared__ float red[8][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float s[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if ((int64_t)blockIdx.x < n_mel_blocks) {
    const int64_t fb = (int64_t)blockIdx.x * LOSS_FR;
    for (int f = wave; f < LOSS_FR; f += 4) {
      const int64_t fr = fb + f;  // flat (b, t) frame index over B x Tm
      if (fr >= B * Tm) break;
      const int64_t b = fr / Tm, t = fr - b * Tm;
      if (mel_pad[fr]) continue;
      if (lane == 0) s[5] += 1.f;
      const float* tg = mel_tgt + (b * tgt_len + t) * n_mel;
      for (int c = lane; c < n_mel; c += 64) {
        const float tv = tg[c];
        s[0] += fabsf(mel_out[fr * n_mel + c] - tv);
        s[1] += fabsf(post_out[fr * n_mel + c] - tv);
      }
    }
  } else {
    for (int64_t i = threadIdx.x; i < B * Ts; i += blockDim.x) {
      if (src_pad[i]) continue;
      const float dp = p_pred[i] - p_tgt[i];
      const float de = e_pred[i] - e_tgt[i];
      const float dd = logd_pred[i] - logf((float)d_tgt[i] + 1.f);
      s[2] += dp * dp;
      s[3] += de * de;
      s[4] += dd * dd;
      s[6] += 1.f;
    }
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const float v = wave_sum(s[k]);
    if (lane == 0) red[k][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8)
    part[(int64_t)blockIdx.x * 8 + threadIdx.x] =
        threadIdx.x < 7 ? red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3]
                        : 0.f;
}

// losses = [total, mel, post, pitch, energy, duration]; dens[0..1] = (mel elements, phonemes)
// 8 sums x 32 lanes: lane j of sum k adds partials j, j+32, ... in double; lanes are then
// added in lane order (deterministic)
__global__ __launch_bounds__(256) void fs2loss_final(const float* part, int64_t np, int n_mel,
                                                     const float* denoms, float* losses,
                                                     float* dens) {
  __shared__ double red[8][33];
  const int k = threadIdx.x >> 5, j = threadIdx.x & 31;
  double v = 0.0;
  for (int64_t p = j; p < np; p += 32) v += part[p * 8 + k];
  red[k][j] = v;
  __syncthreads();
  if (threadIdx.x != 0) return;
  double s[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int kk = 0; kk < 7; ++kk)
    for (int jj = 0; jj < 32; ++jj) s[kk] += red[kk][jj];
  const double dm = denoms ? denoms[0] : s[5] * n_mel;
  const double dsr = denoms ? denoms[1] : s[6];
  dens[0] = (float)dm;
  dens[1] = (float)dsr;
  const float mel = (float)(s[0] / dm), post = (float)(s[1] / dm);
  const float pl = (float)(s[2] / dsr), el = (float)(s[3] / dsr), dl = (float)(s[4] / dsr);
  losses[1] = mel;
  losses[2] = post;
  losses[3] = pl;
  losses[4] = el;
  losses[5] = dl;
  losses[0] = mel + post + dl + pl + el;  // model/loss.py:83-85 order
}

FS2_DEV float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

__global__ void fs2loss_bwd_mel(const float* mel_out, const float* post_out, const float* mel_tgt,
                                int64_t tgt_len, const uint8_t* mel_pad, int64_t B, int64_t Tm,
                                int n_mel, const float* dens, const float* g, float* d_mel,
                                float* d_post) {
  const int64_t n = B * Tm * n_mel;
  const float gm = (g[0] + g[1]) / dens[0], gp = (g[0] + g[2]) / dens[0];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t fr = e / n_mel, c = e - fr * n_mel;
    if (mel_pad[fr]) {
      d_mel[e] = 0.f;
      d_post[e] = 0.f;
      continue;
    }
    const int64_t b = fr / Tm, t = fr - b * Tm;
    const float tv = mel_tgt[(b * tgt_len + t) * n_mel + c];
    d_mel[e] = gm * sgn(mel_out[e] - tv);
    d_post[e] = gp * sgn(post_out[e] - tv);
  }
}

__global__ void fs2loss_bwd_var(const float* p_pred, const float* e_pred, const float* logd_pred,
                                const float* p_tgt, const float* e_tgt, const int64_t* d_tgt,
                                const uint8_t* src_pad, int64_t n, const float* dens,
                                const float* g, float* d_p, float* d_e, float* d_d) {
  const float s = 2.f / dens[1];
  const float gpi = (g[0] + g[3]) * s, ge = (g[0] + g[4]) * s, gd = (g[0] + g[5]) * s;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (src_pad[i]) {
      d_p[i] = d_e[i] = d_d[i] = 0.f;
      continue;
    }
    d_p[i] = gpi * (p_pred[i] - p_tgt[i]);
    d_e[i] = ge * (e_pred[i] - e_tgt[i]);
    d_d[i] = gd * (logd_pred[i] - logf((float)d_tgt[i] + 1.f));
  }
}

// ------------------------------------------------------------------ GMM
FS2_DEV float softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

__global__ void gmm_head_fwd(const float* meta, int in_dim, int K, int D, const float* w_pi,
                             const float* b_pi, const float* w_s, const float* b_s,
                             const float* w_mu, const float* b_mu, float* pi, float* sigma,
                             float* mu, float* sigma_pre) {
  const int64_t b = blockIdx.x;
  const float* m = meta + b * in_dim;
  const int KD = K * D;
  for (int o = threadIdx.x; o < KD; o += blockDim.x) {
    float xs = 0.f, xm = 0.f;
    for (int i = 0; i < in_dim; ++i) {
      xs += w_s[(int64_t)o * in_dim + i] * m[i];
      xm += w_mu[(int64_t)o * in_dim + i] * m[i];
    }
    xs += b_s[o];
    xm += b_mu[o];
    sigma_pre[b * KD + o] = xs;
    sigma[b * KD + o] = softplus(xs);
    mu[b * KD + o] = xm;
  }
  if (threadIdx.x == 0) {
    float z[16], mx = -INFINITY;
    for (int k = 0; k < K; ++k) {
      float x = 0.f;
      for (int i = 0; i < in_dim; ++i) x += w_pi[k * in_dim + i] * m[i];
      z[k] = x + b_pi[k];
      mx = fmaxf(mx, z[k]);
    }
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
      z[k] = expf(z[k] - mx);
      s += z[k];
    }
    for (int k = 0; k < K; ++k) pi[b * K + k] = z[k] / s;
  }
}

// torch.distributions Categorical(probs).logits -> log_softmax, for one row
FS2_DEV void log_mix(const float* pi, int K, float* lm, float* pn, float* sm) {
  float S = 0.f;
  for (int k = 0; k < K; ++k) S += pi[k];
  const float eps = 1.1920928955078125e-07f;
  float mx = -INFINITY;
  for (int k = 0; k < K; ++k) {
    pn[k] = pi[k] / S;
    const float c = fminf(fmaxf(pn[k], eps), 1.f - eps);
    lm[k] = logf(c);
    mx = fmaxf(mx, lm[k]);
  }
  float se = 0.f;
  for (int k = 0; k < K; ++k) se += expf(lm[k] - mx);
  const float lse = mx + logf(se);
  for (int k = 0; k < K; ++k) {
    sm[k] = expf(lm[k] - lse);
    lm[k] -= lse;
  }
}

__global__ void gmm_logprob(const float* e, const float* pi, const float* mu, const float* sigma,
                            int K, int D, float* logp, float* resp) {
  __shared__ float red[4];
  __shared__ float comp[16];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float c0 = logf(sqrtf(2.f * (float)M_PI));
  for (int k = 0; k < K; ++k) {
    float s = 0.f;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const int64_t o = (b * K + k) * D + d;
      const float sg = sigma[o], df = e[b * D + d] - mu[o];
      s += -(df * df) / (2.f * (sg * sg)) - logf(sg) - c0;
    }
    s = wave_sum(s);
    if (lane == 0) red[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0) comp[k] = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float lm[16], pn[16], sm[16], a[16], mx = -INFINITY;
    log_mix(pi + b * K, K, lm, pn, sm);
    for (int k = 0; k < K; ++k) {
      a[k] = comp[k] + lm[k];
      mx = fmaxf(mx, a[k]);
    }
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += expf(a[k] - mx);
    const float l = mx + logf(s);
    logp[b] = l;
    for (int k = 0; k < K; ++k) resp[b * K + k] = expf(a[k] - l);
  }
}

// dL/dz of the pi head output (b, k): through log_softmax, clamp, normalisation, softmax
FS2_DEV float gmm_pi_gz(const float* pi, const float* resp, const float* g, int64_t b, int K, int k) {
  float lm[16], pn[16], sm[16], dpn[16];
  const float* p = pi + b * K;
  log_mix(p, K, lm, pn, sm);
  const float eps = 1.1920928955078125e-07f;
  float S = 0.f;
  for (int j = 0; j < K; ++j) S += p[j];
  for (int j = 0; j < K; ++j) {
    const float dl = g[b] * resp[b * K + j] - sm[j] * g[b];
    const bool in = pn[j] >= eps && pn[j] <= 1.f - eps;
    const float c = fminf(fmaxf(pn[j], eps), 1.f - eps);
    dpn[j] = in ? dl / c : 0.f;
  }
  float t = 0.f;
  for (int j = 0; j < K; ++j) t += dpn[j] * p[j];
  float dot = 0.f, dpk = 0.f;
  for (int j = 0; j < K; ++j) {
    const float dpj = dpn[j] / S - t / (S * S);
    dot += p[j] * dpj;
    if (j == k) dpk = dpj;
  }
  return p[k] * (dpk - dot);
}

// Blocks 0..: one thread per mu / sigma head output, looping over the batch in order.
// Last block: the pi head -- (b, k) gradients for a chunk of the batch into LDS, then one
// thread per (k, input) sums the chunk in batch order.  Deterministic throughout.
// 8 waves per block: for its 64 mu / sigma outputs (one per lane) wave w sums the batch rows
// b = w, w + 8, ... in order, and the 8 wave partials are added in wave order through LDS (a
// single thread walking all B rows was a chain of dependent divisions / exps: 40-60 us on the
// step's critical path at B = 48).  The last block computes the pi head's gradients.
__global__ __launch_bounds__(512) void gmm_head_bwd(const float* meta, const float* e,
                                                    const float* pi, const float* mu,
                                                    const float* sigma, const float* sigma_pre,
                                                    const float* resp, const float* g, int64_t B,
                                                    int in_dim, int K, int D, float* dw_pi,
                                                    float* db_pi, float* dw_s, float* db_s,
                                                    float* dw_mu, float* db_mu) {
  const int KD = K * D;
  if (blockIdx.x == gridDim.x - 1) {
    __shared__ float gzs[256];
    const int CH = 256 / K, t = threadIdx.x;
    const int k_acc = t / (in_dim + 1), i_acc = t - k_acc * (in_dim + 1);
    float acc = 0.f;
    for (int64_t b0 = 0; b0 < B; b0 += CH) {
      const int64_t b = b0 + t / K;
      if (t < CH * K && b < B) gzs[t] = gmm_pi_gz(pi, resp, g, b, K, t % K);
      __syncthreads();
      if (k_acc < K) {
        for (int64_t bb = b0; bb < b0 + CH && bb < B; ++bb) {
          const float gz = gzs[(bb - b0) * K + k_acc];
          acc += i_acc < in_dim ? gz * meta[bb * in_dim + i_acc] : gz;
        }
      }
      __syncthreads();
    }
    if (k_acc < K) {
      if (i_acc < in_dim) dw_pi[k_acc * in_dim + i_acc] += acc;
      else db_pi[k_acc] += acc;
    }
    return;
  }
  __shared__ float red[8][9][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int o = blockIdx.x * 64 + lane;
  const bool act = o < 2 * KD;
  const int kd = o < KD ? o : o - KD;
  const int k = kd / D, dd = kd - k * D;
  float acc_w[8] = {0, 0, 0, 0, 0, 0, 0, 0}, acc_b = 0.f;
  if (act) {
    for (int64_t b = w; b < B; b += 8) {
      const int64_t idx = b * KD + kd;
      const float gg = g[b] * resp[b * K + k];
      const float sg = sigma[idx], df = e[b * D + dd] - mu[idx];
      float gz;
      if (o < KD) {  // mu
        gz = gg * df / (sg * sg);
      } else {  // sigma through softplus
        const float dsg = gg * (df * df / (sg * sg * sg) - 1.f / sg);
        const float x = sigma_pre[idx];
        gz = dsg * (x > 20.f ? 1.f : 1.f / (1.f + expf(-x)));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i < in_dim) acc_w[i] += gz * meta[b * in_dim + i];
      acc_b += gz;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[w][i][lane] = acc_w[i];
  red[w][8][lane] = acc_b;
  __syncthreads();
  if (w != 0 || !act) return;
  float* dw = o < KD ? dw_mu : dw_s;
  float* db = o < KD ? db_mu : db_s;
  for (int i = 0; i < in_dim; ++i) {
    float sw = red[0][i][lane];
#pragma unroll
    for (int v = 1; v < 8; ++v) sw += red[v][i][lane];
    dw[kd * in_dim + i] += sw;
  }
  float sb = red[0][8][lane];
#pragma unroll
  for (int v = 1; v < 8; ++v) sb += red[v][8][lane];
  db[kd] += sb;
}

__global__ void mean_k(const float* x, int64_t n, float* out, const float* den) {
  if (threadIdx.x != 0) return;
  float s = 0.f;  // python sum() over the batch, in order (model/loss.py:104)
  for (int64_t i = 0; i < n; ++i) s += x[i];
  out[0] = s / (den ? den[0] : (float)n);
}

// data-parallel denominators of this rank's batch: [valid mel elements, valid phonemes, B]
__global__ void dp_counts(const int64_t* src_lens, const int64_t* mel_lens, int64_t B,
                          int64_t src_len, int64_t mel_len, int n_mel, float* out) {
  if (threadIdx.x != 0) return;
  double m = 0, s = 0;
  for (int64_t b = 0; b < B; ++b) {
    m += (double)(mel_lens[b] < mel_len ? mel_lens[b] : mel_len);
    s += (double)(src_lens[b] < src_len ? src_lens[b] : src_len);
  }
  out[0] = (float)(m * n_mel);
  out[1] = (float)s;
  out[2] = (float)B;
}

__global__ void gmm_sample(const float* pi, const float* mu, const float* sigma, int64_t B, int K,
                           int D, uint64_t seed, uint64_t offset, float* out, int32_t* comp) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * D) return;
  const int64_t b = e / D, d = e - b * D;
  const u32x4 rc = philox((uint32_t)b, (uint32_t)(b >> 32), (uint32_t)offset, (uint32_t)(offset >> 32), seed);
  const float* p = pi + b * K;
  float S = 0.f;
  for (int k = 0; k < K; ++k) S += p[k];
  const float u = u01(rc.x) * S;
  int c = K - 1;
  float run = 0.f;
  for (int k = 0; k < K; ++k) {
    run += p[k];
    if (u < run) { c = k; break; }
  }
  const uint64_t off2 = offset + 1;
  const u32x4 rn = philox((uint32_t)e, (uint32_t)(e >> 32), (uint32_t)off2, (uint32_t)(off2 >> 32), seed);
  const float u1 = fmaxf(u01(rn.x), 1e-12f), u2 = u01(rn.y);
  const float n = sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
  const int64_t idx = (b * K + c) * D + d;
  out[e] = mu[idx] + sigma[idx] * n;
  if (comp && d == 0) comp[b] = c;
}

}  // namespace fs2

using namespace fs2;

extern "C" {

static int64_t loss_parts(int64_t B, int64_t Tm) { return (B * Tm + LOSS_FR - 1) / LOSS_FR + 1; }

int64_t fs2_fs2loss_ws_bytes(int64_t batch, int64_t mel_len) {
  return (loss_parts(batch, mel_len) * 8 + 4) * 4;
}

int fs2_fs2loss_fwd(const float* mel_out, const float* post_out, const float* mel_tgt,
                     int64_t tgt_len, const float* p_pred, const float* e_pred,
                     const float* logd_pred, const float* p_tgt, const float* e_tgt,
                     const int64_t* d_tgt, const uint8_t* src_pad, const uint8_t* mel_pad,
                     int64_t batch, int64_t src_len, int64_t mel_len, int n_mel,
                     const float* denoms, float* losses, float* ws, int64_t ws_bytes, void* stream) {
  FS2_CHECK_ARG(tgt_len >= mel_len, "fs2_fs2loss_fwd: target shorter than prediction");
  FS2_CHECK_ARG(ws_bytes >= fs2_fs2loss_ws_bytes(batch, mel_len), "fs2_fs2loss_fwd: workspace too small");
  hipStream_t st = as_stream(stream);
  poison(ws, ws_bytes, st);
  const int64_t np = loss_parts(batch, mel_len);
  fs2loss_partial<<<(unsigned)np, 256, 0, st>>>(mel_out, post_out, mel_tgt, tgt_len, p_pred, e_pred,
                                                logd_pred, p_tgt, e_tgt, d_tgt, src_pad, mel_pad,
                                                batch, src_len, mel_len, n_mel, np - 1, ws);
  fs2loss_final<<<1, 256, 0, st>>>(ws, np, n_mel, denoms, losses, ws + np * 8);
  return launch_status("fs2_fs2loss_fwd");
}

int fs2_fs2loss_bwd(const float* mel_out, const float* post_out, const float* mel_tgt,
                     int64_t tgt_len, const float* p_pred, const float* e_pred,
                     const float* logd_pred, const float* p_tgt, const float* e_tgt,
                     const int64_t* d_tgt, const uint8_t* src_pad, const uint8_t* mel_pad,
                     int64_t batch, int64_t src_len, int64_t mel_len, int n_mel, const float* ws,
                     const float* g_losses, float* d_mel_out, float* d_post_out, float* d_p,
                     float* d_e, float* d_logd, void* stream) {
  hipStream_t st = as_stream(stream);
  const float* dens = ws + loss_parts(batch, mel_len) * 8;
  const int64_t n = batch * mel_len * n_mel;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (n > 0)
    fs2loss_bwd_mel<<<(unsigned)blocks, 256, 0, st>>>(mel_out, post_out, mel_tgt, tgt_len, mel_pad,
                                                      batch, mel_len, n_mel, dens, g_losses,
                                                      d_mel_out, d_post_out);
  const int64_t ns = batch * src_len;
  if (ns > 0)
    fs2loss_bwd_var<<<(unsigned)((ns + 255) / 256), 256, 0, st>>>(p_pred, e_pred, logd_pred, p_tgt,
                                                                  e_tgt, d_tgt, src_pad, ns, dens,
                                                                  g_losses, d_p, d_e, d_logd);
  return launch_status("fs2_fs2loss_bwd");
}

int fs2_gmm_head_fwd(const float* meta, int64_t batch, int in_dim, int k, int d,
                     const float* w_pi, const float* b_pi, const float* w_sigma,
                     const float* b_sigma, const float* w_mu, const float* b_mu, float* pi,
                     float* sigma, float* mu, float* sigma_pre, void* stream) {
  FS2_CHECK_ARG(k >= 1 && k <= 16 && in_dim >= 1 && in_dim <= 8, "fs2_gmm_head_fwd: k <= 16, in_dim <= 8");
  if (batch == 0) return FS2_OK;
  gmm_head_fwd<<<(unsigned)batch, 256, 0, as_stream(stream)>>>(meta, in_dim, k, d, w_pi, b_pi, w_sigma,
                                                               b_sigma, w_mu, b_mu, pi, sigma, mu,
                                                               sigma_pre);
  return launch_status("fs2_gmm_head_fwd");
}

int fs2_gmm_logprob(const float* e, const float* pi, const float* mu, const float* sigma,
                    int64_t batch, int k, int d, float* logp, float* resp, float* mean_out,
                    const float* denom, void* stream) {
  FS2_CHECK_ARG(k >= 1 && k <= 16, "fs2_gmm_logprob: k <= 16");
  if (batch == 0) return FS2_OK;
  gmm_logprob<<<(unsigned)batch, 256, 0, as_stream(stream)>>>(e, pi, mu, sigma, k, d, logp, resp);
  if (mean_out) mean_k<<<1, 64, 0, as_stream(stream)>>>(logp, batch, mean_out, denom);
  return launch_status("fs2_gmm_logprob");
}

int fs2_gmm_head_bwd(const float* meta, const float* e, const float* pi, const float* mu,
                     const float* sigma, const float* sigma_pre, const float* resp,
                     const float* g_logp, int64_t batch, int in_dim, int k, int d,
                     float* dw_pi, float* db_pi, float* dw_sigma, float* db_sigma, float* dw_mu,
                     float* db_mu, void* stream) {
  FS2_CHECK_ARG(k >= 1 && k <= 16 && in_dim >= 1 && in_dim <= 8, "fs2_gmm_head_bwd: k <= 16, in_dim <= 8");
  FS2_CHECK_ARG(k * (in_dim + 1) <= 256, "fs2_gmm_head_bwd: k * (in_dim + 1) <= 256");
  const int64_t n = 2LL * k * d;
  gmm_head_bwd<<<(unsigned)((n + 63) / 64 + 1), 512, 0, as_stream(stream)>>>(
      meta, e, pi, mu, sigma, sigma_pre, resp, g_logp, batch, in_dim, k, d, dw_pi, db_pi, dw_sigma,
      db_sigma, dw_mu, db_mu);
  return launch_status("fs2_gmm_head_bwd");
}

int fs2_dp_counts(const int64_t* src_lens, const int64_t* mel_lens, int64_t batch,
                  int64_t src_len, int64_t mel_len, int n_mel, float* out, void* stream) {
  dp_counts<<<1, 64, 0, as_stream(stream)>>>(src_lens, mel_lens, batch, src_len, mel_len, n_mel, out);
  return launch_status("fs2_dp_counts");
}

int fs2_gmm_sample(const float* pi, const float* mu, const float* sigma, int64_t batch, int k,
                   int d, uint64_t seed, uint64_t offset, float* out, int32_t* comp, void* stream) {
  const int64_t n = batch * d;
  if (n == 0) return FS2_OK;
  gmm_sample<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(pi, mu, sigma, batch, k, d,
                                                                        seed, offset, out, comp);
  return launch_status("fs2_gmm_sample");
}

}  // extern "C"
