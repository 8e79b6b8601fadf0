// The --use_clf language discriminator (train.py:168-197): the GE2E SpeechEmbedder's
// LSTM stack (speech_embedder_net.py:65-137), its projection + L2 norm + domain classifier
// head, and GE2ELoss's BCE term (speech_embedder_net.py:165-186), fp32 throughout (the
// reference runs this module in fp32; it is ~2% of the step's FLOPs).
//
// LSTM layer, batch_first (N sequences x T frames, rows n*T + t):
//   * the input projection of all T steps is ONE implicit GEMM (fs2_conv_gemm, taps = 1):
//     gx = x W_ih^T + b_ih + b_hh, (N*T, 4H);
//   * the recurrence runs one launch per step from the C entry point (no host round trip
//     per step): lstm_fwd_step fuses h_{t-1} W_hh^T (h rows staged in LDS, W_hh^T read
//     coalesced along the hidden unit) with the gate nonlinearities and the cell update, and
//     saves the activated gates and cell for the backward;
//   * the backward runs the same T steps in reverse; lstm_bwd_step fuses the recurrent
//     gradient dh_{t} += dgates_{t+1} W_hh (dgates row in LDS) with the gate derivatives, and
//     the input gradient of all steps is again one GEMM: dx = dgates W_ih.
// PyTorch gate order i, f, g, o; h0 = c0 = 0 (nn.LSTM defaults).
#include <math.h>

#include "common.hpp"

namespace fs2 {

constexpr int LSTM_RPT = 1;   // rows per thread
constexpr int LSTM_RB = 4 * LSTM_RPT;  // rows (sequences) per block
constexpr int LSTM_JB = 64;   // hidden units per block
constexpr int LSTM_HMAX = 256;

FS2_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(256) void lstm_fwd_step(const float* __restrict__ gx,
                                                     const float* __restrict__ wt, float* h_all,
                                                     float* c_all, float* act, int N, int T, int H,
                                                     int t) {
  // 4 waves x LSTM_RPT rows each: every W_hh^T element a thread loads serves LSTM_RPT rows
  __shared__ float hs[LSTM_RB][LSTM_HMAX];
  const int tid = threadIdx.x, r0 = tid / LSTM_JB, jj = tid % LSTM_JB;
  const int n0 = blockIdx.x * LSTM_RB;
  for (int e = tid; e < LSTM_RB * H; e += 256) {
    const int rr = e / H, k = e - rr * H, nn = n0 + rr;
    hs[rr][k] = (t > 0 && nn < N) ? h_all[((int64_t)nn * T + t - 1) * H + k] : 0.f;
  }
  __syncthreads();
  const int j = blockIdx.y * LSTM_JB + jj;
  if (j >= H) return;
  float a[LSTM_RPT][4];
#pragma unroll
  for (int q = 0; q < LSTM_RPT; ++q) {
    const int n = n0 + r0 + 4 * q;
    const float* g = gx + ((int64_t)(n < N ? n : 0) * T + t) * 4 * H;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) a[q][gi] = g[gi * H + j];
  }
  if (t > 0) {
    for (int k = 0; k < H; ++k) {
      const float* w = wt + (int64_t)k * 4 * H + j;
      const float w0 = w[0], w1 = w[H], w2 = w[2 * H], w3 = w[3 * H];
#pragma unroll
      for (int q = 0; q < LSTM_RPT; ++q) {
        const float hk = hs[r0 + 4 * q][k];
        a[q][0] = fmaf(hk, w0, a[q][0]);
        a[q][1] = fmaf(hk, w1, a[q][1]);
        a[q][2] = fmaf(hk, w2, a[q][2]);
        a[q][3] = fmaf(hk, w3, a[q][3]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < LSTM_RPT; ++q) {
    const int n = n0 + r0 + 4 * q;
    if (n >= N) continue;
    const int64_t row = (int64_t)n * T + t;
    const float i = sigm(a[q][0]), f = sigm(a[q][1]), gg = tanhf(a[q][2]), o = sigm(a[q][3]);
    const float cp = t > 0 ? c_all[(row - 1) * H + j] : 0.f;
    const float c = f * cp + i * gg;
    c_all[row * H + j] = c;
    h_all[row * H + j] = o * tanhf(c);
    float* ap = act + row * 4 * H;
    ap[j] = i;
    ap[H + j] = f;
    ap[2 * H + j] = gg;
    ap[3 * H + j] = o;
  }
}

// reverse step t: dh = dh_out[t] + dgates_{t+1} W_hh ; gate derivatives ; dc ping-pong
__global__ __launch_bounds__(256) void lstm_bwd_step(const float* __restrict__ dh_out,
                                                     const float* __restrict__ w_hh,
                                                     const float* __restrict__ act,
                                                     const float* __restrict__ c_all,
                                                     float* dgates, const float* dc_in,
                                                     float* dc_out, int N, int T, int H, int t) {
  __shared__ float ds[LSTM_RB][4 * LSTM_HMAX];
  const int tid = threadIdx.x, r0 = tid / LSTM_JB, jj = tid % LSTM_JB;
  const int n0 = blockIdx.x * LSTM_RB;
  const bool has_next = t + 1 < T;
  if (has_next) {
    for (int e = tid; e < LSTM_RB * 4 * H; e += 256) {
      const int rr = e / (4 * H), q = e - rr * 4 * H, nn = n0 + rr;
      ds[rr][q] = nn < N ? dgates[((int64_t)nn * T + t + 1) * 4 * H + q] : 0.f;
    }
  }
  __syncthreads();
  const int j = blockIdx.y * LSTM_JB + jj;
  if (j >= H) return;
  // recurrent gradient, 4 independent partial sums per row (one per gate block of W_hh)
  float acc[LSTM_RPT][4];
#pragma unroll
  for (int q = 0; q < LSTM_RPT; ++q)
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) acc[q][gi] = 0.f;
  if (has_next) {
    for (int u = 0; u < H; ++u) {
      const float w0 = w_hh[(int64_t)u * H + j], w1 = w_hh[(int64_t)(H + u) * H + j];
      const float w2 = w_hh[(int64_t)(2 * H + u) * H + j], w3 = w_hh[(int64_t)(3 * H + u) * H + j];
#pragma unroll
      for (int q = 0; q < LSTM_RPT; ++q) {
        const float* d = ds[r0 + 4 * q];
        acc[q][0] = fmaf(d[u], w0, acc[q][0]);
        acc[q][1] = fmaf(d[H + u], w1, acc[q][1]);
        acc[q][2] = fmaf(d[2 * H + u], w2, acc[q][2]);
        acc[q][3] = fmaf(d[3 * H + u], w3, acc[q][3]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < LSTM_RPT; ++q) {
    const int n = n0 + r0 + 4 * q;
    if (n >= N) continue;
    const int64_t row = (int64_t)n * T + t;
    float dh = (acc[q][0] + acc[q][1]) + (acc[q][2] + acc[q][3]);
    if (dh_out) dh += dh_out[row * H + j];
    const float* ap = act + row * 4 * H;
    const float i = ap[j], f = ap[H + j], gg = ap[2 * H + j], o = ap[3 * H + j];
    const float c = c_all[row * H + j];
    const float cp = t > 0 ? c_all[(row - 1) * H + j] : 0.f;
    const float tc = tanhf(c);
    const float dc = (has_next ? dc_in[(int64_t)n * H + j] : 0.f) + dh * o * (1.f - tc * tc);
    float* dg = dgates + row * 4 * H;
    dg[j] = dc * gg * i * (1.f - i);
    dg[H + j] = dc * cp * f * (1.f - f);
    dg[2 * H + j] = dc * i * (1.f - gg * gg);
    dg[3 * H + j] = dh * tc * o * (1.f - o);
    dc_out[(int64_t)n * H + j] = dc * f;
  }
}

// ---------------------------------------------------------------- discriminator head
// One wave per sequence row: x (the last LSTM frame, 256) -> projection (64) -> L2 norm ->
// Linear 64->64, dropout, ReLU -> Linear 64->64, dropout, ReLU -> Linear 64->1 (logit)
// (speech_embedder_net.py:126-136,146-162, module.py:22-38).  With dlogit (and/or demb)
// the same wave then back-propagates to dx (masks regenerated from the same Philox key).
struct ClfHead {
  const float* x;      // row n at x + n * ldx
  int64_t ldx;
  const float* wp;     // projection (P, D) and its transpose wpt (D, P), bias bp
  const float* wpt;
  const float* bp;
  const float* w0;     // (P, P), w0t, b0
  const float* w0t;
  const float* b0;
  const float* w1;
  const float* w1t;
  const float* b1;
  const float* w2;     // (1, P), b2 (1)
  const float* b2;
  int N, D, P;
  float p_drop;
  const uint64_t* seed;
  uint64_t site;
  float* emb;          // (N, P) or NULL
  float* logit;        // (N) or NULL
  const float* demb;   // backward inputs (NULL: zero)
  const float* dlogit;
  float* dx;           // row n at dx + n * lddx (backward only)
  int64_t lddx;
};

constexpr int CLF_D = 256, CLF_P = 64;

__global__ __launch_bounds__(256) void clf_head_kernel(ClfHead a) {
  __shared__ float xs[4][CLF_D];
  __shared__ float vs[4][CLF_P];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + wave;
  if (n >= a.N) return;  // whole wave
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  for (int k = lane; k < CLF_D; k += 64) xs[wave][k] = a.x[(int64_t)n * a.ldx + k];
  __builtin_amdgcn_wave_barrier();  // LDS rows are wave-private: no block barrier
  // projection + L2 normalisation
  float p = a.bp[lane];
  for (int k = 0; k < CLF_D; ++k) p = fmaf(a.wpt[k * CLF_P + lane], xs[wave][k], p);
  const float nrm = sqrtf(wave_sum(p * p));
  const float e = p / nrm;
  // classifier: dropout masks per (row, layer, unit)
  const uint64_t el = (uint64_t)n * (2 * CLF_P);
  const float m0 = a.p_drop > 0.f ? dropout1(seed, a.site, el + lane, a.p_drop) : 1.f;
  const float m1 = a.p_drop > 0.f ? dropout1(seed, a.site, el + CLF_P + lane, a.p_drop) : 1.f;
  vs[wave][lane] = e;
  __builtin_amdgcn_wave_barrier();
  float z0 = a.b0[lane];
  for (int k = 0; k < CLF_P; ++k) z0 = fmaf(a.w0t[k * CLF_P + lane], vs[wave][k], z0);
  const float a0 = fmaxf(z0 * m0, 0.f);
  __builtin_amdgcn_wave_barrier();
  vs[wave][lane] = a0;
  __builtin_amdgcn_wave_barrier();
  float z1 = a.b1[lane];
  for (int k = 0; k < CLF_P; ++k) z1 = fmaf(a.w1t[k * CLF_P + lane], vs[wave][k], z1);
  const float a1 = fmaxf(z1 * m1, 0.f);
  const float lg = wave_sum(a.w2[lane] * a1) + a.b2[0];
  if (a.emb) a.emb[(int64_t)n * CLF_P + lane] = e;
  if (a.logit && lane == 0) a.logit[n] = lg;
  if (!a.dx) return;
  // ---- backward
  const float dl = a.dlogit ? a.dlogit[n] : 0.f;
  const float dz1 = (a1 > 0.f ? dl * a.w2[lane] : 0.f) * m1;
  __builtin_amdgcn_wave_barrier();
  vs[wave][lane] = dz1;
  __builtin_amdgcn_wave_barrier();
  float da0 = 0.f;
  for (int o = 0; o < CLF_P; ++o) da0 = fmaf(a.w1[o * CLF_P + lane], vs[wave][o], da0);
  const float dz0 = (a0 > 0.f ? da0 : 0.f) * m0;
  __builtin_amdgcn_wave_barrier();
  vs[wave][lane] = dz0;
  __builtin_amdgcn_wave_barrier();
  float de = a.demb ? a.demb[(int64_t)n * CLF_P + lane] : 0.f;
  for (int o = 0; o < CLF_P; ++o) de = fmaf(a.w0[o * CLF_P + lane], vs[wave][o], de);
  // e = p / |p|  ->  dp = (de - e (e . de)) / |p|
  const float ed = wave_sum(e * de);
  const float dp = (de - e * ed) / nrm;
  __builtin_amdgcn_wave_barrier();
  vs[wave][lane] = dp;
  __builtin_amdgcn_wave_barrier();
  for (int k = lane; k < CLF_D; k += 64) {
    float s = 0.f;
    for (int o = 0; o < CLF_P; ++o) s = fmaf(a.wp[o * CLF_D + k], vs[wave][o], s);
    a.dx[(int64_t)n * a.lddx + k] = s;
  }
}

// BCEWithLogits(reduction='sum') per row + its logit gradient scaled by g (device scalar,
// the upstream gradient of the summed loss) times scale (host)
__global__ void bce_logits_kernel(const float* logit, const float* y, int64_t n, float* loss_rows,
                                  const float* g, float scale, float* dlogit) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = logit[i], t = y[i];
  if (loss_rows) loss_rows[i] = fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
  if (dlogit) dlogit[i] = (g ? g[0] : 1.f) * scale * (sigm(x) - t);
}

// rows of (B, T_src, C) re-laid out as (B, T_dst, C): copy min(T_src, T_dst) frames, zero
// the rest (the 150-frame chunking of train.py:178-183 and its gradient)
__global__ void rows_repad_kernel(const float* src, int64_t B, int64_t Ts, int64_t Td, int64_t C,
                                  float* dst) {
  const int64_t total = B * Td * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = e % C, bt = e / C, t = bt % Td, b = bt / Td;
    dst[e] = t < Ts ? src[(b * Ts + t) * C + c] : 0.f;
  }
}

// per-chunk language labels: y[b * rep + k] = meta[b * ld + col]  (train.py:184)
__global__ void repeat_col_kernel(const float* meta, int64_t B, int64_t ld, int col, int rep,
                                  float* y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B * rep) y[i] = meta[(i / rep) * ld + col];
}

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_lstm_layer_fwd(const float* x, int64_t n_seq, int64_t steps, int64_t c_in, int64_t hidden,
                       const float* w_ih, const float* bias, const float* w_hh_t, float* gx,
                       float* h_all, float* c_all, float* act, void* stream) {
  FS2_CHECK_ARG(hidden > 0 && hidden <= LSTM_HMAX && hidden % LSTM_JB == 0 && c_in % 4 == 0,
                "fs2_lstm_layer_fwd: hidden %lld (<= 256, multiple of 64), c_in %% 4",
                (long long)hidden);
  if (n_seq == 0 || steps == 0) return FS2_OK;
  const int64_t rows = n_seq * steps, G = 4 * hidden;
  // input projection of every step: one GEMM (taps = 1), both biases folded into `bias`
  int rc = fs2_conv_gemm(FS2_F32, x, c_in, w_ih, gx, G, rows, rows, c_in, G, 1, 0, nullptr, bias,
                         FS2_EPI_BIAS, nullptr, 0, stream);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)((n_seq + LSTM_RB - 1) / LSTM_RB), (unsigned)(hidden / LSTM_JB));
  for (int t = 0; t < (int)steps; ++t)
    lstm_fwd_step<<<grid, 256, 0, st>>>(gx, w_hh_t, h_all, c_all, act, (int)n_seq, (int)steps,
                                        (int)hidden, t);
  return launch_status("fs2_lstm_layer_fwd");
}

int fs2_lstm_layer_bwd(const float* dh_out, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, const float* w_ih_t, const float* w_hh, const float* act,
                       const float* c_all, float* dgates, float* dc_ws, float* dx, void* stream) {
  FS2_CHECK_ARG(hidden > 0 && hidden <= LSTM_HMAX && hidden % LSTM_JB == 0,
                "fs2_lstm_layer_bwd: hidden %lld (<= 256, multiple of 64)", (long long)hidden);
  if (n_seq == 0 || steps == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)((n_seq + LSTM_RB - 1) / LSTM_RB), (unsigned)(hidden / LSTM_JB));
  float* dc_a = dc_ws;                 // (n_seq, hidden) ping-pong
  float* dc_b = dc_ws + n_seq * hidden;
  for (int t = (int)steps - 1; t >= 0; --t) {
    lstm_bwd_step<<<grid, 256, 0, st>>>(dh_out, w_hh, act, c_all, dgates, dc_a, dc_b, (int)n_seq,
                                        (int)steps, (int)hidden, t);
    float* tmp = dc_a;
    dc_a = dc_b;
    dc_b = tmp;
  }
  int rc = launch_status("fs2_lstm_layer_bwd");
  if (rc || !dx) return rc;
  // input gradient of every step: dx = dgates W_ih (one GEMM with W_ih^T as the weight)
  const int64_t rows = n_seq * steps;
  return fs2_conv_gemm(FS2_F32, dgates, 4 * hidden, w_ih_t, dx, c_in, rows, rows, 4 * hidden, c_in,
                       1, 0, nullptr, nullptr, 0, nullptr, 0, stream);
}

int fs2_clf_head(const float* x, int64_t ldx, int64_t n, const float* wp, const float* wpt,
                 const float* bp, const float* w0, const float* w0t, const float* b0,
                 const float* w1, const float* w1t, const float* b1, const float* w2,
                 const float* b2, float p_drop, const uint64_t* seed, uint64_t site, float* emb,
                 float* logit, const float* demb, const float* dlogit, float* dx, int64_t lddx,
                 void* stream) {
  FS2_CHECK_ARG(x && wpt && bp && w0t && b0 && w1t && b1 && w2 && b2,
                "fs2_clf_head: missing forward operand");
  FS2_CHECK_ARG(!dx || (wp && w0 && w1), "fs2_clf_head: backward needs the natural weights");
  FS2_CHECK_ARG(p_drop <= 0.f || seed, "fs2_clf_head: dropout needs a seed");
  if (n == 0) return FS2_OK;
  ClfHead a{x, ldx, wp, wpt, bp, w0, w0t, b0, w1, w1t, b1, w2, b2, (int)n, CLF_D, CLF_P, p_drop,
            seed, site, emb, logit, demb, dlogit, dx, lddx};
  clf_head_kernel<<<(unsigned)((n + 3) / 4), 256, 0, as_stream(stream)>>>(a);
  return launch_status("fs2_clf_head");
}

int fs2_bce_logits(const float* logit, const float* y, int64_t n, float* loss_rows,
                   const float* g, float scale, float* dlogit, void* stream) {
  if (n == 0) return FS2_OK;
  bce_logits_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(
      logit, y, n, loss_rows, g, scale, dlogit);
  return launch_status("fs2_bce_logits");
}

int fs2_rows_repad(const float* src, int64_t batch, int64_t t_src, int64_t t_dst, int64_t c,
                   float* dst, void* stream) {
  const int64_t total = batch * t_dst * c;
  if (total == 0) return FS2_OK;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  rows_repad_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(src, batch, t_src, t_dst, c,
                                                                      dst);
  return launch_status("fs2_rows_repad");
}

int fs2_repeat_col(const float* meta, int64_t batch, int64_t ld, int col, int rep, float* y,
                   void* stream) {
  const int64_t n = batch * rep;
  if (n == 0) return FS2_OK;
  repeat_col_kernel<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(meta, batch, ld,
                                                                                 col, rep, y);
  return launch_status("fs2_repeat_col");
}

}  // extern "C"
