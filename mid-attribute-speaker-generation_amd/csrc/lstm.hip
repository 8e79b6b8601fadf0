// The --use_clf language discriminator (train.py:168-197): the GE2E SpeechEmbedder's
// LSTM stack (speech_embedder_net.py:65-137), its projection + L2 norm + domain classifier
// head, and GE2ELoss's BCE term (speech_embedder_net.py:165-186), fp32 throughout (the
// reference runs this module in fp32; it is ~2% of the step's FLOPs).
//
// LSTM layer, batch_first (N sequences x T frames, rows n*T + t):
//   * the input projection of all T steps is ONE implicit GEMM (fs2_conv_gemm, taps = 1):
//     gx = x W_ih^T + b_ih + b_hh, (N*T, 4H);
//   * the recurrence runs one launch per step from the C entry point (no host round trip
//     per step): lstm_fwd_step fuses h_{t-1} W_hh^T (f32 MFMA, split-K over the block's
//     waves) with the gate nonlinearities and the cell update, and saves the activated gates
//     and cell for the backward;
//   * the backward runs the same T steps in reverse; lstm_bwd_step fuses the recurrent
//     gradient dh_{t} += dgates_{t+1} W_hh (same MFMA scheme) with the gate derivatives, and
//     the input gradient of all steps is again one GEMM: dx = dgates W_ih.
// PyTorch gate order i, f, g, o; h0 = c0 = 0 (nn.LSTM defaults).
#include <math.h>

#include "common.hpp"

namespace fs2 {

FS2_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// The recurrent products run on the f32-input MFMA (v_mfma_f32_16x16x4_f32: f32 operands,
// f32 accumulation, the fp32 arithmetic of the reference's cuDNN/ATen LSTM).  A step is a
// (N x 4H x H) product, ~50 MFLOP: latency, not throughput, bounds it, so each output tile is
// split over the K dimension across the waves of a block (all loads of a wave issued up
// front) and the partials meet in LDS.  K order inside a 16-wide k group: operand register c
// of lane quarter kq is k = 16 g + 4 kq + c, so every lane fetches a float4 of A and of B.
using f32x4m = __attribute__((__vector_size__(4 * sizeof(float)))) float;

FS2_DEV f32x4m mfma4(float a, float b, f32x4m c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

FS2_DEV void mfma_k16(const float4& a, const float4& b, f32x4m& c0, f32x4m& c1) {
  c0 = mfma4(a.x, b.x, c0);
  c1 = mfma4(a.y, b.y, c1);
  c0 = mfma4(a.z, b.z, c0);
  c1 = mfma4(a.w, b.w, c1);
}

// one wave's share of a split-K tile: kper / (16 GT) trips, each issuing GT float4 loads of
// A and of B before its 4 GT MFMAs
template <int GT>
FS2_DEV void lstm_mfma_share(const float* ap, const float* bp, bool bvalid, int kb, int kper,
                             f32x4m& c0, f32x4m& c1) {
  for (int k = kb; k < kb + kper; k += 16 * GT) {
    float4 av[GT], bv[GT];
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      av[g] = *reinterpret_cast<const float4*>(ap + k + 16 * g);
      bv[g] = *reinterpret_cast<const float4*>(bp + k + 16 * g);
    }
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      if (!bvalid) bv[g] = make_float4(0.f, 0.f, 0.f, 0.f);
      mfma_k16(av[g], bv[g], c0, c1);
    }
  }
}

// the same with two A tiles (rows ap0 / ap1) sharing every B load
template <int GT>
FS2_DEV void lstm_mfma_share2(const float* ap0, const float* ap1, const float* bp, bool bvalid,
                              int kb, int kper, f32x4m (&c)[2][2]) {
  for (int k = kb; k < kb + kper; k += 16 * GT) {
    float4 a0[GT], a1[GT], bv[GT];
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      a0[g] = *reinterpret_cast<const float4*>(ap0 + k + 16 * g);
      a1[g] = *reinterpret_cast<const float4*>(ap1 + k + 16 * g);
      bv[g] = *reinterpret_cast<const float4*>(bp + k + 16 * g);
    }
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      if (!bvalid) bv[g] = make_float4(0.f, 0.f, 0.f, 0.f);
      mfma_k16(a0[g], bv[g], c[0][0], c[0][1]);
      mfma_k16(a1[g], bv[g], c[1][0], c[1][1]);
    }
  }
}

// two A tiles x two B tiles (sequence tiles): every A load feeds two B columns
template <int GT>
FS2_DEV void lstm_mfma_share22(const float* ap0, const float* ap1, const float* bp0,
                               const float* bp1, bool bv0, bool bv1, int kb, int kper,
                               f32x4m (&c)[2][2][2]) {
  for (int k = kb; k < kb + kper; k += 16 * GT) {
    float4 a0[GT], a1[GT], b0[GT], b1[GT];
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      a0[g] = *reinterpret_cast<const float4*>(ap0 + k + 16 * g);
      a1[g] = *reinterpret_cast<const float4*>(ap1 + k + 16 * g);
      b0[g] = *reinterpret_cast<const float4*>(bp0 + k + 16 * g);
      b1[g] = *reinterpret_cast<const float4*>(bp1 + k + 16 * g);
    }
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      if (!bv0) b0[g] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!bv1) b1[g] = make_float4(0.f, 0.f, 0.f, 0.f);
      mfma_k16(a0[g], b0[g], c[0][0][0], c[0][0][1]);
      mfma_k16(a1[g], b0[g], c[1][0][0], c[1][0][1]);
      mfma_k16(a0[g], b1[g], c[0][1][0], c[0][1][1]);
      mfma_k16(a1[g], b1[g], c[1][1][0], c[1][1][1]);
    }
  }
}

constexpr int LSTM_FWD_WAVES = 8;  // split-K ways of the forward tile (K = H)
constexpr int LSTM_FWD_GT = 2;     // 16-k groups per trip (H / 8 = 32 k per wave at H = 256)
constexpr int LSTM_BWD_WAVES = 8;  // split-K ways of the backward tile (K = 4H)

// Forward step t.  Block tile: 4 hidden units (16 gate rows m = 4 uu + gate, so a lane's 4
// accumulators are the i, f, g, o of one (unit, sequence)) x 16 sequences:
//   gates^T[m][n] = sum_k W_hh[gate * H + u][k] h_{t-1}[n][k]  (+ gx, which holds x W_ih^T + b)
// then the cell update; saves h, c and the activated gates for the backward.
__global__ __launch_bounds__(64 * LSTM_FWD_WAVES) void lstm_fwd_step(const float* __restrict__ gx,
                                                     const float* __restrict__ w_hh, float* h_all,
                                                     float* c_all, float* act, int N, int T, int H,
                                                     int t) {
  __shared__ float red[LSTM_FWD_WAVES][4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = blockIdx.x * 4, n0 = blockIdx.y * 16;
  // epilogue thread (wave 0) -> (sequence nn, unit uu), units fastest; its accumulators sit at
  // lane uu*16 + nn.  Its gx and c_{t-1} loads are issued before the product.
  const int uu = threadIdx.x & 3, nn = (threadIdx.x >> 2) & 15, ne = n0 + nn, u = u0 + uu;
  const bool epi = wave == 0 && ne < N;
  const int64_t row = (int64_t)(epi ? ne : 0) * T + t;
  float z[4], cp = 0.f;
  if (epi) {
    const float* g = gx + row * 4 * H;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) z[gi] = g[gi * H + u];
    if (t > 0) cp = c_all[(row - 1) * H + u];
  }
  if (t > 0) {
    const int kq = lane >> 4, r = lane & 15;
    const int m_unit = u0 + (r >> 2), m_gate = r & 3;   // A row of this lane
    const int n = n0 + r;                              // B column of this lane
    const float* ap = w_hh + ((int64_t)m_gate * H + m_unit) * H + 4 * kq;
    const bool nv = n < N;
    const float* bp = h_all + ((int64_t)(nv ? n : 0) * T + t - 1) * H + 4 * kq;
    const int kper = H / LSTM_FWD_WAVES;
    f32x4m c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
    lstm_mfma_share<LSTM_FWD_GT>(ap, bp, nv, wave * kper, kper, c0, c1);
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][i][lane] = c0[i] + c1[i];
  }
  __syncthreads();
  if (!epi) return;
  if (t > 0) {
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      float r = 0.f;
#pragma unroll
      for (int w = 0; w < LSTM_FWD_WAVES; ++w) r += red[w][gi][uu * 16 + nn];
      z[gi] += r;
    }
  }
  // D rows m = 4 * (lane >> 4) + i: lane quarter = unit, register i = gate
  const float i = sigm(z[0]), f = sigm(z[1]), gg = tanhf(z[2]), o = sigm(z[3]);
  const float c = f * cp + i * gg;
  c_all[row * H + u] = c;
  h_all[row * H + u] = o * tanhf(c);
  float* ap = act + row * 4 * H;
  ap[u] = i;
  ap[H + u] = f;
  ap[2 * H + u] = gg;
  ap[3 * H + u] = o;
}

// Reverse step t.  Block tile: 16 hidden units x 16 sequences,
//   dh^T[u][n] = sum_q W_hh^T[u][q] dgates_{t+1}[n][q]  (+ dh_out[t]),
// split over K = 4H across 8 waves, then the gate derivatives and the dc ping-pong, one
// (sequence, unit) per thread (units fastest: coalesced dgates / dc stores).
__global__ __launch_bounds__(512) void lstm_bwd_step(const float* __restrict__ dh_out,
                                                     const float* __restrict__ w_hh_t,
                                                     const float* __restrict__ act,
                                                     const float* __restrict__ c_all,
                                                     float* dgates, const float* dc_in,
                                                     float* dc_out, int N, int T, int H, int t) {
  __shared__ float red[LSTM_BWD_WAVES][4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  const bool has_next = t + 1 < T;
  // epilogue thread (waves 0-3) -> (sequence nn, unit uu), units fastest; its operands are
  // loaded before the product
  const int uu = threadIdx.x & 15, nn = (threadIdx.x >> 4) & 15, ne = n0 + nn, u = u0 + uu;
  const bool epi = threadIdx.x < 256 && ne < N;
  const int64_t row = (int64_t)(epi ? ne : 0) * T + t;
  float dh = 0.f, i = 0.f, f = 0.f, gg = 0.f, o = 0.f, c = 0.f, cp = 0.f, dcn = 0.f;
  if (epi) {
    if (dh_out) dh = dh_out[row * H + u];
    const float* ap = act + row * 4 * H;
    i = ap[u], f = ap[H + u], gg = ap[2 * H + u], o = ap[3 * H + u];
    c = c_all[row * H + u];
    if (t > 0) cp = c_all[(row - 1) * H + u];
    if (has_next) dcn = dc_in[(int64_t)ne * H + u];
  }
  if (has_next) {
    const int kq = lane >> 4, r = lane & 15, n = n0 + r;
    const bool nv = n < N;
    const float* ap = w_hh_t + (int64_t)(u0 + r) * 4 * H + 4 * kq;
    const float* bp = dgates + ((int64_t)(nv ? n : 0) * T + t + 1) * 4 * H + 4 * kq;
    const int kper = 4 * H / LSTM_BWD_WAVES;
    f32x4m c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
    lstm_mfma_share<4>(ap, bp, nv, wave * kper, kper, c0, c1);
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][q][lane] = c0[q] + c1[q];
  }
  __syncthreads();
  if (!epi) return;
  if (has_next) {
    // D row m = unit uu = 4 * (lane >> 4) + q, column = sequence nn = lane & 15
    const int ln = (uu >> 2) * 16 + nn, q = uu & 3;
    float r = 0.f;
#pragma unroll
    for (int w = 0; w < LSTM_BWD_WAVES; ++w) r += red[w][q][ln];
    dh += r;
  }
  const float tc = tanhf(c);
  const float dc = dcn + dh * o * (1.f - tc * tc);
  float* dg = dgates + row * 4 * H;
  dg[u] = dc * gg * i * (1.f - i);
  dg[H + u] = dc * cp * f * (1.f - f);
  dg[2 * H + u] = dc * i * (1.f - gg * gg);
  dg[3 * H + u] = dh * tc * o * (1.f - o);
  dc_out[(int64_t)ne * H + u] = dc * f;
}

// ---------------------------------------------------------------- stacked layers
// The whole L-layer stack as a wavefront: launch s runs layer l at step t = s - l (forward)
// or t = T - 1 - s + (L - 1 - l) (backward), so the stack takes T + L - 1 launches instead
// of L * T, and the inter-layer products move into the step kernels:
//   forward, l >= 1:  gates = b_l + W_ih^l h^{l-1}_t + W_hh^l h^l_{t-1}   (K = 2H)
//   backward, l < L-1: dh^l_t = dgates^{l+1}_t W_ih^{l+1} + dgates^l_{t+1} W_hh^l  (K = 8H)
// (layer l-1's h_t / layer l+1's dgates_t were written by the previous launch).  Layer 0's
// input projection and input gradient stay one GEMM each (c_in = 80 mel channels).
// Buffers are layer-major: h, c (L, rows, H), act, dgates (L, rows, 4H), weights
// w_hh (L, 4H, H), w_ih of layers 1.. (L-1, 4H, H) and their transposes, bias (L, 4H).
struct LstmStackFwd {
  const float* gx0;     // layer 0: x W_ih^T + b (rows, 4H)
  const float* w_ih_up;
  const float* w_hh;
  const float* bias;
  float* h;
  float* c;
  float* act;
  int N, T, H, L, s;
};

// 4 waves, 8 hidden units (two 16-gate-row A tiles) x 32 sequences (two 16-sequence B tiles;
// every weight load feeds both): layer 0 splits the recurrent K = H 4 ways; layers >= 1 give
// the input product (K = H) to waves 0-1 and the recurrent one to waves 2-3.  Each output's
// k order and partial-sum order are those of one 16-sequence tile.
__global__ __launch_bounds__(256) void lstm_stack_fwd_step(LstmStackFwd a) {
  __shared__ float red[4][2][2][4][64];
  const int l = blockIdx.z, t = a.s - l;
  if (t < 0 || t >= a.T) return;  // block-uniform
  const int N = a.N, T = a.T, H = a.H;
  const int64_t rows = (int64_t)N * T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = blockIdx.x * 8, n0 = blockIdx.y * 32;
  float* h_l = a.h + l * rows * H;
  float* c_l = a.c + l * rows * H;
  // epilogue thread -> (sequence tile st, unit tile ut, sequence nn, unit uu)
  const int ut = (threadIdx.x >> 6) & 1, st = threadIdx.x >> 7, uu = threadIdx.x & 3,
            nn = (threadIdx.x >> 2) & 15;
  const int ne = n0 + st * 16 + nn, u = u0 + ut * 4 + uu;
  const bool epi = ne < N;
  const int64_t row = (int64_t)(epi ? ne : 0) * T + t;
  float z[4], cp = 0.f;
  if (epi) {
    const float* g = l == 0 ? a.gx0 + row * 4 * H : a.bias + (int64_t)l * 4 * H;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) z[gi] = g[gi * H + u];
    if (t > 0) cp = c_l[(row - 1) * H + u];
  }
  const int kq = lane >> 4, r = lane & 15;
  const int m_row = (r & 3) * H + u0 + (r >> 2);  // gate row of tile 0 (tile 1: + 4)
  const int nA = n0 + r, nB = n0 + 16 + r;
  const bool nvA = nA < N, nvB = nB < N;
  const int64_t nrowA = (int64_t)(nvA ? nA : 0) * T, nrowB = (int64_t)(nvB ? nB : 0) * T;
  f32x4m c[2][2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) c[x][y][0] = c[x][y][1] = f32x4m{0.f, 0.f, 0.f, 0.f};
  const float* w = nullptr;
  const float* hb = nullptr;  // h rows of the operand (this layer at t - 1, or the one below at t)
  int dt = 0, kb = 0, kper = 0;
  if (l == 0) {
    if (t > 0) {
      w = a.w_hh, hb = h_l, dt = -1;
      kb = wave * (H / 4), kper = H / 4;
    }
  } else if (wave < 2) {
    w = a.w_ih_up + (int64_t)(l - 1) * 4 * H * H;
    hb = a.h + (l - 1) * rows * H, dt = 0;
    kb = wave * (H / 2), kper = H / 2;
  } else if (t > 0) {
    w = a.w_hh + (int64_t)l * 4 * H * H;
    hb = h_l, dt = -1;
    kb = (wave - 2) * (H / 2), kper = H / 2;
  }
  if (w) {
    const float* ap0 = w + (int64_t)m_row * H + 4 * kq;
    lstm_mfma_share22<4>(ap0, ap0 + 4 * H, hb + (nrowA + t + dt) * H + 4 * kq,
                         hb + (nrowB + t + dt) * H + 4 * kq, nvA, nvB, kb, kper, c);
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][x][y][i][lane] = c[x][y][0][i] + c[x][y][1][i];
  __syncthreads();
  if (!epi) return;
#pragma unroll
  for (int gi = 0; gi < 4; ++gi) {
    float acc = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) acc += red[wv][ut][st][gi][uu * 16 + nn];
    z[gi] += acc;
  }
  const float i = sigm(z[0]), f = sigm(z[1]), gg = tanhf(z[2]), o = sigm(z[3]);
  const float cc = f * cp + i * gg;
  c_l[row * H + u] = cc;
  h_l[row * H + u] = o * tanhf(cc);
  float* ap = a.act + (l * rows + row) * 4 * H;
  ap[u] = i;
  ap[H + u] = f;
  ap[2 * H + u] = gg;
  ap[3 * H + u] = o;
}

struct LstmStackBwd {
  const float* dh_out;     // top layer's output gradient (rows, H) or NULL
  const float* w_ih_up_t;  // (L-1, H, 4H): W_ih^T of layers 1..
  const float* w_hh_t;     // (L, H, 4H)
  const float* act;
  const float* c;
  float* dg;               // (L, rows, 4H)
  float* dc;               // (L, 2, N, H) ping-pong by launch parity
  int N, T, H, L, s;
};

// 8 waves, 16 hidden units x 16 sequences: the top layer splits K = 4H (recurrent) 8 ways;
// lower layers give the gradient from the layer above (K = 4H) to waves 0-3 and the
// recurrent one to waves 4-7
__global__ __launch_bounds__(512) void lstm_stack_bwd_step(LstmStackBwd a) {
  __shared__ float red[8][4][64];
  const int l = blockIdx.z, L = a.L, t = a.T - 1 - a.s + (L - 1 - l);
  if (t < 0 || t >= a.T) return;  // block-uniform
  const int N = a.N, T = a.T, H = a.H;
  const int64_t rows = (int64_t)N * T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int u0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  const bool has_next = t + 1 < T, top = l == L - 1;
  float* dg_l = a.dg + l * rows * 4 * H;
  const float* dc_in = a.dc + ((int64_t)l * 2 + (a.s & 1)) * N * H;
  float* dc_out = a.dc + ((int64_t)l * 2 + ((a.s + 1) & 1)) * N * H;
  const int uu = threadIdx.x & 15, nn = (threadIdx.x >> 4) & 15, ne = n0 + nn, u = u0 + uu;
  const bool epi = threadIdx.x < 256 && ne < N;
  const int64_t row = (int64_t)(epi ? ne : 0) * T + t;
  float dh = 0.f, i = 0.f, f = 0.f, gg = 0.f, o = 0.f, c = 0.f, cp = 0.f, dcn = 0.f;
  if (epi) {
    if (top && a.dh_out) dh = a.dh_out[row * H + u];
    const float* ap = a.act + (l * rows + row) * 4 * H;
    i = ap[u], f = ap[H + u], gg = ap[2 * H + u], o = ap[3 * H + u];
    const float* c_l = a.c + l * rows * H;
    c = c_l[row * H + u];
    if (t > 0) cp = c_l[(row - 1) * H + u];
    if (has_next) dcn = dc_in[(int64_t)ne * H + u];
  }
  const int kq = lane >> 4, r = lane & 15, n = n0 + r;
  const bool nv = n < N;
  const int64_t nrow = (int64_t)(nv ? n : 0) * T;
  f32x4m c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
  if (top) {
    if (has_next) {
      const float* ap = a.w_hh_t + ((int64_t)l * H + u0 + r) * 4 * H + 4 * kq;
      const float* bp = dg_l + (nrow + t + 1) * 4 * H + 4 * kq;
      lstm_mfma_share<8>(ap, bp, nv, wave * (H / 2), H / 2, c0, c1);
    }
  } else if (wave < 4) {
    const float* ap = a.w_ih_up_t + ((int64_t)l * H + u0 + r) * 4 * H + 4 * kq;  // layer l+1
    const float* bp = a.dg + (l + 1) * rows * 4 * H + (nrow + t) * 4 * H + 4 * kq;
    lstm_mfma_share<8>(ap, bp, nv, wave * H, H, c0, c1);
  } else if (has_next) {
    const float* ap = a.w_hh_t + ((int64_t)l * H + u0 + r) * 4 * H + 4 * kq;
    const float* bp = dg_l + (nrow + t + 1) * 4 * H + 4 * kq;
    lstm_mfma_share<8>(ap, bp, nv, (wave - 4) * H, H, c0, c1);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[wave][q][lane] = c0[q] + c1[q];
  __syncthreads();
  if (!epi) return;
  {
    const int ln = (uu >> 2) * 16 + nn, q = uu & 3;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) acc += red[w][q][ln];
    dh += acc;
  }
  const float tc = tanhf(c);
  const float dc = dcn + dh * o * (1.f - tc * tc);
  float* dgp = dg_l + row * 4 * H;
  dgp[u] = dc * gg * i * (1.f - i);
  dgp[H + u] = dc * cp * f * (1.f - f);
  dgp[2 * H + u] = dc * i * (1.f - gg * gg);
  dgp[3 * H + u] = dh * tc * o * (1.f - o);
  dc_out[(int64_t)ne * H + u] = dc * f;
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
                       const float* w_ih, const float* bias, const float* w_hh, float* gx,
                       float* h_all, float* c_all, float* act, void* stream) {
  FS2_CHECK_ARG(hidden > 0 && hidden % 256 == 0 && c_in % 4 == 0,
                "fs2_lstm_layer_fwd: hidden %lld (multiple of 256), c_in %% 4",
                (long long)hidden);
  if (n_seq == 0 || steps == 0) return FS2_OK;
  const int64_t rows = n_seq * steps, G = 4 * hidden;
  // input projection of every step: one GEMM (taps = 1), both biases folded into `bias`
  int rc = fs2_conv_gemm(FS2_F32, x, c_in, w_ih, gx, G, rows, rows, c_in, G, 1, 0, nullptr, bias,
                         FS2_EPI_BIAS, nullptr, 0, stream);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(hidden / 4), (unsigned)((n_seq + 15) / 16));
  for (int t = 0; t < (int)steps; ++t)
    lstm_fwd_step<<<grid, 64 * LSTM_FWD_WAVES, 0, st>>>(gx, w_hh, h_all, c_all, act, (int)n_seq, (int)steps,
                                        (int)hidden, t);
  return launch_status("fs2_lstm_layer_fwd");
}

int fs2_lstm_layer_bwd(const float* dh_out, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, const float* w_ih_t, const float* w_hh_t, const float* act,
                       const float* c_all, float* dgates, float* dc_ws, float* dx, void* stream) {
  FS2_CHECK_ARG(hidden > 0 && hidden % 256 == 0,
                "fs2_lstm_layer_bwd: hidden %lld (multiple of 256)", (long long)hidden);
  if (n_seq == 0 || steps == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(hidden / 16), (unsigned)((n_seq + 15) / 16));
  float* dc_a = dc_ws;                 // (n_seq, hidden) ping-pong
  float* dc_b = dc_ws + n_seq * hidden;
  for (int t = (int)steps - 1; t >= 0; --t) {
    lstm_bwd_step<<<grid, 512, 0, st>>>(dh_out, w_hh_t, act, c_all, dgates, dc_a, dc_b, (int)n_seq,
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

int fs2_lstm_stack_fwd(const float* x, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, int layers, const float* w_ih0, const float* w_ih_up,
                       const float* w_hh, const float* bias, float* gx, float* h_all,
                       float* c_all, float* act, void* stream) {
  FS2_CHECK_ARG(hidden > 0 && hidden % 256 == 0 && c_in % 4 == 0 && layers >= 1,
                "fs2_lstm_stack_fwd: hidden %lld (multiple of 256), c_in %% 4, layers >= 1",
                (long long)hidden);
  FS2_CHECK_ARG(layers == 1 || w_ih_up, "fs2_lstm_stack_fwd: w_ih_up needed for layers > 1");
  if (n_seq == 0 || steps == 0) return FS2_OK;
  const int64_t rows = n_seq * steps, G = 4 * hidden;
  int rc = fs2_conv_gemm(FS2_F32, x, c_in, w_ih0, gx, G, rows, rows, c_in, G, 1, 0, nullptr, bias,
                         FS2_EPI_BIAS, nullptr, 0, stream);
  if (rc) return rc;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(hidden / 8), (unsigned)((n_seq + 31) / 32), (unsigned)layers);
  LstmStackFwd a{gx, w_ih_up, w_hh, bias, h_all, c_all, act, (int)n_seq, (int)steps,
                 (int)hidden, layers, 0};
  for (int s = 0; s < (int)steps + layers - 1; ++s) {
    a.s = s;
    lstm_stack_fwd_step<<<grid, 256, 0, st>>>(a);
  }
  return launch_status("fs2_lstm_stack_fwd");
}

int fs2_lstm_stack_bwd(const float* dh_out, int64_t n_seq, int64_t steps, int64_t c_in,
                       int64_t hidden, int layers, const float* w_ih0_t, const float* w_ih_up_t,
                       const float* w_hh_t, const float* act, const float* c_all, float* dgates,
                       float* dc_ws, float* dx, void* stream) {
  FS2_CHECK_ARG(hidden > 0 && hidden % 256 == 0 && layers >= 1,
                "fs2_lstm_stack_bwd: hidden %lld (multiple of 256), layers >= 1",
                (long long)hidden);
  FS2_CHECK_ARG(layers == 1 || w_ih_up_t, "fs2_lstm_stack_bwd: w_ih_up_t needed for layers > 1");
  if (n_seq == 0 || steps == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)(hidden / 16), (unsigned)((n_seq + 15) / 16), (unsigned)layers);
  LstmStackBwd a{dh_out, w_ih_up_t, w_hh_t, act, c_all, dgates, dc_ws, (int)n_seq, (int)steps,
                 (int)hidden, layers, 0};
  for (int s = 0; s < (int)steps + layers - 1; ++s) {
    a.s = s;
    lstm_stack_bwd_step<<<grid, 512, 0, st>>>(a);
  }
  int rc = launch_status("fs2_lstm_stack_bwd");
  if (rc || !dx) return rc;
  const int64_t rows = n_seq * steps;
  return fs2_conv_gemm(FS2_F32, dgates, 4 * hidden, w_ih0_t, dx, c_in, rows, rows, 4 * hidden,
                       c_in, 1, 0, nullptr, nullptr, 0, nullptr, 0, stream);
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
