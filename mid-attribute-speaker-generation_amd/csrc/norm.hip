// LayerNorm (FFT blocks, variance predictors) and training-mode BatchNorm (PostNet).
//
// LayerNorm: one half-wave (32 lanes) per 256-wide row, 8 consecutive channels per lane
// (two 16-B loads, ONE Philox call for the 8 dropout draws: dropout8), half-wave shuffle
// mean/variance.  The call-site
// epilogues of the reference are fused in: dropout + residual before the norm
// (SubLayers.py:54-55,91-93), padded-row zeroing after it (Layers.py:25,28), dropout
// after it and the Linear(256 -> 1) head of the variance predictor (modules.py:209-250).
// Backward recomputes nothing but the dropout masks: xhat and rstd are saved.
// Affine/linear-head gradients are reduced per 32-row block in registers + LDS and then
// summed over blocks in a fixed order (bitwise reproducible).
//
// BatchNorm: column statistics over every (utterance, frame) row, padded frames included (the
// reference's BatchNorm1d sees them, Layers.py:129-137): per 64-row block its sum and centred
// second moment in one pass, combined exactly over the blocks in a fixed order.
#include <math.h>

#include "common.hpp"

namespace fs2 {

constexpr int LN_D = 256;
constexpr int LN_ROWS = 32;  // rows per block in the backward (2 row pairs per wave of 8)

struct LnFwd {
  const float* y;
  const float* res;
  const float* gamma;
  const float* beta;
  float* out;
  float* xhat;
  float* rstd;
  const int64_t* lens;
  int64_t T, rows;
  float p_in, p_out;
  const uint64_t* seed;  // device (read once per thread; NULL when no dropout)
  uint64_t site_in, site_out;
  const float* dot_w;
  const float* dot_b;
  float* dot_out;
  unsigned short* out_t;  // optional bf16 copy of out
};

FS2_DEV bool row_padded(const int64_t* lens, int64_t T, int64_t r) {
  if (!lens) return false;
  const int64_t b = r / T;
  return (r - b * T) >= lens[b];
}

// rows r = 8 * (blockIdx.x + k * gridDim.x) + half-wave index (grid-stride: the dropout key,
// gamma and beta are fetched once per half-wave, not once per row)
__global__ __launch_bounds__(256) void ln_fwd_f32(LnFwd a) {
  const int hl = threadIdx.x & 31;  // lane within the row's half-wave
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  const f32x4 ga0 = ld4(a.gamma + 8 * hl), ga1 = ld4(a.gamma + 8 * hl + 4);
  const f32x4 be0 = ld4(a.beta + 8 * hl), be1 = ld4(a.beta + 8 * hl + 4);
  for (int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); r < a.rows;
       r += (int64_t)gridDim.x * 8) {
  const int64_t e0 = r * LN_D + 8 * hl;
  const bool pad = row_padded(a.lens, a.T, r);
  if (pad && !a.dot_out) {  // masked row: output 0; xhat/rstd are never read (bwd skips it)
    const f32x4 zz = {0.f, 0.f, 0.f, 0.f};
    st4(a.out + e0, zz);
    st4(a.out + e0 + 4, zz);
    if (a.out_t) st8_bf16(a.out_t + e0, zz, zz);
    continue;
  }
  f32x4 z0 = ld4(a.y + e0), z1 = ld4(a.y + e0 + 4);
  if (a.p_in > 0.f) {
    f32x4 m0, m1;
    dropout8(seed, a.site_in, (uint64_t)e0, a.p_in, m0, m1);
    z0 *= m0;
    z1 *= m1;
  }
  if (a.res) {
    z0 += ld4(a.res + e0);
    z1 += ld4(a.res + e0 + 4);
  }
  const float mean = half_sum((z0.x + z0.y + z0.z + z0.w) + (z1.x + z1.y + z1.z + z1.w)) * (1.f / LN_D);
  const f32x4 c0 = z0 - mean, c1 = z1 - mean;
  const float var = half_sum((c0.x * c0.x + c0.y * c0.y + c0.z * c0.z + c0.w * c0.w) +
                             (c1.x * c1.x + c1.y * c1.y + c1.z * c1.z + c1.w * c1.w)) * (1.f / LN_D);
  const float rs = 1.f / sqrtf(var + 1e-5f);
  const f32x4 xh0 = c0 * rs, xh1 = c1 * rs;
  f32x4 u0 = xh0 * ga0 + be0;
  f32x4 u1 = xh1 * ga1 + be1;
  if (a.p_out > 0.f) {
    f32x4 m0, m1;
    dropout8(seed, a.site_out, (uint64_t)e0, a.p_out, m0, m1);
    u0 *= m0;
    u1 *= m1;
  }
  st4(a.out + e0, u0);  // (dot mode masks only the head output)
  st4(a.out + e0 + 4, u1);
  if (a.out_t) st8_bf16(a.out_t + e0, u0, u1);
  st4(a.xhat + e0, xh0);
  st4(a.xhat + e0 + 4, xh1);
  if (hl == 0) a.rstd[r] = rs;
  if (a.dot_out) {
    const f32x4 w0 = ld4(a.dot_w + 8 * hl), w1 = ld4(a.dot_w + 8 * hl + 4);
    const float d = half_sum((u0.x * w0.x + u0.y * w0.y + u0.z * w0.z + u0.w * w0.w) +
                             (u1.x * w1.x + u1.y * w1.y + u1.z * w1.z + u1.w * w1.w));
    if (hl == 0) a.dot_out[r] = pad ? 0.f : d + a.dot_b[0];
  }
  }
}

struct LnBwd {
  const float* dout;
  const float* ddot;
  const float* dot_w;
  const float* xhat;
  const float* rstd;
  const float* gamma;
  const float* beta;
  const int64_t* lens;
  int64_t T, rows;
  float p_in, p_out;
  const uint64_t* seed;
  uint64_t site_in, site_out;
  const float* relu_y;
  float* dy;
  float* dres;
  int dres_add;  // 1: dres += dz ; 0: dres = dz
  float* part;  // [3][nblk][256] dgamma, dbeta, dw_dot partials, then [nblk] db_dot partials
  int64_t nblk;
  unsigned short* dy_t;  // optional bf16 copy of dy
};

// Row pairs: half-wave h of a wave takes row 2i + h, 8 channels per lane.  Column partials
// (8 per lane) are combined over the NSLOT = 16 half-waves (8 waves x 2) of the block through
// LDS in a fixed slot order.
constexpr int LN_BWD_WAVES = 8;  // 8 waves: 3 blocks per CU keep 24 waves' loads in flight

template <bool DDOT>
__global__ __launch_bounds__(LN_BWD_WAVES * 64) void ln_bwd_f32(LnBwd a) {
  constexpr int NSLOT = 2 * LN_BWD_WAVES;
  __shared__ f32x4 red[NSLOT][64];
  __shared__ float redb[NSLOT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int half = lane >> 5, hl = lane & 31, slot = wave * 2 + half;
  const int c8 = 8 * hl;
  const f32x4 gam0 = ld4(a.gamma + c8), gam1 = ld4(a.gamma + c8 + 4);
  const f32x4 bet0 = ld4(a.beta + c8), bet1 = ld4(a.beta + c8 + 4);
  const f32x4 zz = {0.f, 0.f, 0.f, 0.f};
  f32x4 w0 = zz, w1 = zz;
  if constexpr (DDOT) {
    w0 = ld4(a.dot_w + c8);
    w1 = ld4(a.dot_w + c8 + 4);
  }
  f32x4 pg0 = zz, pg1 = zz, pb0 = zz, pb1 = zz, pw0 = zz, pw1 = zz, py0 = zz, py1 = zz;
  float pdb = 0.f;
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  const int64_t rbeg = (int64_t)blockIdx.x * LN_ROWS;
  // Every row pair of the wave is loaded before the first is reduced: the grid is only a
  // few blocks per CU, so the loads of all IT = LN_ROWS / NSLOT iterations must be in flight together
  // (one pair at a time left the kernel latency-bound at ~1 TB/s).
  constexpr int IT = LN_ROWS / NSLOT;
  f32x4 XH[IT][2], DU[IT][2], DR[IT][2];  // DR: the residual gradient added to (dres_add)
  float RS[IT], RD[IT];
  bool LIVE[IT];
  const bool dres_rd = a.dres && a.dres_add;
  // the row loads of iteration `it` (issued for all iterations up front, except with DDOT:
  // there each row is loaded right before it is reduced -- see DESIGN.md section 4,
  // "intermittent LayerNorm-backward rows")
  auto load_row = [&](int it) {
    const int64_t r = rbeg + 2 * (wave + LN_BWD_WAVES * it) + half;
    LIVE[it] = r < a.rows && !row_padded(a.lens, a.T, r);
    XH[it][0] = XH[it][1] = DU[it][0] = DU[it][1] = DR[it][0] = DR[it][1] = zz;
    RS[it] = RD[it] = 0.f;
    if (LIVE[it]) {
      const int64_t e0 = r * LN_D + c8;
      RD[it] = a.rstd[r];
      XH[it][0] = ld4(a.xhat + e0);
      XH[it][1] = ld4(a.xhat + e0 + 4);
      if (dres_rd) {  // fetched with the row, not after its reduction (a second latency wait)
        DR[it][0] = ld4(a.dres + e0);
        DR[it][1] = ld4(a.dres + e0 + 4);
      }
      if constexpr (DDOT) {
        RS[it] = a.ddot[r];  // the dot gradient rides in RS until the row is reduced
      } else {
        DU[it][0] = ld4(a.dout + e0);
        DU[it][1] = ld4(a.dout + e0 + 4);
      }
    }
  };
  if constexpr (!DDOT) {
#pragma unroll
    for (int it = 0; it < IT; ++it) load_row(it);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if constexpr (DDOT) load_row(it);
    const int64_t r = rbeg + 2 * (wave + LN_BWD_WAVES * it) + half;
    if (r >= a.rows) break;
    const int64_t e0 = r * LN_D + c8;
    if (!LIVE[it]) {  // masked row: zero upstream gradient, nothing to add
      if (a.dres && !a.dres_add) {
        st4(a.dres + e0, zz);
        st4(a.dres + e0 + 4, zz);
      }
      if (a.dy) {
        st4(a.dy + e0, zz);
        st4(a.dy + e0 + 4, zz);
      }
      if (a.dy_t) st8_bf16(a.dy_t + e0, zz, zz);
      continue;
    }
    const f32x4 xh0 = XH[it][0], xh1 = XH[it][1];
    f32x4 mo0 = {1.f, 1.f, 1.f, 1.f}, mo1 = mo0;
    if (a.p_out > 0.f) dropout8(seed, a.site_out, (uint64_t)e0, a.p_out, mo0, mo1);
    f32x4 du0, du1;
    if constexpr (DDOT) {
      const float gr = RS[it];
      du0 = gr * w0;
      du1 = gr * w1;
      pw0 += gr * ((xh0 * gam0 + bet0) * mo0);
      pw1 += gr * ((xh1 * gam1 + bet1) * mo1);
      pdb += gr;
    } else {
      du0 = DU[it][0];
      du1 = DU[it][1];
    }
    du0 *= mo0;
    du1 *= mo1;
    pg0 += du0 * xh0;
    pg1 += du1 * xh1;
    pb0 += du0;
    pb1 += du1;
    const f32x4 dxh0 = du0 * gam0, dxh1 = du1 * gam1;
    const float m1 = half_sum((dxh0.x + dxh0.y + dxh0.z + dxh0.w) + (dxh1.x + dxh1.y + dxh1.z + dxh1.w)) *
                     (1.f / LN_D);
    const float m2 = half_sum((dxh0.x * xh0.x + dxh0.y * xh0.y + dxh0.z * xh0.z + dxh0.w * xh0.w) +
                              (dxh1.x * xh1.x + dxh1.y * xh1.y + dxh1.z * xh1.z + dxh1.w * xh1.w)) *
                     (1.f / LN_D);
    const float rs = RD[it];
    const f32x4 dz0 = rs * (dxh0 - m1 - xh0 * m2), dz1 = rs * (dxh1 - m1 - xh1 * m2);
    if (a.dres) {
      st4(a.dres + e0, a.dres_add ? DR[it][0] + dz0 : dz0);
      st4(a.dres + e0 + 4, a.dres_add ? DR[it][1] + dz1 : dz1);
    }
    f32x4 dy0 = dz0, dy1 = dz1;
    if (a.p_in > 0.f) {
      f32x4 mi0, mi1;
      dropout8(seed, a.site_in, (uint64_t)e0, a.p_in, mi0, mi1);
      dy0 *= mi0;
      dy1 *= mi1;
    }
    if (a.relu_y) {
      const f32x4 y0 = ld4(a.relu_y + e0), y1 = ld4(a.relu_y + e0 + 4);
      dy0 = f32x4{y0.x > 0.f ? dy0.x : 0.f, y0.y > 0.f ? dy0.y : 0.f, y0.z > 0.f ? dy0.z : 0.f,
                  y0.w > 0.f ? dy0.w : 0.f};
      dy1 = f32x4{y1.x > 0.f ? dy1.x : 0.f, y1.y > 0.f ? dy1.y : 0.f, y1.z > 0.f ? dy1.z : 0.f,
                  y1.w > 0.f ? dy1.w : 0.f};
    }
    if (a.dy) {
      st4(a.dy + e0, dy0);
      st4(a.dy + e0 + 4, dy1);
    }
    if (a.dy_t) st8_bf16(a.dy_t + e0, dy0, dy1);
    py0 += dy0;  // bias gradient of the layer that produced y (fused colsum)
    py1 += dy1;
  }
  // per kind: red[slot][q], f32x4 q covers channels 4q..4q+3 (lane hl owns q = 2hl, 2hl+1);
  // wave 0 sums the NSLOT = 16 half-waves in slot order
  auto flush = [&](f32x4 lo, f32x4 hi, int kind) {
    red[slot][2 * hl] = lo;
    red[slot][2 * hl + 1] = hi;
    __syncthreads();
    if (wave == 0) {
      f32x4 sum = red[0][lane];
#pragma unroll
      for (int q = 1; q < NSLOT; ++q) sum += red[q][lane];
      st4(a.part + ((int64_t)kind * a.nblk + blockIdx.x) * LN_D + 4 * lane, sum);
    }
    __syncthreads();
  };
  flush(pg0, pg1, 0);
  flush(pb0, pb1, 1);
  if constexpr (DDOT) flush(pw0, pw1, 2);
  flush(py0, py1, 3);
  if (hl == 0) redb[slot] = pdb;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = redb[0];
#pragma unroll
    for (int q = 1; q < NSLOT; ++q) b += redb[q];
    a.part[4 * a.nblk * LN_D + blockIdx.x] = b;
  }
}

// ------------------------------------------------------------------ BatchNorm
constexpr int BN_ROWS = 64;  // rows per partial block: 1,536 blocks at 24,576 rows (latency-bound at 64)

// in-order column sum of partial rows: 32 columns x 32 part lanes per block, 8 loads in flight
// per lane (the 64 x 16 layout with 4 took 24 dependent rounds at the PostNet's 384 parts)
FS2_DEV float col_reduce(const float* part, int64_t nparts, int64_t c, int64_t col, int tx, int ty,
                         float (*red)[33]) {
  float s = 0.f;
  if (col < c) {
#pragma unroll 8
    for (int64_t p = ty; p < nparts; p += 32) s += part[p * c + col];
  }
  red[ty][tx] = s;
  __syncthreads();
  float t = 0.f;
  if (ty == 0) {
#pragma unroll
    for (int y = 0; y < 32; ++y) t += red[y][tx];
  }
  __syncthreads();
  return t;
}

// Both statistics in one pass over z: a block sums its BN_ROWS rows per column (four row lanes,
// added in lane order, as the round-2 mean pass did, so the mean is unchanged), then forms its
// centred second moment M2_b = sum_r (z - mean_b)^2 from the same values held in registers.  bn_stats_final
// combines the blocks exactly: M2 = sum_b [M2_b + n_b (mean_b - mean)^2] (one launch and one HBM
// pass of z fewer than the mean-then-variance pair, and no cancellation).
__global__ __launch_bounds__(256) void bn_stats(const float* z, int64_t rows, int64_t c, float* psum,
                                                float* pm2) {
  const int tx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t col = ((int64_t)blockIdx.x * 64 + tx) * 4;
  const int64_t r0 = (int64_t)blockIdx.y * BN_ROWS;
  const int64_t r1 = r0 + BN_ROWS < rows ? r0 + BN_ROWS : rows;
  __shared__ f32x4 red[4][64];
  // the thread's BN_ROWS / 4 row values stay in registers for the second moment (a re-read
  // from L2 missed on ~40 % of the bytes with every block of the grid in flight)
  constexpr int RPT = BN_ROWS / 4;
  f32x4 v[RPT];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int64_t r = r0 + ry + 4 * i;
    v[i] = (col < c && r < r1) ? ld4(z + r * c + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) s += v[i];
  red[ry][tx] = s;
  __syncthreads();
  const f32x4 tot = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
  const f32x4 mu = tot * (1.f / (float)(r1 - r0));
  __syncthreads();
  f32x4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    if (r0 + ry + 4 * i < r1) {
      const f32x4 d = v[i] - mu;
      q += d * d;
    }
  }
  red[ry][tx] = q;
  __syncthreads();
  if (ry == 0 && col < c) {
    st4(psum + (int64_t)blockIdx.y * c + col, tot);
    st4(pm2 + (int64_t)blockIdx.y * c + col, ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]);
  }
}

// mean (in-order sum of the block sums), the exact block combination of the variance, rstd and
// the running-statistics update, in one launch
__global__ __launch_bounds__(1024) void bn_stats_final(const float* psum, const float* pm2,
                                                       int64_t nparts, int64_t rows, int64_t c,
                                                       float eps, float mom, float* mean, float* rm,
                                                       float* rv, float* rstd, int64_t* nbt) {
  __shared__ float red[32][33];
  __shared__ float mu_s[32];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t col = (int64_t)blockIdx.x * 32 + tx;
  const float s = col_reduce(psum, nparts, c, col, tx, ty, red);
  if (ty == 0) mu_s[tx] = s / (float)rows;
  __syncthreads();
  const float mu = mu_s[tx];
  float q = 0.f;
  if (col < c) {
#pragma unroll 8
    for (int64_t p = ty; p < nparts; p += 32) {
      const int64_t left = rows - p * BN_ROWS;
      const float n = (float)(left < BN_ROWS ? left : BN_ROWS);
      const float d = psum[p * c + col] / n - mu;
      q += pm2[p * c + col] + n * d * d;
    }
  }
  red[ty][tx] = q;
  __syncthreads();
  if (ty != 0 || col >= c) return;
  float t = 0.f;
#pragma unroll
  for (int y = 0; y < 32; ++y) t += red[y][tx];
  const float var = t / (float)rows;
  mean[col] = mu;
  rstd[col] = 1.f / sqrtf(var + eps);
  if (rm) rm[col] = (1.f - mom) * rm[col] + mom * mu;
  if (rv) rv[col] = (1.f - mom) * rv[col] + mom * (rows > 1 ? t / (float)(rows - 1) : var);
  if (nbt && col == 0) nbt[0] += 1;
}

// tanh(x) = 1 - 2 / (exp(2x) + 1) on v_exp_f32 / v_rcp_f32: absolute error ~3e-7 (|tanh| <= 1;
// saturates to +-1 through exp's overflow / underflow), against the libm tanhf's ~30-instruction
// branchy path -- the PostNet BatchNorm kernels evaluate it on every element (forward, and
// again in both backward passes for the derivative 1 - t^2).  That absolute error is a large
// RELATIVE error near 0 (1e-3 at |x| = 1e-4, and |x| < ~1e-7 collapses to 0), so |x| < 1/8
// takes the odd Taylor polynomial x (1 - x^2/3 + 2x^4/15 - 17x^6/315): its first dropped term
// is 62 x^9 / 2835, a relative error below 2e-9 there (and the exp form's relative error above
// 1/8 is below 3e-6)
FS2_DEV float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // exp(2x) = 2^(2x log2 e)
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  const float x2 = x * x;
  const float s = x * fmaf(x2, fmaf(x2, fmaf(x2, -0.053968254f, 0.13333334f), -0.33333334f), 1.f);
  return fabsf(x) < 0.125f ? s : t;
}
FS2_DEV f32x4 tanh4(f32x4 v) {
  return f32x4{tanh_fast(v.x), tanh_fast(v.y), tanh_fast(v.z), tanh_fast(v.w)};
}


// out = act(BN(z)) * dropout (+ res), 8 consecutive elements (same row) per lane
__global__ __launch_bounds__(256) void bn_apply(const float* z, const float* mean, const float* rstd,
                                                const float* gamma, const float* beta, int64_t n8,
                                                int c, int act_tanh, float p, const uint64_t* seed_p,
                                                uint64_t site, const float* res, float* out,
                                                unsigned short* out_t) {
  const uint64_t seed = seed_p ? *seed_p : 0ull;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n8;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e0 = q * 8;
    const int col = (int)(e0 % c);
    f32x4 v0 = (ld4(z + e0) - ld4(mean + col)) * ld4(rstd + col) * ld4(gamma + col) + ld4(beta + col);
    f32x4 v1 = (ld4(z + e0 + 4) - ld4(mean + col + 4)) * ld4(rstd + col + 4) * ld4(gamma + col + 4) +
               ld4(beta + col + 4);
    if (act_tanh) {
      v0 = tanh4(v0);
      v1 = tanh4(v1);
    }
    if (p > 0.f) {
      f32x4 m0, m1;
      dropout8(seed, site, (uint64_t)e0, p, m0, m1);
      v0 *= m0;
      v1 *= m1;
    }
    if (res) {
      v0 += ld4(res + e0);
      v1 += ld4(res + e0 + 4);
    }
    if (out) {
      st4(out + e0, v0);
      st4(out + e0 + 4, v1);
    }
    if (out_t) st8_bf16(out_t + e0, v0, v1);
  }
}

// g = dout * mask * act'(a) for 8 consecutive elements (one Philox call); also returns xhat
FS2_DEV void bn_g8(const float* dout, const float* z, const float* mean, const float* rstd,
                   const float* gamma, const float* beta, int col, int act_tanh, float p,
                   uint64_t seed, uint64_t site, int64_t e0, f32x4 (&g)[2], f32x4 (&xh)[2]) {
  f32x4 m[2] = {{1.f, 1.f, 1.f, 1.f}, {1.f, 1.f, 1.f, 1.f}};
  if (p > 0.f) dropout8(seed, site, (uint64_t)e0, p, m[0], m[1]);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cc = col + 4 * h;
    xh[h] = (ld4(z + e0 + 4 * h) - ld4(mean + cc)) * ld4(rstd + cc);
    g[h] = ld4(dout + e0 + 4 * h) * m[h];
    if (act_tanh) {
      const f32x4 t = tanh4(xh[h] * ld4(gamma + cc) + ld4(beta + cc));
      g[h] *= 1.f - t * t;
    }
  }
}

// column partials of g and g*xhat over the BN_BWD_ROWS rows of block x.  The lane layout follows
// the width: cg = c / 8 column groups (8 channels per lane) x rl row lanes (host: the largest
// power of two with cg * rl <= 512, rl <= BN_BWD_ROWS), so the 80-channel PostNet output keeps
// 320 lanes busy rather than 10 of 64.  Row lane ry takes rows r0 + ry + rl*i in order, loading
// BN_BWD_BATCH rows of dout and z before any arithmetic, and the row-lane partials are summed in
// row-lane order.  32-row blocks (768 at the SYN-48 shape, all resident at 121 VGPRs) measured
// 21.8 / 7.7 us at c = 512 / 80 against 26.6 / 12.8 us for 64-row blocks of one-row-at-a-time
// waves (16-row blocks: 24.0 / 10.3 us, the finals then read twice the parts).
constexpr int BN_BWD_BATCH = 2;  // rows loaded ahead per lane
constexpr int BN_BWD_ROWS = 32;  // rows per partial block of the backward
__global__ __launch_bounds__(512) void bn_bwd_partial(const float* dout, const float* z,
                                                      const float* mean, const float* rstd,
                                                      const float* gamma, const float* beta,
                                                      int64_t rows, int64_t c, int rl,
                                                      int act_tanh, float p, const uint64_t* seed_p,
                                                      uint64_t site, float* part_g, float* part_gx) {
  const uint64_t seed = seed_p ? *seed_p : 0ull;
  const int cg = (int)(c >> 3);
  const int t = threadIdx.x, gx = t % cg, ry = t / cg;
  const int col = gx * 8;
  const int64_t r0 = (int64_t)blockIdx.x * BN_BWD_ROWS;
  const int64_t r1 = r0 + BN_BWD_ROWS < rows ? r0 + BN_BWD_ROWS : rows;
  __shared__ f32x4 red[2][1024];
  f32x4 sg[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, sgx[2] = {sg[0], sg[0]};
  if (ry < rl) {
    f32x4 mu[2], rs[2], ga[2], be[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      mu[h] = ld4(mean + col + 4 * h);
      rs[h] = ld4(rstd + col + 4 * h);
      ga[h] = ld4(gamma + col + 4 * h);
      be[h] = ld4(beta + col + 4 * h);
    }
    for (int64_t rb = r0 + ry; rb < r1; rb += (int64_t)rl * BN_BWD_BATCH) {
      f32x4 dv[BN_BWD_BATCH][2], zv[BN_BWD_BATCH][2];
#pragma unroll
      for (int i = 0; i < BN_BWD_BATCH; ++i) {
        const int64_t r = rb + (int64_t)rl * i;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          dv[i][h] = r < r1 ? ld4(dout + r * c + col + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
          zv[i][h] = r < r1 ? ld4(z + r * c + col + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int i = 0; i < BN_BWD_BATCH; ++i) {
        const int64_t r = rb + (int64_t)rl * i;
        if (r >= r1) break;
        f32x4 m[2] = {{1.f, 1.f, 1.f, 1.f}, {1.f, 1.f, 1.f, 1.f}};
        if (p > 0.f) dropout8(seed, site, (uint64_t)(r * c + col), p, m[0], m[1]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // g = dout * mask * act'(a), xhat = (z - mean) * rstd
          const f32x4 xh = (zv[i][h] - mu[h]) * rs[h];
          f32x4 g = dv[i][h] * m[h];
          if (act_tanh) {
            const f32x4 th = tanh4(xh * ga[h] + be[h]);
            g *= 1.f - th * th;
          }
          sg[h] += g;
          sgx[h] += g * xh;
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    red[0][2 * t + h] = sg[h];
    red[1][2 * t + h] = sgx[h];
  }
  __syncthreads();
  if (t < cg) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f32x4 a = red[0][2 * t + h], b = red[1][2 * t + h];
      for (int y = 1; y < rl; ++y) {
        a += red[0][2 * (y * cg + t) + h];
        b += red[1][2 * (y * cg + t) + h];
      }
      st4(part_g + (int64_t)blockIdx.x * c + col + 4 * h, a);
      st4(part_gx + (int64_t)blockIdx.x * c + col + 4 * h, b);
    }
  }
}

// in-order column sums of two partial arrays at once: 32 columns x 32 part lanes per block, so
// each lane has nparts / 32 loads of each array in flight (the 64 x 16 layout ran two serial
// reductions of 24 dependent rounds each: ~10 us at the PostNet's 384 parts)
FS2_DEV void col_reduce2(const float* pa, const float* pb, int64_t nparts, int64_t c, int64_t col,
                         int tx, int ty, float (*red)[2][33], float& sa, float& sb) {
  float a = 0.f, b = 0.f;
  if (col < c) {
#pragma unroll 8
    for (int64_t p = ty; p < nparts; p += 32) {
      a += pa[p * c + col];
      b += pb[p * c + col];
    }
  }
  red[ty][0][tx] = a;
  red[ty][1][tx] = b;
  __syncthreads();
  sa = sb = 0.f;
  if (ty == 0) {
#pragma unroll
    for (int y = 0; y < 32; ++y) {
      sa += red[y][0][tx];
      sb += red[y][1][tx];
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void bn_bwd_final(const float* part_g, const float* part_gx,
                                                     int64_t nparts, int64_t c, float* sums,
                                                     float* dgamma, float* dbeta) {
  __shared__ float red[32][2][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int64_t col = (int64_t)blockIdx.x * 32 + tx;
  float sg, sgx;
  col_reduce2(part_g, part_gx, nparts, c, col, tx, ty, red, sg, sgx);
  if (ty != 0 || col >= c) return;
  sums[col] = sg;
  sums[c + col] = sgx;
  if (dbeta) dbeta[col] += sg;
  if (dgamma) dgamma[col] += sgx;
}

__global__ __launch_bounds__(256) void bn_bwd_apply(const float* dout, const float* z,
                                                    const float* mean, const float* rstd,
                                                    const float* gamma, const float* beta,
                                                    const float* sums, int64_t n8, int64_t rows,
                                                    int c, int act_tanh, float p,
                                                    const uint64_t* seed_p, uint64_t site, float* dz,
                                                    unsigned short* dz_t) {
  const uint64_t seed = seed_p ? *seed_p : 0ull;
  const float inv_m = 1.f / (float)rows;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n8;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e0 = q * 8;
    const int col = (int)(e0 % c);
    f32x4 g[2], xh[2], v[2];
    bn_g8(dout, z, mean, rstd, gamma, beta, col, act_tanh, p, seed, site, e0, g, xh);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cc = col + 4 * h;
      v[h] = ld4(gamma + cc) * ld4(rstd + cc) *
             (g[h] - ld4(sums + cc) * inv_m - xh[h] * ld4(sums + c + cc) * inv_m);
    }
    if (dz) {
      st4(dz + e0, v[0]);
      st4(dz + e0 + 4, v[1]);
    }
    if (dz_t) st8_bf16(dz_t + e0, v[0], v[1]);
  }
}

static unsigned ew_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace fs2

using namespace fs2;

extern "C" {

// dtype selects the storage of the optional compute copies (out_t / dy_t / dz_t):
// FS2_F32 = none (the fp32 tensors are the GEMM operands), FS2_BF16 = bf16 copies.
static int copy_dtype_ok(int dtype, const char* what) {
  if (dtype == FS2_F32 || dtype == FS2_BF16) return FS2_OK;
  set_error("%s: dtype %d not built", what, dtype);
  return FS2_ERR_DTYPE;
}

int fs2_ln_fwd(int dtype, const float* y, const float* res, const float* gamma, const float* beta,
               float* out, void* out_t, float* xhat, float* rstd, const int64_t* lens,
               int64_t seq_len, int64_t rows, int d, float p_in, float p_out,
               const uint64_t* seed, uint64_t site_in, uint64_t site_out, const float* dot_w,
               const float* dot_b,
               float* dot_out, void* stream) {
  if (int rc = copy_dtype_ok(dtype, "fs2_ln_fwd")) return rc;
  FS2_CHECK_ARG(d == LN_D, "fs2_ln_fwd: only d = 256 is supported (got %d)", d);
  FS2_CHECK_ARG(!lens || seq_len > 0, "fs2_ln_fwd: lens given without seq_len");
  FS2_CHECK_ARG(!dot_out || (dot_w && dot_b), "fs2_ln_fwd: dot_out needs dot_w/dot_b");
  if (rows == 0) return FS2_OK;
  LnFwd a{y, res, gamma, beta, out, xhat, rstd, lens, seq_len, rows, p_in, p_out, seed,
          site_in, site_out, dot_w, dot_b, dot_out,
          dtype == FS2_BF16 ? (unsigned short*)out_t : nullptr};
  int64_t nb = (rows + 7) / 8;
  if (nb > 2048) nb = 2048;  // 8 blocks per CU, grid-stride beyond
  ln_fwd_f32<<<(unsigned)nb, 256, 0, as_stream(stream)>>>(a);
  return launch_status("fs2_ln_fwd");
}

int64_t fs2_ln_bwd_ws_bytes(int64_t rows, int d) {
  const int64_t nblk = (rows + LN_ROWS - 1) / LN_ROWS;
  return (4 * nblk * (int64_t)d + nblk) * 4;
}

int fs2_ln_bwd(int dtype, const float* dout, const float* ddot, const float* dot_w,
               const float* xhat, const float* rstd, const float* gamma, const float* beta,
               const int64_t* lens, int64_t seq_len, int64_t rows, int d, float p_in, float p_out,
               const uint64_t* seed, uint64_t site_in, uint64_t site_out, const float* relu_y,
               float* dy,
               void* dy_t, float* dres, int dres_add, float* dgamma, float* dbeta, float* dw_dot,
               float* db_dot, float* dbias_in, float* ws, int64_t ws_bytes, void* stream) {
  if (int rc = copy_dtype_ok(dtype, "fs2_ln_bwd")) return rc;
  FS2_CHECK_ARG(d == LN_D, "fs2_ln_bwd: only d = 256 is supported (got %d)", d);
  FS2_CHECK_ARG((dout != nullptr) != (ddot != nullptr), "fs2_ln_bwd: give exactly one of dout/ddot");
  FS2_CHECK_ARG(!ddot || dot_w, "fs2_ln_bwd: ddot needs dot_w");
  FS2_CHECK_ARG(ws_bytes >= fs2_ln_bwd_ws_bytes(rows, d), "fs2_ln_bwd: workspace too small");
  if (rows == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  poison(ws, ws_bytes, st);
  const int64_t nblk = (rows + LN_ROWS - 1) / LN_ROWS;
  LnBwd a{dout, ddot, dot_w, xhat, rstd, gamma, beta, lens, seq_len, rows, p_in, p_out, seed,
          site_in, site_out, relu_y, dy, dres, dres_add, ws, nblk,
          dtype == FS2_BF16 ? (unsigned short*)dy_t : nullptr};
  if (ddot) ln_bwd_f32<true><<<(unsigned)nblk, LN_BWD_WAVES * 64, 0, st>>>(a);
  else ln_bwd_f32<false><<<(unsigned)nblk, LN_BWD_WAVES * 64, 0, st>>>(a);
  int rc = launch_status("fs2_ln_bwd");
  if (rc) return rc;
  return fs2_ln_bwd_final(rows, d, ws, ddot != nullptr, dgamma, dbeta, dw_dot, db_dot, dbias_in,
                          stream);
}

int fs2_ln_bwd_final(int64_t rows, int d, const float* ws, int has_ddot, float* dgamma,
                     float* dbeta, float* dw_dot, float* db_dot, float* dbias_in, void* stream) {
  FS2_CHECK_ARG(d == LN_D, "fs2_ln_bwd_final: only d = 256 is supported (got %d)", d);
  if (rows == 0) return FS2_OK;
  const int64_t nblk = (rows + LN_ROWS - 1) / LN_ROWS;
  float* w = const_cast<float*>(ws);
  ColsumJobs jobs{};
  jobs.acc = 1;
  if (dgamma) jobs.add(w, nblk, LN_D, dgamma);
  if (dbeta) jobs.add(w + nblk * LN_D, nblk, LN_D, dbeta);
  if (has_ddot && dw_dot) jobs.add(w + 2 * nblk * LN_D, nblk, LN_D, dw_dot);
  if (has_ddot && db_dot) jobs.add(w + 4 * nblk * LN_D, nblk, 1, db_dot);
  if (dbias_in) jobs.add(w + 3 * nblk * LN_D, nblk, LN_D, dbias_in);
  return colsum_final_multi_launch(jobs, as_stream(stream));
}

int64_t fs2_bn_ws_bytes(int64_t rows, int64_t c) {
  const int64_t nf = (rows + BN_ROWS - 1) / BN_ROWS, nb = (rows + BN_BWD_ROWS - 1) / BN_BWD_ROWS;
  const int64_t nparts = nf > nb ? nf : nb;
  return (2 * nparts * c + 2 * c) * 4;
}

int fs2_bn_fwd(int dtype, const float* z, int64_t rows, int64_t c, const float* gamma,
               const float* beta, float eps, float momentum, float* running_mean,
               float* running_var, float* mean, float* rstd, int act_tanh, float p,
               const uint64_t* seed, uint64_t site, const float* res, float* out, void* out_t,
               float* ws,
               int64_t ws_bytes, int64_t* num_batches_tracked, void* stream) {
  if (int rc = copy_dtype_ok(dtype, "fs2_bn_fwd")) return rc;
  FS2_CHECK_ARG(rows > 0 && c > 0, "fs2_bn_fwd: empty input");
  FS2_CHECK_ARG(ws_bytes >= fs2_bn_ws_bytes(rows, c), "fs2_bn_fwd: workspace too small");
  hipStream_t st = as_stream(stream);
  poison(ws, ws_bytes, st);
  const int64_t nparts = (rows + BN_ROWS - 1) / BN_ROWS;
  FS2_CHECK_ARG(c % 8 == 0, "fs2_bn_fwd: channel count must be a multiple of 8");
  dim3 grid((unsigned)((c + 255) / 256), (unsigned)nparts);
  const unsigned cg = (unsigned)((c + 31) / 32);
  bn_stats<<<grid, 256, 0, st>>>(z, rows, c, ws, ws + nparts * c);
  bn_stats_final<<<cg, 1024, 0, st>>>(ws, ws + nparts * c, nparts, rows, c, eps, momentum, mean,
                                      running_mean, running_var, rstd, num_batches_tracked);
  unsigned short* ot = dtype == FS2_BF16 ? (unsigned short*)out_t : nullptr;
  FS2_CHECK_ARG(out || ot, "fs2_bn_fwd: no output requested");
  bn_apply<<<ew_grid(rows * c / 8), 256, 0, st>>>(z, mean, rstd, gamma, beta, rows * c / 8, (int)c,
                                                  act_tanh, p, seed, site, res, out, ot);
  return launch_status("fs2_bn_fwd");
}

// eval-mode statistics: mean = running_mean, rstd = 1 / sqrt(running_var + eps)
__global__ void bn_eval_stats(const float* rm, const float* rv, int64_t c, float eps, float* mean,
                              float* rstd) {
  const int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= c) return;
  mean[col] = rm[col];
  rstd[col] = 1.f / sqrtf(rv[col] + eps);
}

int fs2_bn_eval_fwd(int dtype, const float* z, int64_t rows, int64_t c, const float* gamma,
                    const float* beta, float eps, const float* running_mean,
                    const float* running_var, float* mean, float* rstd, int act_tanh,
                    const float* res, float* out, void* out_t, void* stream) {
  if (int rc = copy_dtype_ok(dtype, "fs2_bn_eval_fwd")) return rc;
  FS2_CHECK_ARG(rows > 0 && c > 0 && c % 8 == 0, "fs2_bn_eval_fwd: bad shape (c % 8 == 0)");
  FS2_CHECK_ARG(running_mean && running_var && mean && rstd, "fs2_bn_eval_fwd: null statistics");
  hipStream_t st = as_stream(stream);
  unsigned short* ot = dtype == FS2_BF16 ? (unsigned short*)out_t : nullptr;
  FS2_CHECK_ARG(out || ot, "fs2_bn_eval_fwd: no output requested");
  bn_eval_stats<<<(unsigned)((c + 255) / 256), 256, 0, st>>>(running_mean, running_var, c, eps,
                                                             mean, rstd);
  bn_apply<<<ew_grid(rows * c / 8), 256, 0, st>>>(z, mean, rstd, gamma, beta, rows * c / 8, (int)c,
                                                  act_tanh, 0.f, nullptr, 0, res, out, ot);
  return launch_status("fs2_bn_eval_fwd");
}

int fs2_bn_bwd(int dtype, const float* dout, const float* z, const float* mean, const float* rstd,
               const float* gamma, const float* beta, int64_t rows, int64_t c, int act_tanh,
               float p, const uint64_t* seed, uint64_t site, float* dz, void* dz_t,
               float* dgamma,
               float* dbeta, float* ws, int64_t ws_bytes, void* stream) {
  if (int rc = copy_dtype_ok(dtype, "fs2_bn_bwd")) return rc;
  FS2_CHECK_ARG(rows > 0 && c > 0, "fs2_bn_bwd: empty input");
  FS2_CHECK_ARG(ws_bytes >= fs2_bn_ws_bytes(rows, c), "fs2_bn_bwd: workspace too small");
  hipStream_t st = as_stream(stream);
  poison(ws, ws_bytes, st);
  const int64_t nparts = (rows + BN_BWD_ROWS - 1) / BN_BWD_ROWS;
  float* part_g = ws;
  float* part_gx = ws + nparts * c;
  float* sums = ws + 2 * nparts * c;
  FS2_CHECK_ARG(c % 8 == 0, "fs2_bn_bwd: channel count must be a multiple of 8");
  unsigned short* zt = dtype == FS2_BF16 ? (unsigned short*)dz_t : nullptr;
  FS2_CHECK_ARG(dz || zt, "fs2_bn_bwd: no output requested");
  FS2_CHECK_ARG(c <= 4096, "fs2_bn_bwd: at most 4096 channels (got %lld)", (long long)c);
  int rl = 1;  // row lanes: the largest power of two with (c / 8) * rl <= 512, rl <= BN_ROWS
  while (rl < BN_BWD_ROWS && (c / 8) * rl * 2 <= 512) rl *= 2;
  bn_bwd_partial<<<(unsigned)nparts, 512, 0, st>>>(dout, z, mean, rstd, gamma, beta, rows, c, rl,
                                                   act_tanh, p, seed, site, part_g, part_gx);
  bn_bwd_final<<<(unsigned)((c + 31) / 32), 1024, 0, st>>>(part_g, part_gx, nparts, c, sums,
                                                             dgamma, dbeta);
  bn_bwd_apply<<<ew_grid(rows * c / 8), 256, 0, st>>>(dout, z, mean, rstd, gamma, beta, sums,
                                                      rows * c / 8, rows, (int)c, act_tanh, p,
                                                      seed, site, dz, zt);
  return launch_status("fs2_bn_bwd");
}

}  // extern "C"
