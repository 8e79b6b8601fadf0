// LayerNorm (FFT blocks, variance predictors) and training-mode BatchNorm (PostNet).
//
// LayerNorm: one wave per 256-wide row, 4 consecutive channels per lane (one 16-B load,
// one Philox call for the 4 dropout draws), wave-shuffle mean/variance.  The call-site
// epilogues of the reference are fused in: dropout + residual before the norm
// (SubLayers.py:54-55,91-93), padded-row zeroing after it (Layers.py:25,28), dropout
// after it and the Linear(256 -> 1) head of the variance predictor (modules.py:209-250).
// Backward recomputes nothing but the dropout masks: xhat and rstd are saved.
// Affine/linear-head gradients are reduced per 32-row block in registers + LDS and then
// summed over blocks in a fixed order (bitwise reproducible).
//
// BatchNorm: two-pass column statistics over every (utterance, frame) row, padded frames
// included (the reference's BatchNorm1d sees them, Layers.py:129-137).
#include <math.h>

#include "common.hpp"

namespace fs2 {

constexpr int LN_D = 256;
constexpr int LN_ROWS = 32;  // rows per block in the backward (8 per wave)

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

__global__ __launch_bounds__(256) void ln_fwd_f32(LnFwd a) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.rows) return;
  const int64_t e0 = r * LN_D + 4 * lane;
  const bool pad = row_padded(a.lens, a.T, r);
  if (pad && !a.dot_out) {  // masked row: output 0; xhat/rstd are never read (bwd skips it)
    st4(a.out + e0, f32x4{0.f, 0.f, 0.f, 0.f});
    if (a.out_t) st4_bf16(a.out_t + e0, f32x4{0.f, 0.f, 0.f, 0.f});
    return;
  }
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  f32x4 z = ld4(a.y + e0);
  if (a.p_in > 0.f) z *= dropout4(seed, a.site_in, (uint64_t)e0, a.p_in);
  if (a.res) z += ld4(a.res + e0);
  const float mean = wave_sum(z.x + z.y + z.z + z.w) * (1.f / LN_D);
  const f32x4 c = z - mean;
  const float var = wave_sum(c.x * c.x + c.y * c.y + c.z * c.z + c.w * c.w) * (1.f / LN_D);
  const float rs = 1.f / sqrtf(var + 1e-5f);
  const f32x4 xh = c * rs;
  f32x4 u = xh * ld4(a.gamma + 4 * lane) + ld4(a.beta + 4 * lane);
  if (a.p_out > 0.f) u *= dropout4(seed, a.site_out, (uint64_t)e0, a.p_out);
  st4(a.out + e0, u);  // (dot mode masks only the head output)
  if (a.out_t) st4_bf16(a.out_t + e0, u);
  st4(a.xhat + e0, xh);
  if (lane == 0) a.rstd[r] = rs;
  if (a.dot_out) {
    const f32x4 w = ld4(a.dot_w + 4 * lane);
    const float d = wave_sum(u.x * w.x + u.y * w.y + u.z * w.z + u.w * w.w);
    if (lane == 0) a.dot_out[r] = pad ? 0.f : d + a.dot_b[0];
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

__global__ __launch_bounds__(256) void ln_bwd_f32(LnBwd a) {
  __shared__ f32x4 red[4][4][64];
  __shared__ float redb[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const f32x4 gam = ld4(a.gamma + 4 * lane);
  const f32x4 bet = ld4(a.beta + 4 * lane);
  f32x4 w = {0.f, 0.f, 0.f, 0.f};
  if (a.ddot) w = ld4(a.dot_w + 4 * lane);
  f32x4 pg = {0.f, 0.f, 0.f, 0.f}, pb = pg, pw = pg, py = pg;
  float pdb = 0.f;
  const uint64_t seed = a.seed ? *a.seed : 0ull;
  const int64_t rbeg = (int64_t)blockIdx.x * LN_ROWS;
  for (int i = wave; i < LN_ROWS; i += 4) {
    const int64_t r = rbeg + i;
    if (r >= a.rows) break;
    const int64_t e0 = r * LN_D + 4 * lane;
    if (row_padded(a.lens, a.T, r)) {  // masked row: zero upstream gradient, nothing to add
      if (a.dres && !a.dres_add) st4(a.dres + e0, f32x4{0.f, 0.f, 0.f, 0.f});
      if (a.dy) st4(a.dy + e0, f32x4{0.f, 0.f, 0.f, 0.f});
      if (a.dy_t) st4_bf16(a.dy_t + e0, f32x4{0.f, 0.f, 0.f, 0.f});
      continue;
    }
    const f32x4 xh = ld4(a.xhat + e0);
    const f32x4 mo = a.p_out > 0.f ? dropout4(seed, a.site_out, (uint64_t)e0, a.p_out)
                                   : f32x4{1.f, 1.f, 1.f, 1.f};
    f32x4 du;
    if (a.ddot) {
      const float gr = a.ddot[r];
      du = gr * w;
      const f32x4 u = (xh * gam + bet) * mo;
      pw += gr * u;
      pdb += gr;
    } else {
      du = ld4(a.dout + e0);
    }
    du *= mo;
    pg += du * xh;
    pb += du;
    const f32x4 dxh = du * gam;
    const float m1 = wave_sum(dxh.x + dxh.y + dxh.z + dxh.w) * (1.f / LN_D);
    const float m2 =
        wave_sum(dxh.x * xh.x + dxh.y * xh.y + dxh.z * xh.z + dxh.w * xh.w) * (1.f / LN_D);
    const f32x4 dz = a.rstd[r] * (dxh - m1 - xh * m2);
    if (a.dres) st4(a.dres + e0, a.dres_add ? ld4(a.dres + e0) + dz : dz);
    f32x4 dy = dz;
    if (a.p_in > 0.f) dy *= dropout4(seed, a.site_in, (uint64_t)e0, a.p_in);
    if (a.relu_y) {
      const f32x4 yv = ld4(a.relu_y + e0);
      dy.x = yv.x > 0.f ? dy.x : 0.f;
      dy.y = yv.y > 0.f ? dy.y : 0.f;
      dy.z = yv.z > 0.f ? dy.z : 0.f;
      dy.w = yv.w > 0.f ? dy.w : 0.f;
    }
    if (a.dy) st4(a.dy + e0, dy);
    if (a.dy_t) st4_bf16(a.dy_t + e0, dy);
    py += dy;  // bias gradient of the layer that produced y (fused colsum)
  }
  red[0][wave][lane] = pg;
  red[1][wave][lane] = pb;
  red[2][wave][lane] = pw;
  red[3][wave][lane] = py;
  if (lane == 0) redb[wave] = pdb;
  __syncthreads();
  const f32x4 s = red[wave][0][lane] + red[wave][1][lane] + red[wave][2][lane] + red[wave][3][lane];
  st4(a.part + ((int64_t)wave * a.nblk + blockIdx.x) * LN_D + 4 * lane, s);
  if (threadIdx.x == 0)
    a.part[4 * a.nblk * LN_D + blockIdx.x] = redb[0] + redb[1] + redb[2] + redb[3];
}

// ------------------------------------------------------------------ BatchNorm
constexpr int BN_ROWS = 64;

// Column partial sums over BN_ROWS-row chunks, 4 consecutive channels per lane (16-B loads):
// block (x, y) covers channels [256x, 256x+256) of rows [BN_ROWS*y, BN_ROWS*(y+1)), four row
// lanes summed in lane order.  MODE 0: sum z ; MODE 1: sum (z - mean)^2
template <int MODE>
__global__ __launch_bounds__(256) void bn_partial(const float* z, const float* mean, int64_t rows,
                                                  int64_t c, float* part) {
  const int tx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t col = ((int64_t)blockIdx.x * 64 + tx) * 4;
  const int64_t r0 = (int64_t)blockIdx.y * BN_ROWS;
  __shared__ f32x4 red[4][64];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (col < c) {
    const f32x4 mu = MODE == 1 ? ld4(mean + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t r1 = r0 + BN_ROWS < rows ? r0 + BN_ROWS : rows;
#pragma unroll 4
    for (int64_t r = r0 + ry; r < r1; r += 4) {
      const f32x4 v = ld4(z + r * c + col);
      if (MODE == 0) s += v;
      else s += (v - mu) * (v - mu);
    }
  }
  red[ry][tx] = s;
  __syncthreads();
  if (ry == 0 && col < c)
    st4(part + (int64_t)blockIdx.y * c + col, ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]);
}

// in-order column sum of partial rows: 64 columns x 16 lanes per block (see colsum_final)
FS2_DEV float col_reduce(const float* part, int64_t nparts, int64_t c, int64_t col, int tx, int ty,
                         float (*red)[65]) {
  float s = 0.f;
  if (col < c) {
#pragma unroll 4
    for (int64_t p = ty; p < nparts; p += 16) s += part[p * c + col];
  }
  red[ty][tx] = s;
  __syncthreads();
  float t = 0.f;
  if (ty == 0) {
#pragma unroll
    for (int y = 0; y < 16; ++y) t += red[y][tx];
  }
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(1024) void bn_mean_final(const float* part, int64_t nparts, int64_t rows,
                                                      int64_t c, float* mean) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  const float s = col_reduce(part, nparts, c, col, tx, ty, red);
  if (ty == 0 && col < c) mean[col] = s / (float)rows;
}

__global__ __launch_bounds__(1024) void bn_var_final(const float* part, int64_t nparts, int64_t rows,
                                                     int64_t c, float eps, float mom,
                                                     const float* mean, float* rm, float* rv,
                                                     float* rstd) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  const float s = col_reduce(part, nparts, c, col, tx, ty, red);
  if (ty != 0 || col >= c) return;
  const float var = s / (float)rows;
  rstd[col] = 1.f / sqrtf(var + eps);
  if (rm) rm[col] = (1.f - mom) * rm[col] + mom * mean[col];
  if (rv) rv[col] = (1.f - mom) * rv[col] + mom * (rows > 1 ? s / (float)(rows - 1) : var);
}

// out = act(BN(z)) * dropout (+ res), 4 consecutive elements (same row) per lane
__global__ __launch_bounds__(256) void bn_apply(const float* z, const float* mean, const float* rstd,
                                                const float* gamma, const float* beta, int64_t n4,
                                                int c, int act_tanh, float p, const uint64_t* seed_p,
                                                uint64_t site, const float* res, float* out,
                                                unsigned short* out_t) {
  const uint64_t seed = seed_p ? *seed_p : 0ull;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e0 = q * 4;
    const int col = (int)(e0 % c);
    f32x4 v = (ld4(z + e0) - ld4(mean + col)) * ld4(rstd + col) * ld4(gamma + col) + ld4(beta + col);
    if (act_tanh) v = f32x4{tanhf(v.x), tanhf(v.y), tanhf(v.z), tanhf(v.w)};
    if (p > 0.f) v *= dropout4(seed, site, (uint64_t)e0, p);
    if (res) v += ld4(res + e0);
    if (out) st4(out + e0, v);
    if (out_t) st4_bf16(out_t + e0, v);
  }
}

// g = dout * mask * act'(a) for 4 consecutive elements; also returns xhat
FS2_DEV f32x4 bn_g4(const float* dout, const float* z, f32x4 mu, f32x4 rs, f32x4 ga, f32x4 be,
                    int act_tanh, float p, uint64_t seed, uint64_t site, int64_t e0, f32x4* xh_out) {
  const f32x4 xh = (ld4(z + e0) - mu) * rs;
  *xh_out = xh;
  f32x4 g = ld4(dout + e0);
  if (p > 0.f) g *= dropout4(seed, site, (uint64_t)e0, p);
  if (act_tanh) {
    const f32x4 a = xh * ga + be;
    const f32x4 t = {tanhf(a.x), tanhf(a.y), tanhf(a.z), tanhf(a.w)};
    g *= 1.f - t * t;
  }
  return g;
}

__global__ __launch_bounds__(256) void bn_bwd_partial(const float* dout, const float* z,
                                                      const float* mean, const float* rstd,
                                                      const float* gamma, const float* beta,
                                                      int64_t rows, int64_t c, int act_tanh,
                                                      float p, const uint64_t* seed_p,
                                                      uint64_t site, float* part_g, float* part_gx) {
  const uint64_t seed = seed_p ? *seed_p : 0ull;
  const int tx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t col = ((int64_t)blockIdx.x * 64 + tx) * 4;
  const int64_t r0 = (int64_t)blockIdx.y * BN_ROWS;
  __shared__ f32x4 red[2][4][64];
  f32x4 sg = {0.f, 0.f, 0.f, 0.f}, sgx = sg;
  if (col < c) {
    const f32x4 mu = ld4(mean + col), rs = ld4(rstd + col), ga = ld4(gamma + col),
                be = ld4(beta + col);
    const int64_t r1 = r0 + BN_ROWS < rows ? r0 + BN_ROWS : rows;
    for (int64_t r = r0 + ry; r < r1; r += 4) {
      f32x4 xh;
      const f32x4 g = bn_g4(dout, z, mu, rs, ga, be, act_tanh, p, seed, site, r * c + col, &xh);
      sg += g;
      sgx += g * xh;
    }
  }
  red[0][ry][tx] = sg;
  red[1][ry][tx] = sgx;
  __syncthreads();
  if (ry == 0 && col < c) {
    st4(part_g + (int64_t)blockIdx.y * c + col,
        ((red[0][0][tx] + red[0][1][tx]) + red[0][2][tx]) + red[0][3][tx]);
    st4(part_gx + (int64_t)blockIdx.y * c + col,
        ((red[1][0][tx] + red[1][1][tx]) + red[1][2][tx]) + red[1][3][tx]);
  }
}

__global__ __launch_bounds__(1024) void bn_bwd_final(const float* part_g, const float* part_gx,
                                                     int64_t nparts, int64_t c, float* sums,
                                                     float* dgamma, float* dbeta) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + tx;
  const float sg = col_reduce(part_g, nparts, c, col, tx, ty, red);
  const float sgx = col_reduce(part_gx, nparts, c, col, tx, ty, red);
  if (ty != 0 || col >= c) return;
  sums[col] = sg;
  sums[c + col] = sgx;
  if (dbeta) dbeta[col] += sg;
  if (dgamma) dgamma[col] += sgx;
}

__global__ __launch_bounds__(256) void bn_bwd_apply(const float* dout, const float* z,
                                                    const float* mean, const float* rstd,
                                                    const float* gamma, const float* beta,
                                                    const float* sums, int64_t n4, int64_t rows,
                                                    int c, int act_tanh, float p,
                                                    const uint64_t* seed_p, uint64_t site, float* dz,
                                                    unsigned short* dz_t) {
  const uint64_t seed = seed_p ? *seed_p : 0ull;
  const float inv_m = 1.f / (float)rows;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e0 = q * 4;
    const int col = (int)(e0 % c);
    const f32x4 ga = ld4(gamma + col), rs = ld4(rstd + col);
    f32x4 xh;
    const f32x4 g = bn_g4(dout, z, ld4(mean + col), rs, ga, ld4(beta + col), act_tanh, p, seed,
                          site, e0, &xh);
    const f32x4 v = ga * rs * (g - ld4(sums + col) * inv_m - xh * ld4(sums + c + col) * inv_m);
    if (dz) st4(dz + e0, v);
    if (dz_t) st4_bf16(dz_t + e0, v);
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
  ln_fwd_f32<<<(unsigned)((rows + 3) / 4), 256, 0, as_stream(stream)>>>(a);
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
  const int64_t nblk = (rows + LN_ROWS - 1) / LN_ROWS;
  LnBwd a{dout, ddot, dot_w, xhat, rstd, gamma, beta, lens, seq_len, rows, p_in, p_out, seed,
          site_in, site_out, relu_y, dy, dres, dres_add, ws, nblk,
          dtype == FS2_BF16 ? (unsigned short*)dy_t : nullptr};
  ln_bwd_f32<<<(unsigned)nblk, 256, 0, st>>>(a);
  int rc = launch_status("fs2_ln_bwd");
  if (rc) return rc;
  ColsumJobs jobs{};
  jobs.acc = 1;
  if (dgamma) jobs.add(ws, nblk, LN_D, dgamma);
  if (dbeta) jobs.add(ws + nblk * LN_D, nblk, LN_D, dbeta);
  if (ddot && dw_dot) jobs.add(ws + 2 * nblk * LN_D, nblk, LN_D, dw_dot);
  if (ddot && db_dot) jobs.add(ws + 4 * nblk * LN_D, nblk, 1, db_dot);
  if (dbias_in) jobs.add(ws + 3 * nblk * LN_D, nblk, LN_D, dbias_in);
  return colsum_final_multi_launch(jobs, st);
}

int64_t fs2_bn_ws_bytes(int64_t rows, int64_t c) {
  const int64_t nparts = (rows + BN_ROWS - 1) / BN_ROWS;
  return (2 * nparts * c + 2 * c) * 4;
}

int fs2_bn_fwd(int dtype, const float* z, int64_t rows, int64_t c, const float* gamma,
               const float* beta, float eps, float momentum, float* running_mean,
               float* running_var, float* mean, float* rstd, int act_tanh, float p,
               const uint64_t* seed, uint64_t site, const float* res, float* out, void* out_t,
               float* ws,
               int64_t ws_bytes, void* stream) {
  if (int rc = copy_dtype_ok(dtype, "fs2_bn_fwd")) return rc;
  FS2_CHECK_ARG(rows > 0 && c > 0, "fs2_bn_fwd: empty input");
  FS2_CHECK_ARG(ws_bytes >= fs2_bn_ws_bytes(rows, c), "fs2_bn_fwd: workspace too small");
  hipStream_t st = as_stream(stream);
  const int64_t nparts = (rows + BN_ROWS - 1) / BN_ROWS;
  FS2_CHECK_ARG(c % 4 == 0, "fs2_bn_fwd: channel count must be a multiple of 4");
  dim3 grid((unsigned)((c + 255) / 256), (unsigned)nparts);
  const unsigned cg = (unsigned)((c + 63) / 64);
  bn_partial<0><<<grid, 256, 0, st>>>(z, nullptr, rows, c, ws);
  bn_mean_final<<<cg, 1024, 0, st>>>(ws, nparts, rows, c, mean);
  bn_partial<1><<<grid, 256, 0, st>>>(z, mean, rows, c, ws);
  bn_var_final<<<cg, 1024, 0, st>>>(ws, nparts, rows, c, eps, momentum, mean, running_mean,
                                   running_var, rstd);
  unsigned short* ot = dtype == FS2_BF16 ? (unsigned short*)out_t : nullptr;
  FS2_CHECK_ARG(out || ot, "fs2_bn_fwd: no output requested");
  bn_apply<<<ew_grid(rows * c / 4), 256, 0, st>>>(z, mean, rstd, gamma, beta, rows * c / 4, (int)c,
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
  FS2_CHECK_ARG(rows > 0 && c > 0 && c % 4 == 0, "fs2_bn_eval_fwd: bad shape (c % 4 == 0)");
  FS2_CHECK_ARG(running_mean && running_var && mean && rstd, "fs2_bn_eval_fwd: null statistics");
  hipStream_t st = as_stream(stream);
  unsigned short* ot = dtype == FS2_BF16 ? (unsigned short*)out_t : nullptr;
  FS2_CHECK_ARG(out || ot, "fs2_bn_eval_fwd: no output requested");
  bn_eval_stats<<<(unsigned)((c + 255) / 256), 256, 0, st>>>(running_mean, running_var, c, eps,
                                                             mean, rstd);
  bn_apply<<<ew_grid(rows * c / 4), 256, 0, st>>>(z, mean, rstd, gamma, beta, rows * c / 4, (int)c,
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
  const int64_t nparts = (rows + BN_ROWS - 1) / BN_ROWS;
  float* part_g = ws;
  float* part_gx = ws + nparts * c;
  float* sums = ws + 2 * nparts * c;
  FS2_CHECK_ARG(c % 4 == 0, "fs2_bn_bwd: channel count must be a multiple of 4");
  unsigned short* zt = dtype == FS2_BF16 ? (unsigned short*)dz_t : nullptr;
  FS2_CHECK_ARG(dz || zt, "fs2_bn_bwd: no output requested");
  dim3 grid((unsigned)((c + 255) / 256), (unsigned)nparts);
  bn_bwd_partial<<<grid, 256, 0, st>>>(dout, z, mean, rstd, gamma, beta, rows, c, act_tanh, p,
                                       seed, site, part_g, part_gx);
  bn_bwd_final<<<(unsigned)((c + 63) / 64), 1024, 0, st>>>(part_g, part_gx, nparts, c, sums,
                                                             dgamma, dbeta);
  bn_bwd_apply<<<ew_grid(rows * c / 4), 256, 0, st>>>(dout, z, mean, rstd, gamma, beta, sums,
                                                      rows * c / 4, rows, (int)c, act_tanh, p,
                                                      seed, site, dz, zt);
  return launch_status("fs2_bn_bwd");
}

}  // extern "C"
