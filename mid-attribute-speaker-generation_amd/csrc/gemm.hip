// Implicit-GEMM Conv1d / Linear on MFMA for gfx950.
//
// All matmul-shaped work of the training step goes through two kernels:
//   conv_gemm_nt : y[r, o] = sum_{j,c} wk[o, j*Cin+c] * x[r+j-pad, c]   (forward and dX)
//   conv_wgrad_tn: dw[o, j*Cin+c] = sum_r dy[r, o] * x[r+j-pad, c]      (weight gradient)
// The time shift of each tap is applied in the global->LDS loader (zero outside the
// utterance), so no im2col buffer is ever materialised.  Tiles: 4 waves (2x2), BK = 32,
// register-staged double-buffered LDS (one barrier per k-tile).  fp32 uses the exact
// f32-input MFMA v_mfma_f32_16x16x4_f32 with a k-permutation that lets each lane read 8
// consecutive k (two ds_read_b128) per fragment — the same lane->k pattern the bf16
// 16x16x32 MFMA uses, so both share the LDS image.
#include "common.hpp"

namespace fs2 {

constexpr int BK = 32;
constexpr int LDK = BK + 4;  // padded LDS row (floats) for [row][k] images

struct ConvArgs {
  const float* x;
  int64_t ldx;
  const float* w;
  float* y;
  int64_t ldy;
  int64_t M, T;
  int Cin, N, taps, pad, K;
  const float* bias;
  int flags;
  const float* aux;
  int64_t ld_aux;
  int dil;                 // tap dilation (vocoder); 1 elsewhere
  float alpha, scale;      // FS2_EPI_LRELU slope, FS2_EPI_ACC_Y scale
  float* y2;               // FS2_EPI_Y2 output (ld = N)
  float alpha2;
};

// A-operand loader of the NT kernel: 4 consecutive k of row m with the tap shift applied.
FS2_DEV f32x4 load_conv_a(const ConvArgs& a, int64_t m, int k) {
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (m >= a.M || k >= a.K) return z;
  int j = k / a.Cin;
  int c = k - j * a.Cin;
  int64_t s = m / a.T;
  int64_t t = m - s * a.T + (int64_t)j * a.dil - a.pad;
  if (t < 0 || t >= a.T) return z;
  return ld4(a.x + (s * a.T + t) * a.ldx + c);
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_gemm_nt_f32(ConvArgs a) {
  constexpr int MI = BM / 32, NI = BN / 32;  // 16x16 subtiles per wave (2x2 waves)
  constexpr int ACH = BM * BK / 4 / 256, BCH = BN * BK / 4 / 256;
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nk = (a.K + BK - 1) / BK;

  f32x4 ra[ACH], rb[BCH];
  auto gload = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 4;
      ra[i] = load_conv_a(a, m0 + row, k0 + kq);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 4;
      int n = n0 + row, k = k0 + kq;
      rb[i] = (n < a.N && k < a.K) ? ld4(a.w + (int64_t)n * a.K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 4;
      st4(&As[buf][row * LDK + kq], ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 4;
      st4(&Bs[buf][row * LDK + kq], rb[i]);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    f32x4 fa[MI][2], fb[NI][2];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const float* p = &As[cur][(wm * (BM / 2) + i * 16 + r16) * LDK + 8 * g];
      fa[i][0] = ld4(p);
      fa[i][1] = ld4(p + 4);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const float* p = &Bs[cur][(wn * (BN / 2) + j * 16 + r16) * LDK + 8 * g];
      fb[j][0] = ld4(p);
      fb[j][1] = ld4(p + 4);
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][jj >> 2][jj & 3],
                                                           fb[j][jj >> 2][jj & 3], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: D[row = 4g + r][col = r16] of each 16x16 subtile
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + r16;
      if (n >= a.N) continue;
      const float bv = (a.flags & FS2_EPI_BIAS) ? a.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wm * (BM / 2) + i * 16 + 4 * g + r;
        if (m >= a.M) continue;
        float v = acc[i][j][r] + bv;
        if (a.flags & FS2_EPI_ADD_AUX) v += a.aux[m * a.ld_aux + n];
        if (a.flags & FS2_EPI_ACC_Y) v = (v + a.y[m * a.ldy + n]) * a.scale;
        if (a.flags & FS2_EPI_RELU) v = fmaxf(v, 0.f);
        if (a.flags & FS2_EPI_LRELU) v = v >= 0.f ? v : a.alpha * v;
        if (a.flags & FS2_EPI_RELU_MASK_AUX) v = a.aux[m * a.ld_aux + n] > 0.f ? v : 0.f;
        if (a.y) a.y[m * a.ldy + n] = v;
        if (a.flags & FS2_EPI_Y2) a.y2[m * a.N + n] = v >= 0.f ? v : a.alpha2 * v;
      }
    }
}

// ------------------------------------------------------------------------ weight gradient
struct WgradArgs {
  const float* dy;
  int64_t ldy;
  const float* x;
  int64_t ldx;
  float* slab;  // [splits][Cout][Kp]
  int64_t M, T;
  int Cin, Cout, taps, pad, Kp;  // Kp = taps * Cin (output columns)
  int64_t rows_per_split;
};

template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_wgrad_tn_f32(WgradArgs a) {
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int ACH = BM * BK / 4 / 256, BCH = BN * BK / 4 / 256;
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDA];  // [m][o]
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDB];  // [m][j*Cin+c]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int o0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int64_t r_begin = (int64_t)blockIdx.z * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.M) r_end = a.M;
  const int nk = (int)((r_end - r_begin + BK - 1) / BK);

  f32x4 ra[ACH], rb[BCH];
  auto gload = [&](int kt) {
    const int64_t k0 = r_begin + (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int c = tid + i * 256, kr = c / (BM / 4), col = (c % (BM / 4)) * 4;
      int64_t m = k0 + kr;
      int o = o0 + col;
      ra[i] = (m < r_end && o < a.Cout) ? ld4(a.dy + m * a.ldy + o) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int c = tid + i * 256, kr = c / (BN / 4), col = (c % (BN / 4)) * 4;
      int64_t m = k0 + kr;
      int kk = n0 + col;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (m < r_end && kk < a.Kp) {
        int j = kk / a.Cin, ci = kk - j * a.Cin;
        int64_t s = m / a.T;
        int64_t t = m - s * a.T + j - a.pad;
        if (t >= 0 && t < a.T) v = ld4(a.x + (s * a.T + t) * a.ldx + ci);
      }
      rb[i] = v;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int c = tid + i * 256, kr = c / (BM / 4), col = (c % (BM / 4)) * 4;
      st4(&As[buf][kr * LDA + col], ra[i]);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int c = tid + i * 256, kr = c / (BN / 4), col = (c % (BN / 4)) * 4;
      st4(&Bs[buf][kr * LDB + col], rb[i]);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      float fa[MI], fb[NI];
      const int kr = 8 * g + jj;
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = As[cur][kr * LDA + wm * (BM / 2) + i * 16 + r16];
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = Bs[cur][kr * LDB + wn * (BN / 2) + j * 16 + r16];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  float* slab = a.slab + (int64_t)blockIdx.z * a.Cout * a.Kp;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + r16;
      if (n >= a.Kp) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + wm * (BM / 2) + i * 16 + 4 * g + r;
        if (o < a.Cout) slab[(int64_t)o * a.Kp + n] = acc[i][j][r];
      }
    }
}

// dw[o, c, j] += sum_z slab[z][o][j*Cin + c]   (in split order)
__global__ void wgrad_reduce(const float* slab, int splits, int Cout, int Cin, int taps, float* dw) {
  const int64_t Kp = (int64_t)taps * Cin;
  const int64_t total = (int64_t)Cout * Kp;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += slab[(int64_t)z * total + e];
    int64_t o = e / Kp;
    int kk = (int)(e - o * Kp);
    int j = kk / Cin, c = kk - j * Cin;
    dw[(o * Cin + c) * taps + j] += s;
  }
}

// ------------------------------------------------------------------------ weight re-layout
__global__ void weight_prep_f32(const float* w, int Cout, int Cin, int taps, float* wf, float* wb) {
  const int64_t total = (int64_t)Cout * Cin * taps;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t o = e / ((int64_t)Cin * taps);
    int rem = (int)(e - o * Cin * taps);
    int c = rem / taps, j = rem - c * taps;
    float v = w[e];
    if (wf) wf[o * (int64_t)taps * Cin + (int64_t)j * Cin + c] = v;
    if (wb) wb[(int64_t)c * taps * Cout + (int64_t)(taps - 1 - j) * Cout + o] = v;
  }
}

// ------------------------------------------------------------------------ column sums
constexpr int CS_ROWS = 256;  // rows per partial
__global__ void colsum_partial(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* part) {
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ry = threadIdx.x >> 6;  // 4 row lanes
  const int64_t r0 = (int64_t)blockIdx.y * CS_ROWS;
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < cols) {
    int64_t r1 = r0 + CS_ROWS < rows ? r0 + CS_ROWS : rows;
    for (int64_t r = r0 + ry; r < r1; r += 4) s += x[r * ldx + c];
  }
  red[ry][threadIdx.x & 63] = s;
  __syncthreads();
  if (ry == 0 && c < cols)
    part[(int64_t)blockIdx.y * cols + c] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                          red[2][threadIdx.x] + red[3][threadIdx.x];
}
// 64 columns x 16 partial-lanes per block: lane y sums partials y, y+16, ... (independent
// loads in flight), then the 16 lane sums are added in lane order (deterministic).
__global__ __launch_bounds__(1024) void colsum_final(const float* part, int64_t nparts,
                                                     int64_t cols, float* out, int acc) {
  __shared__ float red[16][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + tx;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 4
    for (int64_t p = ty; p < nparts; p += 16) s += part[p * cols + c];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int y = 0; y < 16; ++y) t += red[y][tx];
    out[c] = acc ? out[c] + t : t;
  }
}

// Several independent finals in one launch (blockIdx.y = job), each as colsum_final.
// 16 columns x 64 row groups per block: each thread sums every 64th partial row of its column
// (a dozen loads for the LN backward's 768 partial rows, four in flight), then a fixed-order
// LDS tree over the 64 groups.  Deterministic; the blocks of all jobs run in one launch.
__global__ __launch_bounds__(1024) void colsum_final_multi(ColsumJobs jobs) {
  __shared__ float red[64][17];
  const ColsumJob& jb = jobs.job[blockIdx.y];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t c = (int64_t)blockIdx.x * 16 + tx;
  if ((int64_t)blockIdx.x * 16 >= jb.cols) return;  // block-uniform
  float s = 0.f;
  if (c < jb.cols) {
#pragma unroll 4
    for (int64_t p = ty; p < jb.nparts; p += 64) s += jb.part[p * jb.cols + c];
  }
  red[ty][tx] = s;
  __syncthreads();
#pragma unroll
  for (int h = 32; h > 0; h >>= 1) {
    if (ty < h) red[ty][tx] += red[ty + h][tx];
    __syncthreads();
  }
  if (ty == 0 && c < jb.cols) jb.out[c] = jobs.acc ? jb.out[c] + red[0][tx] : red[0][tx];
}

int colsum_final_multi_launch(const ColsumJobs& jobs, hipStream_t st) {
  if (jobs.n == 0) return FS2_OK;
  int64_t maxc = 0;
  for (int i = 0; i < jobs.n; ++i) maxc = jobs.job[i].cols > maxc ? jobs.job[i].cols : maxc;
  dim3 grid((unsigned)((maxc + 15) / 16), (unsigned)jobs.n);
  colsum_final_multi<<<grid, 1024, 0, st>>>(jobs);
  return launch_status("colsum_final_multi");
}

int colsum_launch(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out, int acc,
                  float* ws, hipStream_t st) {
  const int64_t nparts = (rows + CS_ROWS - 1) / CS_ROWS;
  if (nparts == 0) return FS2_OK;
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)nparts);
  colsum_partial<<<grid, 256, 0, st>>>(x, ldx, rows, cols, ws);
  colsum_final<<<(unsigned)((cols + 63) / 64), 1024, 0, st>>>(ws, nparts, cols, out, acc);
  return launch_status("colsum");
}

int colsum_final_launch(const float* part, int64_t nparts, int64_t cols, float* out, int acc,
                        hipStream_t st) {
  if (cols <= 0) return FS2_OK;
  colsum_final<<<(unsigned)((cols + 63) / 64), 1024, 0, st>>>(part, nparts, cols, out, acc);
  return launch_status("colsum_final");
}

// Weight-gradient decomposition (measured on the step's shapes, scripts/wgrad_sweep.py):
// 128-wide tiles with <= 8 row splits for the large k>1 products, 64-wide tiles with 4..24
// splits (>= 8 k-tiles of 64 rows each) for the small ones, ~1024 blocks where possible.
static int wgrad_tile(int64_t rows, int64_t c_in, int64_t c_out, int taps) {
  (void)rows;
  if (g_tune[FS2_TUNE_WGRAD_TILE]) return g_tune[FS2_TUNE_WGRAD_TILE] == 64 ? 64 : 128;
  return (int64_t)taps * c_in * c_out >= (1 << 20) ? 128 : 64;
}

static int wgrad_splits(int64_t rows, int64_t c_in, int64_t c_out, int taps) {
  if (g_tune[FS2_TUNE_WGRAD_SPLITS]) {
    const int s = g_tune[FS2_TUNE_WGRAD_SPLITS];
    return s < 1 ? 1 : s > 64 ? 64 : s;
  }
  const int64_t Kp = (int64_t)taps * c_in;
  const int bt = wgrad_tile(rows, c_in, c_out, taps);
  const int64_t tiles = ((c_out + bt - 1) / bt) * ((Kp + bt - 1) / bt);
  // k = 1 (tap-major kernel, 4 blocks per CU): at most one round of 1024 blocks -- rounding
  // the split count up put 32 of the decoder QKV product's 1056 blocks in a second round
  // (45.9 -> 33.6 us alone with 21 splits instead of 22)
  int64_t s = taps == 1 ? 1024 / tiles : (1024 + tiles - 1) / tiles;
  const int64_t hi = bt == 128 ? 8 : 24;
  if (s > hi) s = hi;
  if (s < 4) s = 4;
  if (s > rows / 512) s = rows / 512;
  if (s < 1) s = 1;
  return (int)s;
}

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_conv_gemm_ex(int dtype, const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                     int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps, int pad,
                     int dilation, const int64_t* lens, const float* bias, int flags,
                     const void* aux, int64_t ld_aux, float alpha, float scale, void* y2,
                     float alpha2, void* stream) {
  FS2_CHECK_ARG(rows >= 0 && seq_len > 0 && taps >= 1 && dilation >= 1 && pad >= 0 &&
                    pad <= (taps - 1) * dilation,
                "fs2_conv_gemm: bad geometry (taps %d, pad %d, dilation %d)", taps, pad, dilation);
  FS2_CHECK_ARG(!(flags & FS2_EPI_BIAS) || bias, "fs2_conv_gemm: bias flag without bias");
  FS2_CHECK_ARG(!(flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX)) || aux,
                "fs2_conv_gemm: aux flag without aux");
  FS2_CHECK_ARG(!(flags & FS2_EPI_Y2) || y2, "fs2_conv_gemm: Y2 flag without y2");
  FS2_CHECK_ARG(!(flags & FS2_EPI_ACC_Y) || y, "fs2_conv_gemm: ACC_Y needs y");
  FS2_CHECK_ARG(y || (flags & FS2_EPI_Y2), "fs2_conv_gemm: no output");
  if (rows == 0) return FS2_OK;
  const VocEpi ve{dilation, alpha, scale, y2, alpha2};
  if (dtype == FS2_BF16)
    return conv_gemm_bf16_launch(x, ldx, wk, y, ldy, rows, seq_len, c_in, c_out, taps, pad, lens,
                                 bias, flags, aux, ld_aux, ve, as_stream(stream));
  if (dtype != FS2_F32) {
    set_error("fs2_conv_gemm: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  FS2_CHECK_ARG(!(flags & (FS2_EPI_OUT_BF16 | FS2_EPI_AUX_BF16)), "fs2_conv_gemm: bf16 flags on the fp32 path");
  FS2_CHECK_ARG(c_in % 4 == 0 && ldx % 4 == 0, "fs2_conv_gemm: c_in/ldx must be multiples of 4");
  ConvArgs a{(const float*)x, ldx, (const float*)wk, (float*)y, ldy, rows, seq_len, (int)c_in,
             (int)c_out, taps, pad, (int)(taps * c_in), bias, flags, (const float*)aux, ld_aux,
             dilation, alpha, scale, (float*)y2, alpha2};
  hipStream_t st = as_stream(stream);
  const int64_t big = ((rows + 127) / 128) * ((c_out + 127) / 128);
  if (big >= 256) {
    dim3 grid((unsigned)((rows + 127) / 128), (unsigned)((c_out + 127) / 128));
    conv_gemm_nt_f32<128, 128><<<grid, 256, 0, st>>>(a);
  } else {
    dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((c_out + 63) / 64));
    conv_gemm_nt_f32<64, 64><<<grid, 256, 0, st>>>(a);
  }
  return launch_status("fs2_conv_gemm");
}

int fs2_conv_gemm_ln(const void* x, int64_t ldx, const void* wk, int64_t rows, int64_t seq_len,
                     int64_t c_in, int64_t c_out, int taps, int pad, const int64_t* lens,
                     const float* bias, const float* res, const float* gamma, const float* beta,
                     float* out, void* out_t, float* xhat, float* rstd, float p_in,
                     const uint64_t* seed, uint64_t site_in, void* stream) {
  FS2_CHECK_ARG(rows >= 0 && seq_len > 0 && taps >= 1 && pad >= 0 && pad < taps,
                "fs2_conv_gemm_ln: bad geometry");
  FS2_CHECK_ARG(c_out == 256, "fs2_conv_gemm_ln: only c_out = 256 (the LayerNorm width) is built");
  FS2_CHECK_ARG(gamma && beta && out && xhat && rstd, "fs2_conv_gemm_ln: missing LayerNorm tensors");
  FS2_CHECK_ARG(!(p_in > 0.f) || seed, "fs2_conv_gemm_ln: dropout without seed");
  if (rows == 0) return FS2_OK;
  return conv_gemm_ln_glds_launch(x, ldx, wk, rows, seq_len, c_in, taps, pad, lens, bias, res,
                                  gamma, beta, out, out_t, xhat, rstd, p_in, seed, site_in,
                                  as_stream(stream));
}

int fs2_conv_gemm_ln_bwd(const void* x, int64_t ldx, const void* wk, int64_t rows,
                         int64_t seq_len, int64_t c_in, int64_t c_out, int taps, int pad,
                         const int64_t* lens, const float* aux, const float* xhat,
                         const float* rstd, const float* gamma, float* dgamma, float* dbeta,
                         float* dbias_in, float p_in, const uint64_t* seed, uint64_t site_in,
                         float* dres, int dres_add, void* dy_t, float* ws, int64_t ws_bytes,
                         void* stream) {
  FS2_CHECK_ARG(rows >= 0 && seq_len > 0 && taps >= 1 && pad >= 0 && pad < taps,
                "fs2_conv_gemm_ln_bwd: bad geometry");
  FS2_CHECK_ARG(c_out == 256, "fs2_conv_gemm_ln_bwd: only c_out = 256 (the LayerNorm width) is built");
  FS2_CHECK_ARG(xhat && rstd && gamma && dres, "fs2_conv_gemm_ln_bwd: missing LayerNorm tensors");
  FS2_CHECK_ARG(!(p_in > 0.f) || seed, "fs2_conv_gemm_ln_bwd: dropout without seed");
  FS2_CHECK_ARG(ws_bytes >= fs2_ln_bwd_ws_bytes(rows, 256), "fs2_conv_gemm_ln_bwd: workspace too small");
  if (rows == 0) return FS2_OK;
  poison(ws, ws_bytes, as_stream(stream));
  int rc = conv_gemm_lnbwd_glds_launch(x, ldx, wk, rows, seq_len, c_in, taps, pad, lens, aux, xhat,
                                       rstd, gamma, p_in, seed, site_in, dres, dres_add, dy_t, ws,
                                       as_stream(stream));
  if (rc) return rc;
  return fs2_ln_bwd_final(rows, 256, ws, 0, dgamma, dbeta, nullptr, nullptr, dbias_in, stream);
}

int fs2_conv_gemm(int dtype, const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                  int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps, int pad,
                  const int64_t* lens, const float* bias, int flags, const void* aux,
                  int64_t ld_aux, void* stream) {
  FS2_CHECK_ARG(rows >= 0 && seq_len > 0 && taps >= 1 && pad >= 0 && pad < taps,
                "fs2_conv_gemm: bad geometry");
  FS2_CHECK_ARG(!(flags & (FS2_EPI_LRELU | FS2_EPI_ACC_Y | FS2_EPI_Y2)),
                "fs2_conv_gemm: vocoder epilogue flags need fs2_conv_gemm_ex");
  FS2_CHECK_ARG(!(flags & FS2_EPI_BIAS) || bias, "fs2_conv_gemm: bias flag without bias");
  FS2_CHECK_ARG(!(flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX)) || aux,
                "fs2_conv_gemm: aux flag without aux");
  if (rows == 0) return FS2_OK;
  if (dtype == FS2_BF16)
    return conv_gemm_bf16_launch(x, ldx, wk, y, ldy, rows, seq_len, c_in, c_out, taps, pad, lens,
                                 bias, flags, aux, ld_aux, VocEpi{}, as_stream(stream));
  return fs2_conv_gemm_ex(dtype, x, ldx, wk, y, ldy, rows, seq_len, c_in, c_out, taps, pad, 1,
                          lens, bias, flags, aux, ld_aux, 0.f, 1.f, nullptr, 0.f, stream);
}

int fs2_conv_weight_prep(int dtype, const float* w, int64_t c_out, int64_t c_in, int taps,
                         void* w_fwd, void* w_bwd, void* stream) {
  const int64_t total = c_out * c_in * taps;
  if (total == 0) return FS2_OK;
  if (dtype == FS2_BF16) return weight_prep_bf16_launch(w, c_out, c_in, taps, w_fwd, w_bwd, as_stream(stream));
  if (dtype != FS2_F32) {
    set_error("fs2_conv_weight_prep: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  unsigned blocks = (unsigned)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  weight_prep_f32<<<blocks, 256, 0, as_stream(stream)>>>(w, (int)c_out, (int)c_in, taps,
                                                         (float*)w_fwd, (float*)w_bwd);
  return launch_status("fs2_conv_weight_prep");
}

// workspace: split slabs [S][c_out][taps c_in], then the bias partials
int64_t fs2_conv_wgrad_ws_bytes(int64_t rows, int64_t c_in, int64_t c_out, int taps) {
  const int64_t S = wgrad_splits(rows, c_in, c_out, taps);
  const int64_t bias_part = S * c_out > ((rows + CS_ROWS - 1) / CS_ROWS) * c_out
                                ? S * c_out : ((rows + CS_ROWS - 1) / CS_ROWS) * c_out;
  int64_t b = (S * c_out * taps * c_in + bias_part) * 4;
  const int64_t wide = conv_wgrad_wide_ws_floats(rows, c_in, c_out, taps) * 4;  // wgrad.hip
  b = wide > b ? wide : b;
  if (taps == 1) {  // bf16 k = 1: the grouped kernel with one job (wgrad.hip)
    const int64_t job[8] = {0, c_out, 0, c_in, 0, 1, c_in, c_out};
    const int64_t m = wgrad_k1_multi_ws_floats(job, 1, rows) * 4;
    b = m > b ? m : b;
  }
  return b;
}

int fs2_conv_wgrad(int dtype, const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                   float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                   int pad, const int64_t* lens, float* ws, int64_t ws_bytes, void* stream) {
  const int64_t slab_floats = (int64_t)wgrad_splits(rows, c_in, c_out, taps) * c_out * taps * c_in;
  if (dtype == FS2_BF16) {
    FS2_CHECK_ARG(ws_bytes >= fs2_conv_wgrad_ws_bytes(rows, c_in, c_out, taps),
                  "fs2_conv_wgrad: workspace too small");
    if (rows == 0) return FS2_OK;
    poison(ws, ws_bytes, as_stream(stream));
    const int S = wgrad_splits(rows, c_in, c_out, taps);
    if (taps == 1 && !g_tune[FS2_TUNE_LEGACY_GEMM] && g_tune[FS2_TUNE_WGRAD_K1] == 0) {
      // k = 1: the grouped split-K kernel with one job (128 x 128 tiles, one reduce)
      const int64_t job[8] = {(int64_t)dy, ldy, (int64_t)x, ldx, (int64_t)dw, (int64_t)db, c_in, c_out};
      FS2_CHECK_ARG(c_in % 8 == 0 && c_out % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
                        ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dw & 15) == 0,
                    "fs2_conv_wgrad(bf16, k = 1): channel counts / strides must be multiples of 8, "
                    "operands and dw 16-B aligned");
      // the kernel reads lens[row / seq_len] to skip all-padding k-tiles
      FS2_CHECK_ARG(lens == nullptr || (seq_len > 0 && rows % seq_len == 0),
                    "fs2_conv_wgrad(bf16, k = 1): with lens, rows must be batch x seq_len");
      return wgrad_k1_multi_launch(job, 1, rows, seq_len, lens, ws, as_stream(stream));
    }
    if (!g_tune[FS2_TUNE_LEGACY_GEMM])
      return conv_wgrad_glds_launch(dy, ldy, x, ldx, dw, db, rows, seq_len, c_in, c_out, taps, pad,
                                    lens, S, wgrad_tile(rows, c_in, c_out, taps), ws,
                                    as_stream(stream));
    int rc = conv_wgrad_bf16_launch(dy, ldy, x, ldx, ws, rows, seq_len, c_in, c_out, taps, pad, S,
                                    as_stream(stream));
    if (rc) return rc;
    const int64_t total = c_out * c_in * taps;
    unsigned blocks = (unsigned)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    wgrad_reduce<<<blocks, 256, 0, as_stream(stream)>>>(ws, S, (int)c_out, (int)c_in, taps, dw);
    if (db) return colsum_bf16_launch(dy, ldy, rows, c_out, db, 1, ws + slab_floats, as_stream(stream));
    return launch_status("fs2_conv_wgrad");
  }
  if (dtype != FS2_F32) {
    set_error("fs2_conv_wgrad: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  FS2_CHECK_ARG(c_in % 4 == 0 && c_out % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0,
                "fs2_conv_wgrad: channel counts / strides must be multiples of 4");
  FS2_CHECK_ARG(ws_bytes >= fs2_conv_wgrad_ws_bytes(rows, c_in, c_out, taps),
                "fs2_conv_wgrad: workspace too small");
  if (rows == 0) return FS2_OK;
  poison(ws, ws_bytes, as_stream(stream));
  const int S = wgrad_splits(rows, c_in, c_out, taps);
  int64_t rps = (rows + S - 1) / S;
  rps = (rps + BK - 1) / BK * BK;
  WgradArgs a{(const float*)dy, ldy, (const float*)x, ldx, ws, rows, seq_len, (int)c_in,
              (int)c_out, taps, pad, (int)(taps * c_in), rps};
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)((c_out + 127) / 128), (unsigned)((taps * c_in + 127) / 128), (unsigned)S);
  conv_wgrad_tn_f32<128, 128><<<grid, 256, 0, st>>>(a);
  const int64_t total = c_out * c_in * taps;
  unsigned blocks = (unsigned)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  wgrad_reduce<<<blocks, 256, 0, st>>>(ws, S, (int)c_out, (int)c_in, taps, dw);
  if (db) return colsum_launch((const float*)dy, ldy, rows, c_out, db, 1, ws + slab_floats, st);
  return launch_status("fs2_conv_wgrad");
}

int64_t fs2_conv_wgrad_k1_multi_ws_bytes(const int64_t* jobs, int n_jobs, int64_t rows) {
  int64_t b = wgrad_k1_multi_ws_floats(jobs, n_jobs, rows) * 4;
  for (int j = 0; j < n_jobs; ++j) {  // the fp32 path runs the jobs one by one
    const int64_t w = fs2_conv_wgrad_ws_bytes(rows, jobs[8 * j + 6], jobs[8 * j + 7], 1);
    b = w > b ? w : b;
  }
  return b;
}

int fs2_conv_wgrad_k1_multi(int dtype, const int64_t* jobs, int n_jobs, int64_t rows,
                            int64_t seq_len, const int64_t* lens, float* ws, int64_t ws_bytes,
                            void* stream) {
  FS2_CHECK_ARG(jobs && n_jobs >= 1 && n_jobs <= 4, "fs2_conv_wgrad_k1_multi: 1..4 jobs");
  FS2_CHECK_ARG(ws_bytes >= fs2_conv_wgrad_k1_multi_ws_bytes(jobs, n_jobs, rows),
                "fs2_conv_wgrad_k1_multi: workspace too small");
  FS2_CHECK_ARG(seq_len > 0 && rows % seq_len == 0, "fs2_conv_wgrad_k1_multi: rows must be batch x seq_len");
  if (rows == 0) return FS2_OK;
  poison(ws, ws_bytes, as_stream(stream));
  if (dtype == FS2_BF16 && !g_tune[FS2_TUNE_LEGACY_GEMM])
    return wgrad_k1_multi_launch(jobs, n_jobs, rows, seq_len, lens, ws, as_stream(stream));
  for (int j = 0; j < n_jobs; ++j) {
    const int64_t* r = jobs + 8 * j;
    const int rc = fs2_conv_wgrad(dtype, (const void*)r[0], r[1], (const void*)r[2], r[3],
                                  (float*)r[4], (float*)r[5], rows, seq_len, r[6], r[7], 1, 0, lens,
                                  ws, ws_bytes, stream);
    if (rc) return rc;
  }
  return FS2_OK;
}

int64_t fs2_colsum_ws_bytes(int64_t rows, int64_t cols) {
  return ((rows + CS_ROWS - 1) / CS_ROWS) * cols * 4;
}

int fs2_colsum(int dtype, const void* x, int64_t ldx, int64_t rows, int64_t cols, float* out,
               int accumulate, float* ws, int64_t ws_bytes, void* stream) {
  FS2_CHECK_ARG(ws_bytes >= fs2_colsum_ws_bytes(rows, cols), "fs2_colsum: workspace too small");
  poison(ws, ws_bytes, as_stream(stream));
  if (rows == 0) {
    if (!accumulate) (void)hipMemsetAsync(out, 0, cols * 4, as_stream(stream));
    return FS2_OK;
  }
  if (dtype == FS2_BF16)
    return colsum_bf16_launch(x, ldx, rows, cols, out, accumulate, ws, as_stream(stream));
  if (dtype != FS2_F32) {
    set_error("fs2_colsum: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  return colsum_launch((const float*)x, ldx, rows, cols, out, accumulate, ws, as_stream(stream));
}

}  // extern "C"
