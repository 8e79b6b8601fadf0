// bf16 implicit-GEMM Conv1d / Linear on gfx950 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// Same two products as gemm.hip (forward/dX "NT", weight-gradient "TN"); operands are bf16
// compute copies of fp32 master data, accumulation and the weight-gradient slabs are fp32.
//   NT: 4 waves (2x2), BM x BN tile, BK = 64 (two 32-deep MFMA k-steps), LDS images
//       [row][k] with 144-B rows (conflict-free ds_read_b128 fragments), register-staged
//       double buffer, one barrier per k-tile; conv tap shift in the A loader.
//   TN: operands arrive k-major ([rows of the reduction][channels]); the LDS images keep
//       that layout and the MFMA fragments are read with ds_read_b64_tr_b16 (gfx950's
//       transposing LDS read): each 16-lane group reads 4 k-rows x 16 columns and every lane
//       receives its column's 4 consecutive k.  A fragment's 8 k are taken from rows
//       {4g..4g+3} and {16+4g..16+4g+3} of the 32-row k-step (the same permutation on both
//       operands), which with a 288-B row stride makes each 32-lane half hit 64 distinct
//       banks.
#include "common.hpp"

namespace fs2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct ConvArgsB {
  const u16* x;
  int64_t ldx;
  const u16* w;
  void* y;
  int64_t ldy;
  int64_t M, T;
  int Cin, N, taps, pad, K;
  const float* bias;
  int flags;
  const void* aux;
  int64_t ld_aux;
};

FS2_DEV uint4 zero4() { return make_uint4(0u, 0u, 0u, 0u); }

FS2_DEV uint4 load_conv_a_bf16(const ConvArgsB& a, int64_t m, int k) {
  if (m >= a.M || k >= a.K) return zero4();
  const int j = k / a.Cin;
  const int c = k - j * a.Cin;
  const int64_t s = m / a.T;
  const int64_t t = m - s * a.T + j - a.pad;
  if (t < 0 || t >= a.T) return zero4();
  return *reinterpret_cast<const uint4*>(a.x + (s * a.T + t) * a.ldx + c);
}

FS2_DEV float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
FS2_DEV u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // round-to-nearest-even (v_cvt_pk_bf16_f32)
  return *reinterpret_cast<u16*>(&b);
}

FS2_DEV void epilogue_store(const ConvArgsB& a, int64_t m, int n, float v) {
  if (a.flags & FS2_EPI_ADD_AUX)
    v += (a.flags & FS2_EPI_AUX_BF16) ? bf2f(((const u16*)a.aux)[m * a.ld_aux + n])
                                      : ((const float*)a.aux)[m * a.ld_aux + n];
  if (a.flags & FS2_EPI_RELU) v = fmaxf(v, 0.f);
  if (a.flags & FS2_EPI_RELU_MASK_AUX) {
    const float av = (a.flags & FS2_EPI_AUX_BF16) ? bf2f(((const u16*)a.aux)[m * a.ld_aux + n])
                                                  : ((const float*)a.aux)[m * a.ld_aux + n];
    v = av > 0.f ? v : 0.f;
  }
  if (a.flags & FS2_EPI_OUT_BF16) ((u16*)a.y)[m * a.ldy + n] = f2bf(v);
  else ((float*)a.y)[m * a.ldy + n] = v;
}

template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_gemm_nt_bf16(ConvArgsB a) {
  constexpr int BKE = 64;           // k elements per tile
  constexpr int LDE = BKE + 8;      // padded LDS row (elements) = 144 B
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int ACH = BM * BKE / 8 / 256, BCH = BN * BKE / 8 / 256;
  __shared__ __attribute__((aligned(16))) u16 As[2][BM * LDE];
  __shared__ __attribute__((aligned(16))) u16 Bs[2][BN * LDE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int nk = (a.K + BKE - 1) / BKE;

  uint4 ra[ACH], rb[BCH];
  auto gload = [&](int kt) {
    const int k0 = kt * BKE;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 8;
      ra[i] = load_conv_a_bf16(a, m0 + row, k0 + kq);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 8;
      const int n = n0 + row, k = k0 + kq;
      rb[i] = (n < a.N && k < a.K) ? *reinterpret_cast<const uint4*>(a.w + (int64_t)n * a.K + k)
                                   : zero4();
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 8;
      *reinterpret_cast<uint4*>(&As[buf][row * LDE + kq]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, row = c >> 3, kq = (c & 7) * 8;
      *reinterpret_cast<uint4*>(&Bs[buf][row * LDE + kq]) = rb[i];
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
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(
            &As[cur][(wm * (BM / 2) + i * 16 + r16) * LDE + ks * 32 + 8 * g]);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(
            &Bs[cur][(wn * (BN / 2) + j * 16 + r16) * LDE + ks * 32 + 8 * g]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

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
        if (m < a.M) epilogue_store(a, m, n, acc[i][j][r] + bv);
      }
    }
}

// ------------------------------------------------------------------------ weight gradient
struct WgradArgsB {
  const u16* dy;
  int64_t ldy;
  const u16* x;
  int64_t ldx;
  float* slab;
  int64_t M, T;
  int Cin, Cout, taps, pad, Kp;
  int64_t rows_per_split;
};

template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_wgrad_tn_bf16(WgradArgsB a) {
  constexpr int BKE = 64;                 // reduction rows per tile (two 32-row k-steps)
  constexpr int LDA = BM + 16, LDB = BN + 16;  // elements; 288-B rows for BM = 128
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int ACH = BM * BKE / 8 / 256, BCH = BN * BKE / 8 / 256;
  __shared__ __attribute__((aligned(16))) u16 As[2][BKE * LDA];  // [m][o]
  __shared__ __attribute__((aligned(16))) u16 Bs[2][BKE * LDB];  // [m][j*Cin + c]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r16 = lane & 15;
  const int o0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int64_t r_begin = (int64_t)blockIdx.z * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.M) r_end = a.M;
  const int nk = (int)((r_end - r_begin + BKE - 1) / BKE);

  uint4 ra[ACH], rb[BCH];
  auto gload = [&](int kt) {
    const int64_t k0 = r_begin + (int64_t)kt * BKE;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, kr = c / (BM / 8), col = (c % (BM / 8)) * 8;
      const int64_t m = k0 + kr;
      const int o = o0 + col;
      ra[i] = (m < r_end && o < a.Cout) ? *reinterpret_cast<const uint4*>(a.dy + m * a.ldy + o)
                                        : zero4();
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, kr = c / (BN / 8), col = (c % (BN / 8)) * 8;
      const int64_t m = k0 + kr;
      const int kk = n0 + col;
      uint4 v = zero4();
      if (m < r_end && kk < a.Kp) {
        const int j = kk / a.Cin, ci = kk - j * a.Cin;
        const int64_t s = m / a.T;
        const int64_t t = m - s * a.T + j - a.pad;
        if (t >= 0 && t < a.T) v = *reinterpret_cast<const uint4*>(a.x + (s * a.T + t) * a.ldx + ci);
      }
      rb[i] = v;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * 256, kr = c / (BM / 8), col = (c % (BM / 8)) * 8;
      *reinterpret_cast<uint4*>(&As[buf][kr * LDA + col]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * 256, kr = c / (BN / 8), col = (c % (BN / 8)) * 8;
      *reinterpret_cast<uint4*>(&Bs[buf][kr * LDB + col]) = rb[i];
    }
  };
  // fragment of 16 columns at col0 for k-step ks: rows {4g+q} and {16+4g+q} (+32 ks)
  auto tr_frag = [&](const u16* img, int ld, int col0, int ks) -> bf16x8 {
    const u16* p0 = img + (ks * 32 + 4 * g + q) * ld + col0 + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 16 * ld));
    const auto v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
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
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = tr_frag(As[cur], LDA, wm * (BM / 2) + i * 16, ks);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = tr_frag(Bs[cur], LDB, wn * (BN / 2) + j * 16, ks);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
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

__global__ void weight_prep_bf16(const float* w, int Cout, int Cin, int taps, u16* wf, u16* wb) {
  const int64_t total = (int64_t)Cout * Cin * taps;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = e / ((int64_t)Cin * taps);
    const int rem = (int)(e - o * Cin * taps);
    const int c = rem / taps, j = rem - c * taps;
    const u16 v = f2bf(w[e]);
    if (wf) wf[o * (int64_t)taps * Cin + (int64_t)j * Cin + c] = v;
    if (wb) wb[(int64_t)c * taps * Cout + (int64_t)(taps - 1 - j) * Cout + o] = v;
  }
}

// All layers' re-layouts in one launch.  jobs[j] = {src, c_out, c_in, taps, w_fwd, w_bwd,
// first tile, end tile} (int64); a job has ceil(c_out/64) x ceil(c_in/CT) tiles, numbered
// consecutively over the jobs (CT = fs2_weight_prep_tile_channels).  Block b re-lays out
// one tile: 64 output channels x CT input channels x all taps.  The source rows are read as
// contiguous CT*taps runs into LDS (already cast), then w_fwd is written as CT-long runs per
// (o, tap) and w_bwd as 64-long runs per (c, tap).
template <typename OutT>
__global__ __launch_bounds__(256) void weight_prep_tiles(const int64_t* __restrict__ jobs, int n_jobs) {
  constexpr int CT = sizeof(OutT) == 2 ? 32 : 16;
  constexpr int MAXT = 9;
  constexpr int LD = CT * MAXT + 1;  // odd row stride (in OutT units of 2 or 4 B)
  __shared__ OutT tile[64 * LD];
  int lo = 0, hi = n_jobs - 1;
  while (lo < hi) {  // last job whose first tile <= blockIdx.x
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid * 8 + 6] <= (int64_t)blockIdx.x) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* jb = jobs + (int64_t)lo * 8;
  const float* w = (const float*)jb[0];
  const int Cout = (int)jb[1], Cin = (int)jb[2], taps = (int)jb[3];
  OutT* wf = (OutT*)jb[4];
  OutT* wb = (OutT*)jb[5];
  const int t = (int)(blockIdx.x - jb[6]), tiles_c = (Cin + CT - 1) / CT;
  const int tc = t % tiles_c, to = t / tiles_c;
  const int o0 = to * 64, c0 = tc * CT;
  const int no = Cout - o0 < 64 ? Cout - o0 : 64;
  const int nc = Cin - c0 < CT ? Cin - c0 : CT;
  const int run = nc * taps;  // contiguous source elements per row
  const int64_t Q = (int64_t)Cin * taps;
  if constexpr (sizeof(OutT) == 2) {
    // 16-B vector path (full tiles of aligned rows: every step weight but the odd edges):
    // float4 source reads, 8 x bf16 = 16-B stores of w_fwd (8 channels of one (o, tap)) and
    // w_bwd (8 output channels of one (c, tap))
    const bool vec = no == 64 && nc == CT && (Q % 4) == 0 && (Cin % 8) == 0 && (Cout % 8) == 0 &&
                     (((uintptr_t)w | (uintptr_t)wf | (uintptr_t)wb) & 15) == 0;
    if (vec) {
      const int run4 = run / 4;  // CT * taps is a multiple of 4 (CT = 32)
      for (int e = threadIdx.x; e < 64 * run4; e += 256) {
        const int r = e / run4, q4 = e - r * run4;
        const f32x4 v = ld4(w + (int64_t)(o0 + r) * Q + (int64_t)c0 * taps + 4 * q4);
        OutT* t = tile + r * LD + 4 * q4;
        t[0] = f2bf(v.x);
        t[1] = f2bf(v.y);
        t[2] = f2bf(v.z);
        t[3] = f2bf(v.w);
      }
      __syncthreads();
      if (wf) {  // wf[o, j*Cin + c]: per (o, j) a run of CT = 4 x 8 channels
        for (int e = threadIdx.x; e < 64 * taps * (CT / 8); e += 256) {
          const int c8 = (e % (CT / 8)) * 8, rj = e / (CT / 8), j = rj % taps, r = rj / taps;
          const OutT* t = tile + r * LD + c8 * taps + j;
          uint4 o;
          o.x = (uint32_t)t[0] | ((uint32_t)t[taps] << 16);
          o.y = (uint32_t)t[2 * taps] | ((uint32_t)t[3 * taps] << 16);
          o.z = (uint32_t)t[4 * taps] | ((uint32_t)t[5 * taps] << 16);
          o.w = (uint32_t)t[6 * taps] | ((uint32_t)t[7 * taps] << 16);
          *reinterpret_cast<uint4*>(wf + (int64_t)(o0 + r) * Q + (int64_t)j * Cin + c0 + c8) = o;
        }
      }
      if (wb) {  // wb[c*taps + taps-1-j, o]: per (c, j) a run of 64 = 8 x 8 output channels
        for (int e = threadIdx.x; e < CT * taps * 8; e += 256) {
          const int r8 = (e & 7) * 8, cj = e >> 3, j = cj % taps, c = cj / taps;
          const OutT* t = tile + r8 * LD + c * taps + j;
          uint4 o;
          o.x = (uint32_t)t[0] | ((uint32_t)t[LD] << 16);
          o.y = (uint32_t)t[2 * LD] | ((uint32_t)t[3 * LD] << 16);
          o.z = (uint32_t)t[4 * LD] | ((uint32_t)t[5 * LD] << 16);
          o.w = (uint32_t)t[6 * LD] | ((uint32_t)t[7 * LD] << 16);
          *reinterpret_cast<uint4*>(wb + ((int64_t)(c0 + c) * taps + (taps - 1 - j)) * Cout + o0 + r8) = o;
        }
      }
      return;
    }
  }
  for (int e = threadIdx.x; e < no * run; e += 256) {
    const int r = e / run, q = e - r * run;
    const float v = w[(int64_t)(o0 + r) * Q + (int64_t)c0 * taps + q];
    if constexpr (sizeof(OutT) == 2) tile[r * LD + q] = f2bf(v);
    else tile[r * LD + q] = v;
  }
  __syncthreads();
  if (wf) {  // wf[o, j*Cin + c]
    for (int e = threadIdx.x; e < no * taps * CT; e += 256) {
      const int c = e % CT, rj = e / CT, j = rj % taps, r = rj / taps;
      if (c < nc) wf[(int64_t)(o0 + r) * Q + (int64_t)j * Cin + c0 + c] = tile[r * LD + c * taps + j];
    }
  }
  if (wb) {  // wb[c*taps + taps-1-j, o]
    for (int e = threadIdx.x; e < nc * taps * 64; e += 256) {
      const int r = e & 63, cj = e >> 6, j = cj % taps, c = cj / taps;
      if (r < no)
        wb[((int64_t)(c0 + c) * taps + (taps - 1 - j)) * Cout + o0 + r] = tile[r * LD + c * taps + j];
    }
  }
}

__global__ void cast_bf16_kernel(const float* x, u16* y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

__global__ void colsum_partial_bf16(const u16* x, int64_t ldx, int64_t rows, int64_t cols, float* part) {
  const int64_t c = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int ry = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * 256;
  __shared__ float red[4][64];
  float s = 0.f;
  if (c < cols) {
    const int64_t r1 = r0 + 256 < rows ? r0 + 256 : rows;
    for (int64_t r = r0 + ry; r < r1; r += 4) s += bf2f(x[r * ldx + c]);
  }
  red[ry][threadIdx.x & 63] = s;
  __syncthreads();
  if (ry == 0 && c < cols)
    part[(int64_t)blockIdx.y * cols + c] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                          red[2][threadIdx.x] + red[3][threadIdx.x];
}

// ------------------------------------------------------------------------ launchers
int conv_gemm_bf16_launch(const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                          int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                          int pad, const int64_t* lens, const float* bias, int flags,
                          const void* aux, int64_t ld_aux, const VocEpi& ve, hipStream_t st) {
  const bool voc = ve.dil != 1 || (flags & (FS2_EPI_LRELU | FS2_EPI_ACC_Y | FS2_EPI_Y2)) || !y;
  if (!g_tune[FS2_TUNE_LEGACY_GEMM] || voc)  // the round-1 kernels have no vocoder epilogue
    return conv_gemm_glds_launch(x, ldx, wk, y, ldy, rows, seq_len, c_in, c_out, taps, pad, lens,
                                 bias, flags, aux, ld_aux, ve, st);
  FS2_CHECK_ARG(c_in % 8 == 0 && ldx % 8 == 0, "fs2_conv_gemm(bf16): c_in/ldx must be multiples of 8");
  ConvArgsB a{(const u16*)x, ldx, (const u16*)wk, y, ldy, rows, seq_len, (int)c_in, (int)c_out,
              taps, pad, (int)(taps * c_in), bias, flags, aux, ld_aux};
  const int64_t big = ((rows + 127) / 128) * ((c_out + 127) / 128);
  if (big >= 256) {
    dim3 grid((unsigned)((rows + 127) / 128), (unsigned)((c_out + 127) / 128));
    conv_gemm_nt_bf16<128, 128><<<grid, 256, 0, st>>>(a);
  } else {
    dim3 grid((unsigned)((rows + 63) / 64), (unsigned)((c_out + 63) / 64));
    conv_gemm_nt_bf16<64, 64><<<grid, 256, 0, st>>>(a);
  }
  return launch_status("fs2_conv_gemm(bf16)");
}

int conv_wgrad_bf16_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* slab,
                           int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                           int pad, int splits, hipStream_t st) {
  FS2_CHECK_ARG(c_in % 8 == 0 && c_out % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0,
                "fs2_conv_wgrad(bf16): channel counts / strides must be multiples of 8");
  int64_t rps = (rows + splits - 1) / splits;
  rps = (rps + 63) / 64 * 64;
  WgradArgsB a{(const u16*)dy, ldy, (const u16*)x, ldx, slab, rows, seq_len, (int)c_in,
               (int)c_out, taps, pad, (int)(taps * c_in), rps};
  dim3 grid((unsigned)((c_out + 127) / 128), (unsigned)((taps * c_in + 127) / 128), (unsigned)splits);
  conv_wgrad_tn_bf16<128, 128><<<grid, 256, 0, st>>>(a);
  return launch_status("fs2_conv_wgrad(bf16)");
}

int weight_prep_bf16_launch(const float* w, int64_t c_out, int64_t c_in, int taps, void* wf,
                            void* wb, hipStream_t st) {
  const int64_t total = c_out * c_in * taps;
  unsigned blocks = (unsigned)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  weight_prep_bf16<<<blocks, 256, 0, st>>>(w, (int)c_out, (int)c_in, taps, (u16*)wf, (u16*)wb);
  return launch_status("fs2_conv_weight_prep(bf16)");
}

int colsum_bf16_launch(const void* x, int64_t ldx, int64_t rows, int64_t cols, float* out, int acc,
                       float* ws, hipStream_t st) {
  const int64_t nparts = (rows + 255) / 256;
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)nparts);
  colsum_partial_bf16<<<grid, 256, 0, st>>>((const u16*)x, ldx, rows, cols, ws);
  return colsum_final_launch(ws, nparts, cols, out, acc, st);
}

}  // namespace fs2

extern "C" int fs2_weight_prep_tile_channels(int dtype) { return dtype == FS2_BF16 ? 32 : 16; }

extern "C" int fs2_weight_prep_batch(int dtype, const int64_t* jobs, int n_jobs, int64_t n_tiles,
                                     void* stream) {
  if (n_jobs <= 0 || n_tiles <= 0) return FS2_OK;
  if (dtype == FS2_BF16)
    fs2::weight_prep_tiles<unsigned short><<<(unsigned)n_tiles, 256, 0, as_stream(stream)>>>(jobs, n_jobs);
  else if (dtype == FS2_F32)
    fs2::weight_prep_tiles<float><<<(unsigned)n_tiles, 256, 0, as_stream(stream)>>>(jobs, n_jobs);
  else {
    fs2::set_error("fs2_weight_prep_batch: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  return fs2::launch_status("fs2_weight_prep_batch");
}

extern "C" int fs2_cast_bf16(const float* x, void* y, int64_t n, void* stream) {
  if (n <= 0) return FS2_OK;
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  fs2::cast_bf16_kernel<<<(unsigned)b, 256, 0, as_stream(stream)>>>(x, (unsigned short*)y, n);
  return fs2::launch_status("fs2_cast_bf16");
}
