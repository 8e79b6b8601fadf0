// bf16 fused attention (d_head = 128) on v_mfma_f32_16x16x32_bf16, fp32 softmax/accumulate.
//
// Same decomposition as attention.hip (transposed scores: each lane owns one query column
// in the forward / dQ kernels, one key column in the dK/dV kernel), with every wave owning
// TWO 16-row groups (32 queries, or 32 keys in dK/dV): each K/V/Q/dO fragment read from LDS
// feeds two MFMAs, halving the LDS traffic per FLOP, and a workgroup of NW waves covers
// 32 NW rows, so each K/V (Q/dO) tile is staged once per 32 NW rows.  The dQ kernel also
// forms delta = rowsum(dO * O) for its queries (no separate launch) and publishes it for the
// dK/dV kernel that follows on the stream.  The second product of
// each kernel contracts over keys (or queries), which sit in the *rows* of the LDS tiles:
// its A operand is read with ds_read_b64_tr_b16 (4 consecutive rows of one column per lane),
// and its B operand is the fp32 score accumulator packed to bf16 in place — the MFMA
// C-layout gives lane (g, col) the rows {16s + 4g + r}, so the 8 k-slots of a 32-deep step
// are taken as rows {32c + 4g + r} u {32c + 16 + 4g + r} on both operands.
#include <math.h>

#include <type_traits>

#include "common.hpp"

namespace fs2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace {
constexpr int DH = 128;
constexpr int QB = 64;
// LDS row strides of the 64 x 128 tiles.  288-B rows (72 dwords: row r starts at bank 8r mod
// 64) are conflict-free both for ds_read_b128 row fragments (16 rows x 16 B in its 4 lane
// groups) and for ds_read_b64_tr_b16 (8 rows x 32 B per 32-lane group); the dQ and dK/dV
// kernels read the same K / Q / dO tiles both ways.  (272-B rows, round 2's row stride, were
// 2-way conflicted on both: 22-43 % of the attention kernels' LDS cycles, SQ_LDS_BANK_CONFLICT;
// 0 now, decoder backward 91 -> 87 us.)
constexpr int LDR = DH + 16;
constexpr int LDT = DH + 16;

#define MFMA_BF16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

FS2_DEV float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
FS2_DEV u16 f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<u16*>(&b);
}

// register-staged copy of a 64 x 128 tile by NT threads: 1024 16-B pieces, PER = 1024 / NT
// per thread (issued before the MFMA work on the previous tile, so the global latency
// overlaps it), stored to LDS after a barrier
template <int NT>
FS2_DEV void load_regs(uint4 (&r)[1024 / NT], const u16* base, int64_t ld, int r0, int nrows, int tid) {
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int c = tid + i * NT, row = c >> 4, col = (c & 15) * 8;
    const int rr = r0 + row;
    r[i] = rr < nrows ? *reinterpret_cast<const uint4*>(base + (int64_t)rr * ld + col)
                      : make_uint4(0u, 0u, 0u, 0u);
  }
}
template <int LDS_LD, int NT>
FS2_DEV void store_regs(u16* dst, const uint4 (&r)[1024 / NT], int tid) {
#pragma unroll
  for (int i = 0; i < 1024 / NT; ++i) {
    const int c = tid + i * NT, row = c >> 4, col = (c & 15) * 8;
    *reinterpret_cast<uint4*>(&dst[row * LDS_LD + col]) = r[i];
  }
}

// the 4 x 16-B fragments of LDS row `row` (d = 32c + 8g .. +7)
template <int LD>
FS2_DEV void row_frags(bf16x8 (&f)[4], const u16* S, int row, int g) {
  const u16* p = S + row * LD + 8 * g;
#pragma unroll
  for (int c = 0; c < 4; ++c) f[c] = *reinterpret_cast<const bf16x8*>(p + 32 * c);
}

// sum over d = 128 of A-row fragments x B fragments (4 chained MFMAs)
FS2_DEV f32x4 chain4(const bf16x8 (&a)[4], const bf16x8 (&b)[4]) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) acc = MFMA_BF16(a[c], b[c], acc);
  return acc;
}

// per-lane row fragment: d = 32c + 8g .. +7 for c < 4
FS2_DEV void load_frag(bf16x8 (&f)[4], const u16* rowp, int g) {
#pragma unroll
  for (int c = 0; c < 4; ++c) f[c] = *reinterpret_cast<const bf16x8*>(rowp + 32 * c + 8 * g);
}

// S-type product over d = 128: rows (row0 + r16) of an LDS tile (stride LD) x lane fragment
template <int LD>
FS2_DEV f32x4 dot_tile(const u16* S, int row0, const bf16x8 (&f)[4], int g, int r16) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const u16* p = S + (row0 + r16) * LD + 8 * g;
#pragma unroll
  for (int c = 0; c < 4; ++c) acc = MFMA_BF16(*reinterpret_cast<const bf16x8*>(p + 32 * c), f[c], acc);
  return acc;
}

// transposed fragment of 16 columns (col0..) over rows {rb + 4g + q} and {rb + 16 + 4g + q}
template <int LD>
FS2_DEV bf16x8 tr_frag(const u16* img, int rb, int col0, int g, int q, int p) {
  const u16* p0 = img + (rb + 4 * g + q) * LD + col0 + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 16 * LD));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

FS2_DEV bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (__bf16)a.x; r[1] = (__bf16)a.y; r[2] = (__bf16)a.z; r[3] = (__bf16)a.w;
  r[4] = (__bf16)b.x; r[5] = (__bf16)b.y; r[6] = (__bf16)b.z; r[7] = (__bf16)b.w;
  return r;
}

// acc[ds] += sum over 32 rows (rb..rb+31) of T^T[d][row] * w[row]   (8 d-subtiles)
template <int LD>
FS2_DEV void accum_t(f32x4 (&acc)[8], const u16* S, int rb, const bf16x8& w, int g, int q, int p) {
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) acc[ds] = MFMA_BF16(tr_frag<LD>(S, rb, 16 * ds, g, q, p), w, acc[ds]);
}

// acc[j][ds] += sum over 32 rows (rb..rb+31) of T^T[d][row] * w[j][row] for two B operands
// (8 d-subtiles): each transposed fragment read from LDS feeds two MFMAs
template <int LD>
FS2_DEV void accum_t2(f32x4 (&acc)[2][8], const u16* S, int rb, const bf16x8& w0, const bf16x8& w1,
                      int g, int q, int p) {
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) {
    const bf16x8 a = tr_frag<LD>(S, rb, 16 * ds, g, q, p);
    acc[0][ds] = MFMA_BF16(a, w0, acc[0][ds]);
    acc[1][ds] = MFMA_BF16(a, w1, acc[1][ds]);
  }
}

FS2_DEV void store4_bf16(u16* p, const f32x4& v) {
  uint2 w;
  w.x = (uint32_t)f2bf(v.x) | ((uint32_t)f2bf(v.y) << 16);
  w.y = (uint32_t)f2bf(v.z) | ((uint32_t)f2bf(v.w) << 16);
  *reinterpret_cast<uint2*>(p) = w;
}

// The values of output fragments 2d (columns 32d + 4g .. + 3 of the lane's row) and 2d + 1
// (columns 32d + 16 + 4g .. + 3) stored as ONE 16-B vector per lane instead of two 8-B ones:
// v_permlane16_swap exchanges them between the 16-lane rows g and g ^ 1 (same row of the
// output), so even rows g store columns 32d + 4g .. + 7 and odd rows 32d + 16 + 4(g - 1) .. + 7.
// Half the store instructions of an issue-bound store tail (the guide's T21, for 16-lane rows);
// same bytes, same values.  p = the row's column 32d; both lanes of a pair must be active.
FS2_DEV void store8x2_bf16(u16* p, const f32x4& a, const f32x4& b, int g) {
  const uint32_t a0 = (uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16);
  const uint32_t a1 = (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16);
  const uint32_t b0 = (uint32_t)f2bf(b.x) | ((uint32_t)f2bf(b.y) << 16);
  const uint32_t b1 = (uint32_t)f2bf(b.z) | ((uint32_t)f2bf(b.w) << 16);
  const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
  const bool odd = g & 1;
  uint4 o;
  o.x = odd ? s0[0] : a0;
  o.y = odd ? s1[0] : a1;
  o.z = odd ? b0 : s0[1];
  o.w = odd ? b1 : s1[1];
  *reinterpret_cast<uint4*>(p + 4 * g + (odd ? 12 : 0)) = o;
}
}  // namespace


// ---- one 16-row group per wave, 64 rows per 4-wave workgroup (the T = 128 encoder shapes:
// twice the workgroups of the two-group kernels below, at 4 waves per SIMD)
__global__ __launch_bounds__(256) void attn_fwd_bf16_g1(const u16* __restrict__ qkv, u16* __restrict__ o,
                                                     float* __restrict__ lse,
                                                     const int64_t* __restrict__ lens, int T, int H,
                                                     float scale) {
  __shared__ __attribute__((aligned(16))) u16 Ks[QB * LDR];
  __shared__ __attribute__((aligned(16))) u16 Vs[QB * LDT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blockIdx.x * QB;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* obase = o + (int64_t)b * T * ldo + h * DH;

  if (q0 >= L) {
    for (int e = tid; e < QB * DH / 8; e += 256) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, q = q0 + row;
      if (q < T) *reinterpret_cast<uint4*>(obase + (int64_t)q * ldo + col) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < QB && q0 + tid < T) lse[(int64_t)bh * T + q0 + tid] = 0.f;
    return;
  }
  const int q = q0 + wave * 16 + r16;
  bf16x8 qf[4];
  load_frag(qf, base + (int64_t)min(q, T - 1) * ld + h * DH, g);

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 oacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (L + QB - 1) / QB;
  const u16* kbase = base + (int64_t)H * DH + h * DH;
  const u16* vbase = base + 2LL * H * DH + h * DH;
  uint4 kr[4], vr[4];
  load_regs<256>(kr, kbase, ld, 0, T, tid);
  load_regs<256>(vr, vbase, ld, 0, T, tid);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    store_regs<LDR, 256>(Ks, kr, tid);
    store_regs<LDT, 256>(Vs, vr, tid);
    __syncthreads();
    if (kt + 1 < nkt) {  // next tile's loads in flight during this tile's MFMAs
      load_regs<256>(kr, kbase, ld, (kt + 1) * QB, T, tid);
      load_regs<256>(vr, vbase, ld, (kt + 1) * QB, T, tid);
    }
    f32x4 s[4];
    float mt = -INFINITY;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = dot_tile<LDR>(Ks, 16 * st, qf, g, r16);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * QB + 16 * st + 4 * g + r;
        const float x = key < L ? s[st][r] * scale : -INFINITY;
        s[st][r] = x;
        mt = fmaxf(mt, x);
      }
    }
    mt = group4_max(mt);
    const float m_new = fmaxf(m_run, mt);
    const float alpha = __expf(m_run - m_new);
    float ps = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = __expf(s[st][r] - m_new);
        s[st][r] = pv;
        ps += pv;
      }
    ps = group4_sum(ps);
    l_run = l_run * alpha + ps;
    m_run = m_new;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) oacc[ds] *= alpha;
#pragma unroll
    for (int c = 0; c < 2; ++c) accum_t<LDT>(oacc, Vs, 32 * c, pack8(s[2 * c], s[2 * c + 1]), g, q4, p4);
  }
  if (q < T) {
    const float inv = 1.f / l_run;
#pragma unroll
    for (int d = 0; d < 4; ++d)
      store8x2_bf16(obase + (int64_t)q * ldo + 32 * d, oacc[2 * d] * inv, oacc[2 * d + 1] * inv, g);
    if (g == 0) lse[(int64_t)bh * T + q] = m_run + __logf(l_run);
  }
}

__global__ void attn_bwd_delta_bf16_g1(const u16* __restrict__ o, const u16* __restrict__ d_o,
                                    float* __restrict__ delta, int64_t rows, int T, int H) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= rows * H) return;
  const int64_t r = w / H;
  const int h = (int)(w - r * H);
  const u16* po = o + r * H * DH + h * DH + 2 * lane;
  const u16* pd = d_o + r * H * DH + h * DH + 2 * lane;
  float s = wave_sum(bf2f(po[0]) * bf2f(pd[0]) + bf2f(po[1]) * bf2f(pd[1]));
  if (lane == 0) {
    const int64_t b = r / T, q = r - b * T;
    delta[(b * H + h) * T + q] = s;
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq_bf16_g1(const u16* __restrict__ qkv,
                                                        const u16* __restrict__ d_o,
                                                        const float* __restrict__ lse,
                                                        const float* __restrict__ delta,
                                                        u16* __restrict__ d_qkv,
                                                        const int64_t* __restrict__ lens, int T,
                                                        int H, float scale) {
  __shared__ __attribute__((aligned(16))) u16 Ks[QB * LDR];
  __shared__ __attribute__((aligned(16))) u16 Vs[QB * LDR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blockIdx.x * QB;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* dbase = d_qkv + (int64_t)b * T * ld + h * DH;

  if (q0 >= L) {
    for (int e = tid; e < QB * DH / 8; e += 256) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, qq = q0 + row;
      if (qq < T) *reinterpret_cast<uint4*>(dbase + (int64_t)qq * ld + col) = make_uint4(0u, 0u, 0u, 0u);
    }
    return;
  }
  const int q = q0 + wave * 16 + r16;
  const int qc = min(q, T - 1);
  bf16x8 qf[4], df[4];
  load_frag(qf, base + (int64_t)qc * ld + h * DH, g);
  load_frag(df, d_o + ((int64_t)b * T + qc) * ldo + h * DH, g);
  const float my_lse = lse[(int64_t)bh * T + qc];
  const float my_delta = delta[(int64_t)bh * T + qc];
  const bool qvalid = q < L;

  f32x4 dq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (L + QB - 1) / QB;
  const u16* kbase = base + (int64_t)H * DH + h * DH;
  const u16* vbase = base + 2LL * H * DH + h * DH;
  uint4 kr[4], vr[4];
  load_regs<256>(kr, kbase, ld, 0, T, tid);
  load_regs<256>(vr, vbase, ld, 0, T, tid);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    store_regs<LDR, 256>(Ks, kr, tid);
    store_regs<LDR, 256>(Vs, vr, tid);
    __syncthreads();
    if (kt + 1 < nkt) {
      load_regs<256>(kr, kbase, ld, (kt + 1) * QB, T, tid);
      load_regs<256>(vr, vbase, ld, (kt + 1) * QB, T, tid);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 dsv[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int st = 2 * c + half;
        const f32x4 s = dot_tile<LDR>(Ks, 16 * st, qf, g, r16);   // S^T[key][q]
        const f32x4 dp = dot_tile<LDR>(Vs, 16 * st, df, g, r16);  // dP^T[key][q]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * QB + 16 * st + 4 * g + r;
          const float pv = (key < L && qvalid) ? __expf(s[r] * scale - my_lse) : 0.f;
          dsv[half][r] = pv * (dp[r] - my_delta);
        }
      }
      accum_t<LDR>(dq, Ks, 32 * c, pack8(dsv[0], dsv[1]), g, q4, p4);  // dQ^T += K^T dS^T
    }
  }
  if (q < T) {
#pragma unroll
    for (int d = 0; d < 4; ++d)
      store8x2_bf16(dbase + (int64_t)q * ld + 32 * d, dq[2 * d] * scale, dq[2 * d + 1] * scale, g);
  }
}

template <int MINB>
__global__ __launch_bounds__(256, MINB) void attn_bwd_dkdv_bf16_g1(const u16* __restrict__ qkv,
                                                          const u16* __restrict__ d_o,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta,
                                                          u16* __restrict__ d_qkv,
                                                          const int64_t* __restrict__ lens, int T,
                                                          int H, float scale) {
  __shared__ __attribute__((aligned(16))) u16 Qs[QB * LDR];
  __shared__ __attribute__((aligned(16))) u16 Ds[QB * LDR];
  __shared__ float lse_s[QB], del_s[QB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int k0 = blockIdx.x * QB;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* dk_base = d_qkv + (int64_t)b * T * ld + (int64_t)H * DH + h * DH;
  u16* dv_base = d_qkv + (int64_t)b * T * ld + 2LL * H * DH + h * DH;

  if (k0 >= L) {
    for (int e = tid; e < QB * DH / 8; e += 256) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, k = k0 + row;
      if (k < T) {
        *reinterpret_cast<uint4*>(dk_base + (int64_t)k * ld + col) = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(dv_base + (int64_t)k * ld + col) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    return;
  }
  const int key = k0 + wave * 16 + r16;
  const int kc = min(key, T - 1);
  bf16x8 kf[4], vf[4];
  load_frag(kf, base + (int64_t)kc * ld + (int64_t)H * DH + h * DH, g);
  load_frag(vf, base + (int64_t)kc * ld + 2LL * H * DH + h * DH, g);
  const bool kvalid = key < L;

  f32x4 dk[8], dv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nqt = (L + QB - 1) / QB;
  const u16* qbase = base + h * DH;
  const u16* dobase = d_o + (int64_t)b * T * ldo + h * DH;
  uint4 qr[4], dr[4];
  float lr_ = 0.f, dl_ = 0.f;
  auto load_q = [&](int qt) {
    load_regs<256>(qr, qbase, ld, qt * QB, T, tid);
    load_regs<256>(dr, dobase, ldo, qt * QB, T, tid);
    if (tid < QB) {
      const int qq = qt * QB + tid;
      lr_ = qq < T ? lse[(int64_t)bh * T + qq] : 0.f;
      dl_ = qq < T ? delta[(int64_t)bh * T + qq] : 0.f;
    }
  };
  load_q(0);
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();
    store_regs<LDR, 256>(Qs, qr, tid);
    store_regs<LDR, 256>(Ds, dr, tid);
    if (tid < QB) {
      lse_s[tid] = lr_;
      del_s[tid] = dl_;
    }
    __syncthreads();
    if (qt + 1 < nqt) load_q(qt + 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 pp[2], dsv[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int qs = 2 * c + half;
        const f32x4 s = dot_tile<LDR>(Qs, 16 * qs, kf, g, r16);   // S[q][key]
        const f32x4 dp = dot_tile<LDR>(Ds, 16 * qs, vf, g, r16);  // dP[q][key]
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * qs + 4 * g + r, qq = qt * QB + ql;
          const float pv = (qq < L && kvalid) ? __expf(s[r] * scale - lse_s[ql]) : 0.f;
          pp[half][r] = pv;
          dsv[half][r] = pv * (dp[r] - del_s[ql]);
        }
      }
      accum_t<LDR>(dv, Ds, 32 * c, pack8(pp[0], pp[1]), g, q4, p4);    // dV^T += dO^T P
      accum_t<LDR>(dk, Qs, 32 * c, pack8(dsv[0], dsv[1]), g, q4, p4);  // dK^T += Q^T dS
    }
  }
  if (key < T) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      store8x2_bf16(dk_base + (int64_t)key * ld + 32 * d, dk[2 * d] * scale, dk[2 * d + 1] * scale, g);
      store8x2_bf16(dv_base + (int64_t)key * ld + 32 * d, dv[2 * d], dv[2 * d + 1], g);
    }
  }
}

// ---- two 16-row groups per wave
template <int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_fwd_bf16(const u16* __restrict__ qkv, u16* __restrict__ o,
                                                         float* __restrict__ lse,
                                                         const int64_t* __restrict__ lens, int T, int H,
                                                         float scale) {
  constexpr int NT = NW * 64, QBLK = NW * 32, PER = 1024 / NT;
  __shared__ __attribute__((aligned(16))) u16 Ks[QB * LDR];
  __shared__ __attribute__((aligned(16))) u16 Vs[QB * LDT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blockIdx.x * QBLK;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* obase = o + (int64_t)b * T * ldo + h * DH;

  if (q0 >= L) {  // fully padded query block: outputs are masked downstream; write zeros
    for (int e = tid; e < QBLK * DH / 8; e += NT) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, q = q0 + row;
      if (q < T) *reinterpret_cast<uint4*>(obase + (int64_t)q * ldo + col) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < QBLK && q0 + tid < T) lse[(int64_t)bh * T + q0 + tid] = 0.f;
    return;
  }
  bf16x8 qf[2][4];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    load_frag(qf[gq], base + (int64_t)min(q, T - 1) * ld + h * DH, g);
  }
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
  f32x4 oacc[2][8];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq)
#pragma unroll
    for (int i = 0; i < 8; ++i) oacc[gq][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (L + QB - 1) / QB;
  const u16* kbase = base + (int64_t)H * DH + h * DH;
  const u16* vbase = base + 2LL * H * DH + h * DH;
  uint4 kr[PER], vr[PER];
  load_regs<NT>(kr, kbase, ld, 0, T, tid);
  load_regs<NT>(vr, vbase, ld, 0, T, tid);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    store_regs<LDR, NT>(Ks, kr, tid);
    store_regs<LDT, NT>(Vs, vr, tid);
    __syncthreads();
    if (kt + 1 < nkt) {  // next tile's loads in flight during this tile's MFMAs
      load_regs<NT>(kr, kbase, ld, (kt + 1) * QB, T, tid);
      load_regs<NT>(vr, vbase, ld, (kt + 1) * QB, T, tid);
    }
    f32x4 s[2][4];  // S^T[key 16 st + 4 g + r][query r16] per query group
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      bf16x8 kfr[4];
      row_frags<LDR>(kfr, Ks, 16 * st + r16, g);
#pragma unroll
      for (int gq = 0; gq < 2; ++gq) s[gq][st] = chain4(kfr, qf[gq]);
    }
#pragma unroll
    for (int gq = 0; gq < 2; ++gq) {
      float mt = -INFINITY;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * QB + 16 * st + 4 * g + r;
          const float x = key < L ? s[gq][st][r] * scale : -INFINITY;
          s[gq][st][r] = x;
          mt = fmaxf(mt, x);
        }
      mt = group4_max(mt);
      const float m_new = fmaxf(m_run[gq], mt);
      const float alpha = __expf(m_run[gq] - m_new);
      float ps = 0.f;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __expf(s[gq][st][r] - m_new);
          s[gq][st][r] = pv;
          ps += pv;
        }
      ps = group4_sum(ps);
      l_run[gq] = l_run[gq] * alpha + ps;
      m_run[gq] = m_new;
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) oacc[gq][ds] *= alpha;
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
      accum_t2<LDT>(oacc, Vs, 32 * c, pack8(s[0][2 * c], s[0][2 * c + 1]),
                    pack8(s[1][2 * c], s[1][2 * c + 1]), g, q4, p4);
  }
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    if (q < T) {
      const float inv = 1.f / l_run[gq];
#pragma unroll
      for (int ds = 0; ds < 8; ++ds)
        store4_bf16(obase + (int64_t)q * ldo + 16 * ds + 4 * g, oacc[gq][ds] * inv);
      if (g == 0) lse[(int64_t)bh * T + q] = m_run[gq] + __logf(l_run[gq]);
    }
  }
}

// dQ, plus delta[q] = sum_d dO[q, d] O[q, d] for the block's queries (written to `delta` for
// the dK/dV kernel; padded queries get 0)
template <int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_dq_bf16(const u16* __restrict__ qkv,
                                                            const u16* __restrict__ o,
                                                            const u16* __restrict__ d_o,
                                                            const float* __restrict__ lse,
                                                            float* __restrict__ delta,
                                                            u16* __restrict__ d_qkv,
                                                            const int64_t* __restrict__ lens, int T,
                                                            int H, float scale) {
  constexpr int NT = NW * 64, QBLK = NW * 32, PER = 1024 / NT;
  __shared__ __attribute__((aligned(16))) u16 Ks[QB * LDR];
  __shared__ __attribute__((aligned(16))) u16 Vs[QB * LDR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blockIdx.x * QBLK;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* dbase = d_qkv + (int64_t)b * T * ld + h * DH;

  if (q0 >= L) {
    for (int e = tid; e < QBLK * DH / 8; e += NT) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, qq = q0 + row;
      if (qq < T) *reinterpret_cast<uint4*>(dbase + (int64_t)qq * ld + col) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < QBLK && q0 + tid < T) delta[(int64_t)bh * T + q0 + tid] = 0.f;
    return;
  }
  bf16x8 qf[2][4], df[2][4];
  float my_lse[2], my_delta[2];
  bool qvalid[2];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    const int qc = min(q, T - 1);
    load_frag(qf[gq], base + (int64_t)qc * ld + h * DH, g);
    load_frag(df[gq], d_o + ((int64_t)b * T + qc) * ldo + h * DH, g);
    bf16x8 of[4];
    load_frag(of, o + ((int64_t)b * T + qc) * ldo + h * DH, g);
    float part = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) part += (float)of[c][e] * (float)df[gq][c][e];
    qvalid[gq] = q < L;
    my_delta[gq] = qvalid[gq] ? group4_sum(part) : 0.f;
    my_lse[gq] = lse[(int64_t)bh * T + qc];
    if (g == 0 && q < T) delta[(int64_t)bh * T + q] = my_delta[gq];
  }

  f32x4 dq[2][8];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq)
#pragma unroll
    for (int i = 0; i < 8; ++i) dq[gq][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (L + QB - 1) / QB;
  const u16* kbase = base + (int64_t)H * DH + h * DH;
  const u16* vbase = base + 2LL * H * DH + h * DH;
  uint4 kr[PER], vr[PER];
  load_regs<NT>(kr, kbase, ld, 0, T, tid);
  load_regs<NT>(vr, vbase, ld, 0, T, tid);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    store_regs<LDR, NT>(Ks, kr, tid);
    store_regs<LDR, NT>(Vs, vr, tid);
    __syncthreads();
    if (kt + 1 < nkt) {
      load_regs<NT>(kr, kbase, ld, (kt + 1) * QB, T, tid);
      load_regs<NT>(vr, vbase, ld, (kt + 1) * QB, T, tid);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 dsv[2][2];  // [query group][half]
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int st = 2 * c + half;
        bf16x8 kfr[4], vfr[4];
        row_frags<LDR>(kfr, Ks, 16 * st + r16, g);
        row_frags<LDR>(vfr, Vs, 16 * st + r16, g);
#pragma unroll
        for (int gq = 0; gq < 2; ++gq) {
          const f32x4 s = chain4(kfr, qf[gq]);   // S^T[key][q]
          const f32x4 dp = chain4(vfr, df[gq]);  // dP^T[key][q]
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kt * QB + 16 * st + 4 * g + r;
            const float pv = (key < L && qvalid[gq]) ? __expf(s[r] * scale - my_lse[gq]) : 0.f;
            dsv[gq][half][r] = pv * (dp[r] - my_delta[gq]);
          }
        }
      }
      accum_t2<LDR>(dq, Ks, 32 * c, pack8(dsv[0][0], dsv[0][1]), pack8(dsv[1][0], dsv[1][1]), g,
                    q4, p4);  // dQ^T += K^T dS^T
    }
  }
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    if (q < T) {
#pragma unroll
      for (int ds = 0; ds < 8; ++ds)
        store4_bf16(dbase + (int64_t)q * ld + 16 * ds + 4 * g, dq[gq][ds] * scale);
    }
  }
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dkdv_bf16(const u16* __restrict__ qkv,
                                                              const u16* __restrict__ d_o,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ delta,
                                                              u16* __restrict__ d_qkv,
                                                              const int64_t* __restrict__ lens,
                                                              int T, int H, float scale) {
  constexpr int NT = NW * 64, KBLK = NW * 32, PER = 1024 / NT;
  __shared__ __attribute__((aligned(16))) u16 Qs[QB * LDR];
  __shared__ __attribute__((aligned(16))) u16 Ds[QB * LDR];
  __shared__ float lse_s[QB], del_s[QB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int q4 = r16 >> 2, p4 = r16 & 3;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int k0 = blockIdx.x * KBLK;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* dk_base = d_qkv + (int64_t)b * T * ld + (int64_t)H * DH + h * DH;
  u16* dv_base = d_qkv + (int64_t)b * T * ld + 2LL * H * DH + h * DH;

  if (k0 >= L) {
    for (int e = tid; e < KBLK * DH / 8; e += NT) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, k = k0 + row;
      if (k < T) {
        *reinterpret_cast<uint4*>(dk_base + (int64_t)k * ld + col) = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(dv_base + (int64_t)k * ld + col) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    return;
  }
  bf16x8 kf[2][4], vf[2][4];
  bool kvalid[2];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) {
    const int key = k0 + wave * 32 + kg * 16 + r16;
    const int kc = min(key, T - 1);
    load_frag(kf[kg], base + (int64_t)kc * ld + (int64_t)H * DH + h * DH, g);
    load_frag(vf[kg], base + (int64_t)kc * ld + 2LL * H * DH + h * DH, g);
    kvalid[kg] = key < L;
  }
  f32x4 dk[2][8], dv[2][8];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int i = 0; i < 8; ++i) dk[kg][i] = dv[kg][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nqt = (L + QB - 1) / QB;
  const u16* qbase = base + h * DH;
  const u16* dobase = d_o + (int64_t)b * T * ldo + h * DH;
  uint4 qr[PER], dr[PER];
  float lr_ = 0.f, dl_ = 0.f;
  auto load_q = [&](int qt) {
    load_regs<NT>(qr, qbase, ld, qt * QB, T, tid);
    load_regs<NT>(dr, dobase, ldo, qt * QB, T, tid);
    if (tid < QB) {
      const int qq = qt * QB + tid;
      lr_ = qq < T ? lse[(int64_t)bh * T + qq] : 0.f;
      dl_ = qq < T ? delta[(int64_t)bh * T + qq] : 0.f;
    }
  };
  load_q(0);
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();
    store_regs<LDR, NT>(Qs, qr, tid);
    store_regs<LDR, NT>(Ds, dr, tid);
    if (tid < QB) {
      lse_s[tid] = lr_;
      del_s[tid] = dl_;
    }
    __syncthreads();
    if (qt + 1 < nqt) load_q(qt + 1);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 pp[2][2], dsv[2][2];  // [key group][half]
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int qs = 2 * c + half;
        bf16x8 qfr[4], dfr[4];
        row_frags<LDR>(qfr, Qs, 16 * qs + r16, g);
        row_frags<LDR>(dfr, Ds, 16 * qs + r16, g);
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
          const f32x4 s = chain4(qfr, kf[kg]);   // S[q][key]
          const f32x4 dp = chain4(dfr, vf[kg]);  // dP[q][key]
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ql = 16 * qs + 4 * g + r, qq = qt * QB + ql;
            const float pv = (qq < L && kvalid[kg]) ? __expf(s[r] * scale - lse_s[ql]) : 0.f;
            pp[kg][half][r] = pv;
            dsv[kg][half][r] = pv * (dp[r] - del_s[ql]);
          }
        }
      }
      accum_t2<LDR>(dv, Ds, 32 * c, pack8(pp[0][0], pp[0][1]), pack8(pp[1][0], pp[1][1]), g, q4,
                    p4);  // dV^T += dO^T P
      accum_t2<LDR>(dk, Qs, 32 * c, pack8(dsv[0][0], dsv[0][1]), pack8(dsv[1][0], dsv[1][1]), g,
                    q4, p4);  // dK^T += Q^T dS
    }
  }
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) {
    const int key = k0 + wave * 32 + kg * 16 + r16;
    if (key < T) {
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) {
        store4_bf16(dk_base + (int64_t)key * ld + 16 * ds + 4 * g, dk[kg][ds] * scale);
        store4_bf16(dv_base + (int64_t)key * ld + 16 * ds + 4 * g, dv[kg][ds]);
      }
    }
  }
}

// ---- LDS-DMA staged kernels (T >= 256; FS2_TUNE_ATTN_DMA = 0, default) -------------------
// The K / V (Q / dO) tiles arrive by buffer_load ... lds into a ring of LDS slots: no register
// round trip, no ds_write, ONE barrier per tile, and the next tile's DMA in flight under the
// current tile's MFMAs.  Tile image: 64 rows x 256 B, 16-B chunk ch of row r stored at chunk
// ch ^ ((r & 7) << 1).  That one image is conflict-free for both reads the kernels make of it:
// the row-fragment reads (ds_read_b128 of the 16x16x32 operand: rows r16, chunks g + 4c) and
// the transposed reads (ds_read_b64_tr_b16: rows 4g + q of an 8-aligned group, chunks
// 2 ds + p / 2).  A DMA wave-instruction writes its 64 x 16 B contiguously (4 rows), so the
// swizzle is applied on the source side: lane i of the instruction staging rows 4I .. 4I + 3
// fetches logical chunk (i & 15) ^ swz(row) of row 4I + i / 16.
// Softmax VALU work, which at d_head = 128 costs more issue cycles per score than the MFMAs
// (v_exp_f32 is quarter rate): scores stay unscaled, the row maximum is taken on them (scale
// > 0), and p = exp2(fma(s, scale log2 e, -m')) is one FMA + v_exp_f32 per score; keys are
// masked only in the last (partial) key tile; invalid queries carry lse = +inf into the
// backward (p = 0 with no per-score select); the O *= alpha rescale is skipped when no lane's
// running maximum moved (alpha == 1 exactly: the skip is exact).  Results match the
// register-staged kernels to fp32 rounding of the exponent argument (tests: within 2e-3).
namespace {
constexpr int IMG = 64 * DH;  // elements of one tile image

FS2_DEV int swz(int r) { return (r & 7) << 1; }

// per-lane LDS-DMA sources of a 64-row tile staged by NW waves (16 / NW instructions each)
template <int NW>
struct TileDma {
  static constexpr int NI = 16 / NW;
  uint32_t vo[NI];
  int row[NI];
  FS2_DEV void init(int64_t ld, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int I = wave * NI + j, r = 4 * I + (lane >> 4);
      row[j] = r;
      vo[j] = (uint32_t)((r * ld + (((lane & 15) ^ swz(r)) << 3)) * 2);
    }
  }
  // rows t0 .. t0 + 63 of the [nrows][ld] matrix behind rs into img (rows past nrows: zeros)
  FS2_DEV void issue(__amdgpu_buffer_rsrc_t rs, u16* img, int t0, int nrows, int64_t ld,
                     int wave) const {
    const int lim = nrows - t0;
    const uint32_t so = (uint32_t)(t0 * ld * 2);
#pragma unroll
    for (int j = 0; j < NI; ++j) glds16_buf(rs, img + (wave * NI + j) * 512, row[j] < lim ? vo[j] : kOOB, so);
  }
};

// per-lane read offsets into a tile image: row fragments (chunks g + 4c of row r16) and
// transposed blocks (rows 4g + q, columns 16 ds + 4p)
struct ImgRd {
  int ro[4], to[8];
  FS2_DEV void init(int g, int r16, int q, int p) {
#pragma unroll
    for (int c = 0; c < 4; ++c) ro[c] = r16 * DH + (((g + 4 * c) ^ swz(r16)) << 3);
    const int r = 4 * g + q;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) to[ds] = r * DH + (((2 * ds + (p >> 1)) ^ swz(r)) << 3) + 4 * (p & 1);
  }
  // the 4 row fragments of rows row0 + r16 (row0 % 16 == 0)
  FS2_DEV void rows(bf16x8 (&f)[4], const u16* img, int row0) const {
#pragma unroll
    for (int c = 0; c < 4; ++c) f[c] = *reinterpret_cast<const bf16x8*>(img + row0 * DH + ro[c]);
  }
  // transposed fragment of columns 16 ds .. over rows {rb + 4g + q} u {rb + 16 + 4g + q}
  FS2_DEV bf16x8 tr(const u16* img, int rb, int ds) const {
    const u16* p0 = img + rb * DH + to[ds];
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 16 * DH));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
};

FS2_DEV f32x4 chain4_img(const ImgRd& rd, const u16* img, int row0, const bf16x8 (&b)[4]) {
  bf16x8 a[4];
  rd.rows(a, img, row0);
  return chain4(a, b);
}

// The ring: slot s of STAGES holds NM tile images; prologue issues tiles 0 .. STAGES-2; per tile
// kt: counted vmcnt (tile kt landed), barrier (visible to all waves, and every wave is done with
// tile kt-1 whose slot the refill overwrites), refill with tile kt + STAGES - 1, compute.
// The last tile (the only one holding keys / queries past the length) runs a separate body,
// peeled out of the loop (a branch between two inlined bodies inside it spilled registers).
template <int STAGES, int PER, typename Issue, typename Full, typename Last>
FS2_DEV void tile_loop(int nt, Issue&& issue, Full&& full, Last&& last) {
  for (int t = 0; t < STAGES - 1 && t < nt; ++t) issue(t, t);
  auto step = [&](int kt) {
    const int ahead = nt - 1 - kt < STAGES - 2 ? nt - 1 - kt : STAGES - 2;
    vm_wait_tiles<PER>(ahead);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nt) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
  };
  for (int kt = 0; kt + 1 < nt; ++kt) {
    step(kt);
    full(kt, kt % STAGES);
  }
  if (nt > 0) {
    step(nt - 1);
    last(nt - 1, (nt - 1) % STAGES);
  }
}
}  // namespace

// (query / key block, bh) of this workgroup.  xg != 0: the blocks of one (utterance, head) are
// dealt to one XCD -- blocks b and b + 8 share an XCD under round-robin dispatch (speed only,
// never correctness) -- so its K / V (Q / dO) tiles are fetched into one L2, while the (b, h)
// pairs still go round-robin over the XCDs (a length mix on each).  Needs gridDim.y % 8 == 0.
namespace {
FS2_DEV void attn_block(int xg, int& blk, int& bh) {
  blk = blockIdx.x;
  bh = blockIdx.y;
  if (xg) {
    const int nx = gridDim.x, lin = blockIdx.y * nx + blockIdx.x;
    const int slot = lin >> 3, grp = slot / nx;
    bh = (lin & 7) + 8 * grp;
    blk = slot - grp * nx;
  }
}
}  // namespace

// forward: 4 waves x 32 queries (two 16-row groups per wave), K / V tiles by LDS-DMA
template <int STAGES>
__global__ __launch_bounds__(256, STAGES == 2 ? 2 : 1) void attn_fwd_dma(
    const u16* __restrict__ qkv, u16* __restrict__ o, float* __restrict__ lse,
    const int64_t* __restrict__ lens, int T, int H, float scale, int xg) {
  constexpr int NW = 4, NT = 256, QBLK = 128;
  __shared__ __attribute__((aligned(1024))) u16 smem[STAGES * 2 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q4 = r16 >> 2, p4 = r16 & 3;
  int blk, bh;
  attn_block(xg, blk, bh);
  const int b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blk * QBLK;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* obase = o + (int64_t)b * T * ldo + h * DH;

  if (q0 >= L) {
    for (int e = tid; e < QBLK * DH / 8; e += NT) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, q = q0 + row;
      if (q < T) *reinterpret_cast<uint4*>(obase + (int64_t)q * ldo + col) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < QBLK && q0 + tid < T) lse[(int64_t)bh * T + q0 + tid] = 0.f;
    return;
  }
  const auto k_rs = buf_rsrc(base + (int64_t)H * DH + h * DH, (int64_t)T * ld * 2);
  const auto v_rs = buf_rsrc(base + 2LL * H * DH + h * DH, (int64_t)T * ld * 2);
  TileDma<NW> dma;
  dma.init(ld, wave, lane);
  ImgRd rd;
  rd.init(g, r16, q4, p4);
  const int nkt = (L + QB - 1) / QB;
  auto issue = [&](int kt, int slot) {
    u16* Ks = smem + slot * 2 * IMG;
    dma.issue(k_rs, Ks, kt * QB, T, ld, wave);
    dma.issue(v_rs, Ks + IMG, kt * QB, T, ld, wave);
  };

  bf16x8 qf[2][4];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    load_frag(qf[gq], base + (int64_t)min(q, T - 1) * ld + h * DH, g);
  }
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
  f32x4 oacc[2][8];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq)
#pragma unroll
    for (int i = 0; i < 8; ++i) oacc[gq][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float c2 = scale * 1.4426950408889634f;  // scores -> log2 units
  auto body = [&](auto mask_c, int kt, int slot) {
    constexpr bool MASK = decltype(mask_c)::value;
    const u16* Ks = smem + slot * 2 * IMG;
    const u16* Vs = Ks + IMG;
    f32x4 s[2][4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      bf16x8 kfr[4];
      rd.rows(kfr, Ks, 16 * st);
#pragma unroll
      for (int gq = 0; gq < 2; ++gq) s[gq][st] = chain4(kfr, qf[gq]);
    }
    float alpha[2];
#pragma unroll
    for (int gq = 0; gq < 2; ++gq) {
      float mt = -INFINITY;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (MASK && kt * QB + 16 * st + 4 * g + r >= L) s[gq][st][r] = -INFINITY;
          mt = fmaxf(mt, s[gq][st][r]);
        }
      mt = group4_max(mt);
      const float m_new = fmaxf(m_run[gq], mt * c2);
      alpha[gq] = __builtin_amdgcn_exp2f(m_run[gq] - m_new);
      float ps = 0.f;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = __builtin_amdgcn_exp2f(fmaf(s[gq][st][r], c2, -m_new));
          s[gq][st][r] = pv;
          ps += pv;
        }
      ps = group4_sum(ps);
      l_run[gq] = l_run[gq] * alpha[gq] + ps;
      m_run[gq] = m_new;
    }
    // O *= alpha unless no lane's maximum moved (then alpha == 1 everywhere: exact skip); on
    // the first tile O is zero
    if (kt > 0 && __ballot(alpha[0] != 1.f || alpha[1] != 1.f)) {
#pragma unroll
      for (int gq = 0; gq < 2; ++gq)
#pragma unroll
        for (int ds = 0; ds < 8; ++ds) oacc[gq][ds] *= alpha[gq];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bf16x8 w0 = pack8(s[0][2 * c], s[0][2 * c + 1]), w1 = pack8(s[1][2 * c], s[1][2 * c + 1]);
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) {
        const bf16x8 a = rd.tr(Vs, 32 * c, ds);
        oacc[0][ds] = MFMA_BF16(a, w0, oacc[0][ds]);
        oacc[1][ds] = MFMA_BF16(a, w1, oacc[1][ds]);
      }
    }
  };
  tile_loop<STAGES, 2 * TileDma<NW>::NI>(nkt, issue, [&](int kt, int slot) { body(std::false_type{}, kt, slot); },
      [&](int kt, int slot) { body(std::true_type{}, kt, slot); });
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    if (q < T) {
      const float inv = 1.f / l_run[gq];
#pragma unroll
      for (int d = 0; d < 4; ++d)
        store8x2_bf16(obase + (int64_t)q * ldo + 32 * d, oacc[gq][2 * d] * inv, oacc[gq][2 * d + 1] * inv, g);
      if (g == 0) lse[(int64_t)bh * T + q] = (m_run[gq] + __log2f(l_run[gq])) * 0.6931471805599453f;
    }
  }
}

// dQ (+ delta), 4 waves x 32 queries, K / V tiles by LDS-DMA
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_dma(
    const u16* __restrict__ qkv, const u16* __restrict__ o, const u16* __restrict__ d_o,
    const float* __restrict__ lse, float* __restrict__ delta, u16* __restrict__ d_qkv,
    const int64_t* __restrict__ lens, int T, int H, float scale, int xg) {
  constexpr int NW = 4, NT = 256, QBLK = 128, STAGES = 2;
  __shared__ __attribute__((aligned(1024))) u16 smem[STAGES * 2 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q4 = r16 >> 2, p4 = r16 & 3;
  int blk, bh;
  attn_block(xg, blk, bh);
  const int b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blk * QBLK;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* dbase = d_qkv + (int64_t)b * T * ld + h * DH;

  if (q0 >= L) {
    for (int e = tid; e < QBLK * DH / 8; e += NT) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, qq = q0 + row;
      if (qq < T) *reinterpret_cast<uint4*>(dbase + (int64_t)qq * ld + col) = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid < QBLK && q0 + tid < T) delta[(int64_t)bh * T + q0 + tid] = 0.f;
    return;
  }
  const auto k_rs = buf_rsrc(base + (int64_t)H * DH + h * DH, (int64_t)T * ld * 2);
  const auto v_rs = buf_rsrc(base + 2LL * H * DH + h * DH, (int64_t)T * ld * 2);
  TileDma<NW> dma;
  dma.init(ld, wave, lane);
  ImgRd rd;
  rd.init(g, r16, q4, p4);
  const int nkt = (L + QB - 1) / QB;
  auto issue = [&](int kt, int slot) {
    u16* Ks = smem + slot * 2 * IMG;
    dma.issue(k_rs, Ks, kt * QB, T, ld, wave);
    dma.issue(v_rs, Ks + IMG, kt * QB, T, ld, wave);
  };
  issue(0, 0);  // the first tile's DMA flies under the delta computation

  bf16x8 qf[2][4], df[2][4];
  float my_lse[2], my_delta[2];
  bool qvalid[2];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    const int qc = min(q, T - 1);
    load_frag(qf[gq], base + (int64_t)qc * ld + h * DH, g);
    load_frag(df[gq], d_o + ((int64_t)b * T + qc) * ldo + h * DH, g);
    bf16x8 of[4];
    load_frag(of, o + ((int64_t)b * T + qc) * ldo + h * DH, g);
    float part = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) part += (float)of[c][e] * (float)df[gq][c][e];
    qvalid[gq] = q < L;
    my_delta[gq] = qvalid[gq] ? group4_sum(part) : 0.f;
    // lse in log2 units; an invalid query's +inf makes every p of its column 0
    my_lse[gq] = qvalid[gq] ? lse[(int64_t)bh * T + qc] * 1.4426950408889634f : INFINITY;
    if (g == 0 && q < T) delta[(int64_t)bh * T + q] = my_delta[gq];
  }
  const float c2 = scale * 1.4426950408889634f;

  f32x4 dq[2][8];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq)
#pragma unroll
    for (int i = 0; i < 8; ++i) dq[gq][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto body = [&](auto mask_c, int kt, int slot) {
    constexpr bool MASK = decltype(mask_c)::value;
    const u16* Ks = smem + slot * 2 * IMG;
    const u16* Vs = Ks + IMG;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 dsv[2][2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int st = 2 * c + half;
        bf16x8 kfr[4], vfr[4];
        rd.rows(kfr, Ks, 16 * st);
        rd.rows(vfr, Vs, 16 * st);
#pragma unroll
        for (int gq = 0; gq < 2; ++gq) {
          const f32x4 s = chain4(kfr, qf[gq]);
          const f32x4 dp = chain4(vfr, df[gq]);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float pv = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -my_lse[gq]));
            if (MASK && kt * QB + 16 * st + 4 * g + r >= L) pv = 0.f;
            dsv[gq][half][r] = pv * (dp[r] - my_delta[gq]);
          }
        }
      }
      const bf16x8 w0 = pack8(dsv[0][0], dsv[0][1]), w1 = pack8(dsv[1][0], dsv[1][1]);
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) {
        const bf16x8 a = rd.tr(Ks, 32 * c, ds);
        dq[0][ds] = MFMA_BF16(a, w0, dq[0][ds]);
        dq[1][ds] = MFMA_BF16(a, w1, dq[1][ds]);
      }
    }
  };
  // tile 0 is already in flight: the ring starts at tile 1
  tile_loop<STAGES, 2 * TileDma<NW>::NI>(nkt, [&](int kt, int slot) { if (kt > 0) issue(kt, slot); },
                                        [&](int kt, int slot) { body(std::false_type{}, kt, slot); },
      [&](int kt, int slot) { body(std::true_type{}, kt, slot); });
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    const int q = q0 + wave * 32 + gq * 16 + r16;
    if (q < T) {
#pragma unroll
      for (int d = 0; d < 4; ++d)
        store8x2_bf16(dbase + (int64_t)q * ld + 32 * d, dq[gq][2 * d] * scale, dq[gq][2 * d + 1] * scale, g);
    }
  }
}

// dK / dV: 4 waves x 16 keys, Q / dO tiles (+ the tile's lse / delta) by LDS-DMA
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_dma(
    const u16* __restrict__ qkv, const u16* __restrict__ d_o, const float* __restrict__ lse,
    const float* __restrict__ delta, u16* __restrict__ d_qkv, const int64_t* __restrict__ lens,
    int T, int H, float scale, int xg) {
  constexpr int NW = 4, STAGES = 2;
  constexpr int SLOT_E = 2 * IMG + 2 * QB * 2;  // Q image, dO image, lse[64], delta[64] (fp32)
  __shared__ __attribute__((aligned(1024))) u16 smem[STAGES * SLOT_E];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q4 = r16 >> 2, p4 = r16 & 3;
  int blk, bh;
  attn_block(xg, blk, bh);
  const int b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int k0 = blk * QB;
  const u16* base = qkv + (int64_t)b * T * ld;
  u16* dk_base = d_qkv + (int64_t)b * T * ld + (int64_t)H * DH + h * DH;
  u16* dv_base = d_qkv + (int64_t)b * T * ld + 2LL * H * DH + h * DH;

  if (k0 >= L) {
    for (int e = tid; e < QB * DH / 8; e += 256) {
      const int row = e / (DH / 8), col = (e % (DH / 8)) * 8, k = k0 + row;
      if (k < T) {
        *reinterpret_cast<uint4*>(dk_base + (int64_t)k * ld + col) = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(dv_base + (int64_t)k * ld + col) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    return;
  }
  const auto q_rs = buf_rsrc(base + h * DH, (int64_t)T * ld * 2);
  const auto d_rs = buf_rsrc(d_o + (int64_t)b * T * ldo + h * DH, (int64_t)T * ldo * 2);
  const auto l_rs = buf_rsrc(lse + (int64_t)bh * T, (int64_t)T * 4);
  const auto e_rs = buf_rsrc(delta + (int64_t)bh * T, (int64_t)T * 4);
  TileDma<NW> dq_dma, do_dma;
  dq_dma.init(ld, wave, lane);
  do_dma.init(ldo, wave, lane);
  ImgRd rd;
  rd.init(g, r16, q4, p4);
  const int nqt = (L + QB - 1) / QB;
  auto issue = [&](int qt, int slot) {
    u16* Qs = smem + slot * SLOT_E;
    dq_dma.issue(q_rs, Qs, qt * QB, T, ld, wave);
    do_dma.issue(d_rs, Qs + IMG, qt * QB, T, ldo, wave);
    // wave 0: the tile's lse, wave 1: its delta (queries past T read as 0)
    if (wave < 2)
      glds4_buf(wave == 0 ? l_rs : e_rs, Qs + 2 * IMG + wave * 2 * QB,
                lane < T - qt * QB ? (uint32_t)(lane * 4) : kOOB, (uint32_t)(qt * QB * 4));
  };

  const int key = k0 + wave * 16 + r16;
  const int kc = min(key, T - 1);
  bf16x8 kf[4], vf[4];
  load_frag(kf, base + (int64_t)kc * ld + (int64_t)H * DH + h * DH, g);
  load_frag(vf, base + (int64_t)kc * ld + 2LL * H * DH + h * DH, g);
  const bool kvalid = key < L;

  f32x4 dk[8], dv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float c2 = scale * 1.4426950408889634f;
  auto body = [&](auto mask_c, int qt, int slot) {
    constexpr bool MASK = decltype(mask_c)::value;
    const u16* Qs = smem + slot * SLOT_E;
    const u16* Ds = Qs + IMG;
    const float* lse_s = reinterpret_cast<const float*>(Qs + 2 * IMG);
    const float* del_s = lse_s + QB;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 pp[2], dsv[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int qs = 2 * c + half;
        const f32x4 s = chain4_img(rd, Qs, 16 * qs, kf);
        const f32x4 dp = chain4_img(rd, Ds, 16 * qs, vf);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * qs + 4 * g + r;
          float pv = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lse_s[ql] * 1.4426950408889634f));
          if (MASK && qt * QB + ql >= L) pv = 0.f;
          pp[half][r] = pv;
          dsv[half][r] = pv * (dp[r] - del_s[ql]);
        }
      }
      const bf16x8 wp = pack8(pp[0], pp[1]), wd = pack8(dsv[0], dsv[1]);
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) dv[ds] = MFMA_BF16(rd.tr(Ds, 32 * c, ds), wp, dv[ds]);
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) dk[ds] = MFMA_BF16(rd.tr(Qs, 32 * c, ds), wd, dk[ds]);
    }
  };
  // with 2 slots every wait drains the wave's DMA (vmcnt(0)): the per-wave count may differ
  tile_loop<STAGES, 1>(nqt, issue, [&](int qt, int slot) { body(std::false_type{}, qt, slot); },
      [&](int qt, int slot) { body(std::true_type{}, qt, slot); });
  if (!kvalid) {  // padded keys: zero gradients (their p were not masked per score)
#pragma unroll
    for (int i = 0; i < 8; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (key < T) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      store8x2_bf16(dk_base + (int64_t)key * ld + 32 * d, dk[2 * d] * scale, dk[2 * d + 1] * scale, g);
      store8x2_bf16(dv_base + (int64_t)key * ld + 32 * d, dv[2 * d], dv[2 * d + 1], g);
    }
  }
}

// NW waves per workgroup (32 NW query / key rows): 4 from T = 256 on, 2 below (the encoder's
// T = 128 keeps two workgroups per (utterance, head))
int attn_fwd_bf16_launch(const void* qkv, void* o, float* lse, const int64_t* lens, int64_t batch,
                         int64_t seq_len, int heads, float scale, hipStream_t st) {
  const int dma = g_tune[FS2_TUNE_ATTN_DMA];
  if (seq_len >= 256 && g_tune[FS2_TUNE_ATTN] >= 0 && dma >= 0) {
    dim3 grid((unsigned)((seq_len + 127) / 128), (unsigned)(batch * heads));
    const int xg = g_tune[FS2_TUNE_ATTN_XCD] >= 0 && (batch * heads) % 8 == 0;
    if (dma == 1)
      attn_fwd_dma<3><<<grid, 256, 0, st>>>((const u16*)qkv, (u16*)o, lse, lens, (int)seq_len, heads, scale, xg);
    else
      attn_fwd_dma<2><<<grid, 256, 0, st>>>((const u16*)qkv, (u16*)o, lse, lens, (int)seq_len, heads, scale, xg);
  } else if (seq_len >= 256 && g_tune[FS2_TUNE_ATTN] >= 0) {
    dim3 grid((unsigned)((seq_len + 127) / 128), (unsigned)(batch * heads));
    attn_fwd_bf16<4><<<grid, 256, 0, st>>>((const u16*)qkv, (u16*)o, lse, lens, (int)seq_len, heads, scale);
  } else {
    dim3 grid((unsigned)((seq_len + QB - 1) / QB), (unsigned)(batch * heads));
    attn_fwd_bf16_g1<<<grid, 256, 0, st>>>((const u16*)qkv, (u16*)o, lse, lens, (int)seq_len, heads, scale);
  }
  return launch_status("fs2_attn_fwd(bf16)");
}

int attn_bwd_bf16_launch(const void* qkv, const void* o, const void* d_o, const float* lse,
                         void* d_qkv, const int64_t* lens, int64_t batch, int64_t seq_len,
                         int heads, float scale, float* ws, hipStream_t st) {
  const int tune = g_tune[FS2_TUNE_ATTN];
  dim3 grid1((unsigned)((seq_len + QB - 1) / QB), (unsigned)(batch * heads));
  dim3 grid2((unsigned)((seq_len + 127) / 128), (unsigned)(batch * heads));
  const bool dma = seq_len >= 256 && g_tune[FS2_TUNE_ATTN_DMA] >= 0 && (tune == 0 || tune == 1);
  const int xg = g_tune[FS2_TUNE_ATTN_XCD] >= 0 && (batch * heads) % 8 == 0;
  if (dma) {  // dQ with delta fused, LDS-DMA staged
    attn_bwd_dq_dma<<<grid2, 256, 0, st>>>((const u16*)qkv, (const u16*)o, (const u16*)d_o, lse, ws,
                                           (u16*)d_qkv, lens, (int)seq_len, heads, scale, xg);
  } else if (seq_len >= 256 && tune >= 0) {  // dQ with delta fused
    attn_bwd_dq_bf16<4><<<grid2, 256, 0, st>>>((const u16*)qkv, (const u16*)o, (const u16*)d_o, lse, ws,
                                               (u16*)d_qkv, lens, (int)seq_len, heads, scale);
  } else {
    const int64_t rows = batch * seq_len;
    attn_bwd_delta_bf16_g1<<<(unsigned)((rows * heads * 64 + 255) / 256), 256, 0, st>>>(
        (const u16*)o, (const u16*)d_o, ws, rows, (int)seq_len, heads);
    attn_bwd_dq_bf16_g1<<<grid1, 256, 0, st>>>((const u16*)qkv, (const u16*)d_o, lse, ws, (u16*)d_qkv,
                                               lens, (int)seq_len, heads, scale);
  }
  // dK/dV: one 16-key group per wave at two workgroups per CU (221 VGPRs) by default --
  // decoder backward 99 -> 87 us against the two-group kernel, whose 415 registers allow one
  // workgroup per CU (384 workgroups = 1.5 rounds of the CUs)
  if (dma && tune == 0)
    attn_bwd_dkdv_dma<<<grid1, 256, 0, st>>>((const u16*)qkv, (const u16*)d_o, lse, ws, (u16*)d_qkv,
                                             lens, (int)seq_len, heads, scale, xg);
  else if (seq_len >= 256 && tune == 2)
    attn_bwd_dkdv_bf16<4><<<grid2, 256, 0, st>>>((const u16*)qkv, (const u16*)d_o, lse, ws, (u16*)d_qkv,
                                                 lens, (int)seq_len, heads, scale);
  else if (tune == 3)
    attn_bwd_dkdv_bf16_g1<3><<<grid1, 256, 0, st>>>((const u16*)qkv, (const u16*)d_o, lse, ws,
                                                    (u16*)d_qkv, lens, (int)seq_len, heads, scale);
  else if (tune == -1 || tune == 1)
    attn_bwd_dkdv_bf16_g1<1><<<grid1, 256, 0, st>>>((const u16*)qkv, (const u16*)d_o, lse, ws,
                                                    (u16*)d_qkv, lens, (int)seq_len, heads, scale);
  else
    attn_bwd_dkdv_bf16_g1<2><<<grid1, 256, 0, st>>>((const u16*)qkv, (const u16*)d_o, lse, ws,
                                                    (u16*)d_qkv, lens, (int)seq_len, heads, scale);
  return launch_status("fs2_attn_bwd(bf16)");
}

}  // namespace fs2
