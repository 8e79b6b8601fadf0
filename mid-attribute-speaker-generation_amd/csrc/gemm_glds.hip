// bf16 implicit-GEMM Conv1d / Linear, forward and dX ("NT"), staged by LDS-DMA.
//
//   y[r, o] = epilogue( sum_{j,c} wk[o, j*Cin + c] * x[r + j - pad, c] )
//
// Tile BM x BN x 64, 4 waves (2 x 2), v_mfma_f32_16x16x32_bf16.  Both operand tiles are
// filled with global_load_lds_dwordx4: one wave-instruction writes 1 KiB = 8 rows x 128 B of
// a lane-linear [rows][64] bf16 image.  The image is XOR-swizzled on the SOURCE address
// (16-B chunk c of row R lands at chunk c ^ ((R >> 1) & 7)), so the ds_read_b128 fragment
// reads of 16 consecutive rows hit 16 distinct 16-B bank slots.  The conv tap shift lives in
// the per-lane source address: rows outside their utterance (and rows/channels past the
// matrix edge) read a 16-B zero line instead, so padding costs no branches in the loop.
// Row-dependent address parts (utterance start, frame index) are computed once per block;
// per k-tile only the tap index and channel offset change (scalar when Cin % 64 == 0).
//
// STAGES = 1: load; vmcnt(0); barrier; MFMA; barrier (occupancy 3-4 blocks/CU hides the
//             load phase of one block under the MFMA phase of the others).
// STAGES = 2: the next tile's DMA is issued before the current tile's MFMAs and stays in
//             flight across the barrier (counted vmcnt, raw s_barrier).
//
// Blocks are renumbered XCD-aware (bijective remap): each XCD runs a contiguous range of
// (m, n) tiles, n fastest, so an A row band is fetched from HBM once per XCD L2.
//
// Epilogue: accumulators go through LDS (fp32, 132-float rows, conflict-free writes) and
// leave as 8-element row vectors: bias, residual/aux add, ReLU, ReLU-mask and the bf16 cast
// are applied on 16-B (bf16) / 32-B (fp32) coalesced stores.
#include <mutex>
#include <type_traits>

#include "common.hpp"

namespace fs2 {

typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));
typedef unsigned short u16;

__device__ __attribute__((aligned(128))) uint4 g_zero_line[8];  // zero source for OOB chunks

struct GldsArgs {
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
  int tiles_m, tiles_n;
  int vec;    // 8-wide epilogue legal (N, ldy, ld_aux multiples of 8; aligned pointers)
  int group;  // n-tiles per tile group (see the block order below)
  const int64_t* lens;  // optional utterance lengths: all-padding row tiles are not computed
  int dil;              // tap dilation (vocoder convs; 1 elsewhere)
  float alpha, scale;   // FS2_EPI_LRELU slope, FS2_EPI_ACC_Y scale
  u16* y2;              // FS2_EPI_Y2 bf16 output (ld = N)
  float alpha2;
  int kz;               // halo kernel: channel-block splits (0/1 = none; see halo_splitk_reduce)
  float* slab;          // kz > 1: [kz][M][N] fp32 partial products
  // LayerNorm epilogue (fs2_conv_gemm_ln; 256-wide tiles hold whole rows): ln_out != NULL
  const float* ln_res;
  const float* ln_gamma;
  const float* ln_beta;
  float* ln_out;
  u16* ln_out_t;
  float* ln_xhat;
  float* ln_rstd;
  const uint64_t* ln_seed;
  uint64_t ln_site;
  float ln_p;
  // LayerNorm-backward epilogue (fs2_conv_gemm_ln_bwd, ln_mode 1): ln_out = dres, ln_out_t =
  // the bf16 dy copy, ln_xhat / ln_rstd read; column partials into ln_part ([4][ln_nblk][256])
  int ln_mode;
  int ln_dres_add;
  float* ln_part;
  int64_t ln_nblk;
};

// Are rows [r0, r1) all padding (t >= lens[b] for r = b*T + t)?  Scalar, block-uniform.
FS2_DEV bool rows_all_padding(const int64_t* lens, int64_t T, int64_t r0, int64_t r1) {
  int64_t s = r0 / T;
  if (r0 - s * T < lens[s]) return false;
  for (++s; s * T < r1; ++s)
    if (lens[s] > 0) return false;
  return true;
}

// With lens (all-padding row tiles skipped) the XCD-contiguous tile order would give each XCD
// a contiguous run of utterances, and the XCD holding the longest ones would set the launch
// time.  m-tiles are therefore visited in a stride permutation (tm' -> tm' * s mod tiles_m,
// s ~ tiles_m / 8 coprime with tiles_m): each XCD's contiguous run of tm' lands on m-tiles
// spread over the whole batch.  Every n-tile of an m-tile stays on one XCD (A-row reuse).
FS2_DEV int igcd(int a, int b) {
  while (b) {
    const int t = a % b;
    a = b;
    b = t;
  }
  return a;
}

FS2_DEV int m_interleave(int tm, int tiles_m, bool on) {
  if (!on || tiles_m < 16) return tm;
  int s = tiles_m / 8 + 1;
  while (igcd(s, tiles_m) != 1) ++s;
  return (int)(((int64_t)tm * s) % tiles_m);
}

FS2_DEV void glds16(const void* src, u16* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(
      (const __attribute__((address_space(1))) void*)src,
      (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

FS2_DEV float bfv(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
FS2_DEV u16 fbv(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<u16*>(&b);
}

// s_waitcnt lgkmcnt(0) with vmcnt / expcnt left at their maxima (gfx9 simm16 encoding), for
// __builtin_amdgcn_s_waitcnt: unlike inline asm, the compiler's wait-count pass sees it.
constexpr int kLgkm0 = 0xC07F;

// Wait until at most n (0..8, wave-uniform) vector-memory instructions are in flight.
FS2_DEV void vm_wait_n(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

// The k-loop.  STAGES == 1: load; vmcnt(0); barrier; MFMA; barrier.  STAGES >= 2: a ring of
// LDS stages with STAGES-1 tiles issued ahead; per tile: counted vmcnt (the tile landed, later
// ones may stay in flight), ONE raw barrier (the tile is visible to every wave AND every wave
// has finished the previous tile, whose slot the refill below overwrites), refill, MFMA.
template <int STAGES, int PER, typename Issue, typename Compute>
FS2_DEV void kloop(int nk, Issue&& issue, Compute&& compute) {
  if constexpr (STAGES == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      issue(kt, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      compute(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    for (int t = 0; t < STAGES - 1 && t < nk; ++t) issue(t, t);
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = nk - 1 - kt < STAGES - 2 ? nk - 1 - kt : STAGES - 2;
      vm_wait_tiles<PER>(ahead);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
      compute(kt % STAGES);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

// Workgroup barrier of the epilogues: LDS writes retired (lgkmcnt(0)), then a raw s_barrier.
// __syncthreads() would also wait vmcnt(0); at the end of the kernels no DMA is in flight and
// the two are the same.  (The epilogues share no global memory between threads.)
FS2_DEV void epi_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// LayerNorm epilogue of a 256-wide tile (whole rows): the fs2_ln_fwd row computation on the
// accumulators instead of a stored fp32 y -- z = dropout(acc + bias, p) + res, mean / variance
// over the half-wave's 256 channels (8 per lane, the fs2_ln_fwd lane layout), out = xhat *
// gamma + beta, padded rows written as 0 (xhat / rstd not written there: the backward skips
// them).  Same operations in the same order as fs2_conv_gemm + fs2_ln_fwd: bitwise equal.
template <int BM, int NWAVE, int WN>
FS2_DEV void nt_epilogue_ln(const GldsArgs& a, f32x4 (&acc)[BM / 32][256 / WN / 16], u16* smem,
                            int64_t m0, bool skip, int tid, int wm, int wn, int g, int r16) {
  constexpr int MI = BM / 32, NI = 256 / WN / 16, EPI_LD = 256 + 4;
  constexpr int RPP = NWAVE * 2;  // rows per pass: one per half-wave
  float* Cs = reinterpret_cast<float*>(smem);
  const int hl = tid & 31;
  const uint64_t seed = a.ln_seed ? *a.ln_seed : 0ull;
  const f32x4 ga0 = ld4(a.ln_gamma + 8 * hl), ga1 = ld4(a.ln_gamma + 8 * hl + 4);
  const f32x4 be0 = ld4(a.ln_beta + 8 * hl), be1 = ld4(a.ln_beta + 8 * hl + 4);
  f32x4 bi0 = f32x4{0.f, 0.f, 0.f, 0.f}, bi1 = bi0;
  if ((a.flags & FS2_EPI_BIAS) && !skip) {
    bi0 = ld4(a.bias + 8 * hl);
    bi1 = ld4(a.bias + 8 * hl + 4);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(i * 16 + 4 * g + r) * EPI_LD + wn * (256 / WN) + j * 16 + r16] = acc[i][j][r];
    }
    epi_barrier();
#pragma unroll
    for (int p = 0; p < (BM / 2) / RPP; ++p) {
      const int rr = p * RPP + (tid >> 5);
      const int64_t m = m0 + h * (BM / 2) + rr;
      if (m >= a.M) continue;  // half-wave uniform
      const int64_t e0 = m * 256 + 8 * hl;
      const bool pad = a.lens && (m % a.T) >= a.lens[m / a.T];
      if (pad) {
        const f32x4 zz = {0.f, 0.f, 0.f, 0.f};
        st4(a.ln_out + e0, zz);
        st4(a.ln_out + e0 + 4, zz);
        if (a.ln_out_t) st8_bf16(a.ln_out_t + e0, zz, zz);
        continue;
      }
      f32x4 z0 = *reinterpret_cast<const f32x4*>(Cs + rr * EPI_LD + 8 * hl);
      f32x4 z1 = *reinterpret_cast<const f32x4*>(Cs + rr * EPI_LD + 8 * hl + 4);
      z0 += bi0;
      z1 += bi1;
      if (a.ln_p > 0.f) {
        f32x4 k0, k1;
        dropout8(seed, a.ln_site, (uint64_t)e0, a.ln_p, k0, k1);
        z0 *= k0;
        z1 *= k1;
      }
      if (a.ln_res) {
        z0 += ld4(a.ln_res + e0);
        z1 += ld4(a.ln_res + e0 + 4);
      }
      const float mean =
          half_sum((z0.x + z0.y + z0.z + z0.w) + (z1.x + z1.y + z1.z + z1.w)) * (1.f / 256);
      const f32x4 c0 = z0 - mean, c1 = z1 - mean;
      const float var = half_sum((c0.x * c0.x + c0.y * c0.y + c0.z * c0.z + c0.w * c0.w) +
                                 (c1.x * c1.x + c1.y * c1.y + c1.z * c1.z + c1.w * c1.w)) *
                        (1.f / 256);
      const float rs = 1.f / sqrtf(var + 1e-5f);
      const f32x4 xh0 = c0 * rs, xh1 = c1 * rs;
      const f32x4 u0 = xh0 * ga0 + be0, u1 = xh1 * ga1 + be1;
      st4(a.ln_out + e0, u0);
      st4(a.ln_out + e0 + 4, u1);
      if (a.ln_out_t) st8_bf16(a.ln_out_t + e0, u0, u1);
      st4(a.ln_xhat + e0, xh0);
      st4(a.ln_xhat + e0 + 4, xh1);
      if (hl == 0) a.ln_rstd[m] = rs;
    }
    epi_barrier();
  }
}

// LayerNorm-BACKWARD epilogue of a 256-wide tile: the GEMM's rows are the upstream gradient of
// a LayerNorm (dout = acc + aux, the residual-gradient add of fs2_conv_gemm's FS2_EPI_ADD_AUX),
// and fs2_ln_bwd's row computation runs on them: dz = rstd (g dout - mean(g dout) - xhat
// mean(g dout xhat)) into dres (written, or added with dres_add), dy = dz * dropout_in into the
// bf16 copy, padded rows zero.  Each 32-row half of the tile is one fs2_ln_bwd block: its
// column partials of dout xhat, dout and dy (dgamma, dbeta, the fused bias gradient) are summed
// over the 8 half-waves in a fixed order into ln_part, reduced by fs2_ln_bwd_final.
template <int BM, int NWAVE, int WN>
FS2_DEV void nt_epilogue_lnbwd(const GldsArgs& a, f32x4 (&acc)[BM / 32][256 / WN / 16], u16* smem,
                               int64_t m0, int tid, int wm, int wn, int g, int r16) {
  static_assert(BM / 2 == 32 && NWAVE == 4, "one 32-row LayerNorm block per tile half");
  constexpr int MI = BM / 32, NI = 256 / WN / 16, EPI_LD = 256 + 4;
  float* Cs = reinterpret_cast<float*>(smem);
  f32x4* red = reinterpret_cast<f32x4*>(Cs + 32 * EPI_LD);  // [3 kinds][8 half-waves][64]
  const int hl = tid & 31, hw = tid >> 5;
  const bool use_aux = a.flags & FS2_EPI_ADD_AUX;
  const uint64_t seed = a.ln_seed ? *a.ln_seed : 0ull;
  const f32x4 gam0 = ld4(a.ln_gamma + 8 * hl), gam1 = ld4(a.ln_gamma + 8 * hl + 4);
  const f32x4 zz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(i * 16 + 4 * g + r) * EPI_LD + wn * (256 / WN) + j * 16 + r16] = acc[i][j][r];
    }
    epi_barrier();
    f32x4 pg0 = zz, pg1 = zz, pb0 = zz, pb1 = zz, py0 = zz, py1 = zz;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int rr = hw + 8 * p;
      const int64_t m = m0 + h * 32 + rr;
      if (m >= a.M) continue;  // half-wave uniform
      const int64_t e0 = m * 256 + 8 * hl;
      const bool pad = a.lens && (m % a.T) >= a.lens[m / a.T];
      if (pad) {  // masked row: zero upstream gradient
        if (!a.ln_dres_add) {
          st4(a.ln_out + e0, zz);
          st4(a.ln_out + e0 + 4, zz);
        }
        if (a.ln_out_t) st8_bf16(a.ln_out_t + e0, zz, zz);
        continue;
      }
      f32x4 du0 = *reinterpret_cast<const f32x4*>(Cs + rr * EPI_LD + 8 * hl);
      f32x4 du1 = *reinterpret_cast<const f32x4*>(Cs + rr * EPI_LD + 8 * hl + 4);
      if (use_aux) {
        const float* ap = (const float*)a.aux + m * a.ld_aux + 8 * hl;
        du0 += ld4(ap);
        du1 += ld4(ap + 4);
      }
      const f32x4 xh0 = ld4(a.ln_xhat + e0), xh1 = ld4(a.ln_xhat + e0 + 4);
      pg0 += du0 * xh0;
      pg1 += du1 * xh1;
      pb0 += du0;
      pb1 += du1;
      const f32x4 dxh0 = du0 * gam0, dxh1 = du1 * gam1;
      const float m1 = half_sum((dxh0.x + dxh0.y + dxh0.z + dxh0.w) + (dxh1.x + dxh1.y + dxh1.z + dxh1.w)) *
                       (1.f / 256);
      const float m2 = half_sum((dxh0.x * xh0.x + dxh0.y * xh0.y + dxh0.z * xh0.z + dxh0.w * xh0.w) +
                                (dxh1.x * xh1.x + dxh1.y * xh1.y + dxh1.z * xh1.z + dxh1.w * xh1.w)) *
                       (1.f / 256);
      const float rs = a.ln_rstd[m];
      const f32x4 dz0 = rs * (dxh0 - m1 - xh0 * m2), dz1 = rs * (dxh1 - m1 - xh1 * m2);
      st4(a.ln_out + e0, a.ln_dres_add ? ld4(a.ln_out + e0) + dz0 : dz0);
      st4(a.ln_out + e0 + 4, a.ln_dres_add ? ld4(a.ln_out + e0 + 4) + dz1 : dz1);
      f32x4 dy0 = dz0, dy1 = dz1;
      if (a.ln_p > 0.f) {
        f32x4 mi0, mi1;
        dropout8(seed, a.ln_site, (uint64_t)e0, a.ln_p, mi0, mi1);
        dy0 *= mi0;
        dy1 *= mi1;
      }
      if (a.ln_out_t) st8_bf16(a.ln_out_t + e0, dy0, dy1);
      py0 += dy0;
      py1 += dy1;
    }
    const int64_t blk = (m0 + h * 32) / 32;
    const bool live = m0 + h * 32 < a.M;  // block-uniform
    red[(0 * 8 + hw) * 64 + 2 * hl] = pg0;
    red[(0 * 8 + hw) * 64 + 2 * hl + 1] = pg1;
    red[(1 * 8 + hw) * 64 + 2 * hl] = pb0;
    red[(1 * 8 + hw) * 64 + 2 * hl + 1] = pb1;
    red[(2 * 8 + hw) * 64 + 2 * hl] = py0;
    red[(2 * 8 + hw) * 64 + 2 * hl + 1] = py1;
    epi_barrier();
    if (live && tid < 3 * 64) {  // waves 0-2: one kind each, the 8 half-waves in order
      const int kind = tid >> 6, q = tid & 63;
      f32x4 s = red[(kind * 8) * 64 + q];
#pragma unroll
      for (int k = 1; k < 8; ++k) s += red[(kind * 8 + k) * 64 + q];
      const int slot = kind == 2 ? 3 : kind;  // fs2_ln_bwd's part layout: dgamma, dbeta, -, dbias
      st4(a.ln_part + ((int64_t)slot * a.ln_nblk + blk) * 256 + 4 * q, s);
    }
    epi_barrier();
  }
}

// Epilogue through LDS, one half of the tile's rows at a time: bias, aux add, ReLU / ReLU-mask,
// bf16 cast on 8-element row vectors (16-B / 32-B coalesced stores).  Shared by the NT kernels.
// WM waves per column of the tile (each BM / WM rows, MI = BM / WM / 16 fragments; WM / 2 per
// half).  SROW > 0 (conv_gemm_tapreg): fragment i of a wave holds the rows i + SROW * m
// (m = 0..15) of its band; the fragments are staged as usual and the store pass maps each
// output row back to its (fragment, m) slot.
template <int BM, int BN, bool VOC, int NWAVE = 4, int WN = 2, int WM = 2, int SROW = 0,
          bool BF16D = false>
FS2_DEV void nt_epilogue(const GldsArgs& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], u16* smem,
                         int64_t m0, int n0, bool skip, int tid, int wm, int wn, int g, int r16) {
  constexpr int MI = BM / WM / 16, NI = BN / WN / 16;
  constexpr int WR = BM / WM, WPH = WM / 2;  // rows per wave, waves per half
  static_assert(WM % 2 == 0 && (SROW == 0 || MI % SROW == 0), "epilogue layout");
  constexpr int EPI_LD = BN + 4;
  if constexpr (BN == 256 && !VOC && WM == 2 && SROW == 0) {
    if (a.ln_out) {
      if constexpr (BM == 64) {
        if (a.ln_mode == 1) {
          nt_epilogue_lnbwd<BM, NWAVE, WN>(a, acc, smem, m0, tid, wm, wn, g, r16);
          return;
        }
      }
      nt_epilogue_ln<BM, NWAVE, WN>(a, acc, smem, m0, skip, tid, wm, wn, g, r16);
      return;
    }
  }
  if (skip && (a.flags & FS2_EPI_SKIP_NOSTORE)) return;  // block-uniform
  if constexpr (BF16D && !VOC) {
    // bf16 output with a column-only epilogue (bias, ReLU): applied in the accumulator layout
    // (the bias of a lane's column is one value per 16-column fragment), rounded to bf16 and
    // written to LDS as ONE whole tile -- half the LDS bytes of the fp32 half-tile passes and a
    // single barrier -- then stored as 16-B row vectors.  Same operations per element: bitwise
    // equal to the fp32 path below.
    constexpr int LDB = BN + 4;  // u16 row stride: 8 B pad
    static_assert(BM * LDB <= (BM / 2) * (BN + 4) * 2, "bf16 tile fits the epilogue region");
    const bool rmask = (a.flags & FS2_EPI_RELU_MASK_AUX) && (a.flags & FS2_EPI_AUX_BF16);
    if (a.vec && (a.flags & FS2_EPI_OUT_BF16) && !(a.flags & FS2_EPI_ADD_AUX) &&
        (rmask || !(a.flags & FS2_EPI_RELU_MASK_AUX))) {
      constexpr int TPR = BN / 8, RPP = NWAVE * 64 / TPR, NPB = BM / RPP, NPF = NPB / 2;
      const int cc = (tid % TPR) * 8;
      const int n = n0 + cc;
      // ReLU mask (bf16 aux > 0): applied to the bf16 row vectors -- rounding 0 gives 0, so the
      // mask commutes with the rounding.  The first half of the passes' aux rows is loaded
      // before the LDS write, the second half one pass ahead of its use.
      uint4 am[NPB];
      if (rmask) {
#pragma unroll
        for (int p = 0; p < NPF; ++p) {
          const int64_t m = m0 + p * RPP + tid / TPR;
          am[p] = m < a.M && n < a.N ? *reinterpret_cast<const uint4*>((const u16*)a.aux + m * a.ld_aux + n)
                                      : uint4{0u, 0u, 0u, 0u};
        }
      }
      const bool relu = a.flags & FS2_EPI_RELU;
      const bool bias = (a.flags & FS2_EPI_BIAS) && !skip;
      float bj[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wn * (BN / WN) + j * 16 + r16;
        bj[j] = bias && col < a.N ? a.bias[col] : 0.f;
      }
      u16* Cb = smem;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[i][j][r];
            if (bias) v += bj[j];
            if (relu) v = fmaxf(v, 0.f);
            // output row of accumulator (i, 4g + r): SROW > 0 (conv_gemm_tapreg) holds rows
            // i % SROW + SROW * m of the wave's band i / SROW (see below)
            const int row = SROW > 0 ? wm * WR + (i / (SROW > 0 ? SROW : 1)) * 16 * SROW +
                                           i % (SROW > 0 ? SROW : 1) + SROW * (4 * g + r)
                                     : wm * WR + i * 16 + 4 * g + r;
            Cb[row * LDB + wn * (BN / WN) + j * 16 + r16] = fbv(v);
          }
      epi_barrier();
#pragma unroll
      for (int p = 0; p < NPB; ++p) {
        if (rmask && p + NPF < NPB) {
          const int64_t m = m0 + (p + NPF) * RPP + tid / TPR;
          am[p + NPF] = m < a.M && n < a.N
                            ? *reinterpret_cast<const uint4*>((const u16*)a.aux + m * a.ld_aux + n)
                            : uint4{0u, 0u, 0u, 0u};
        }
        const int rr = p * RPP + tid / TPR;
        const int64_t m = m0 + rr;
        if (m >= a.M || n >= a.N) continue;
        uint4 o = *reinterpret_cast<const uint4*>(Cb + rr * LDB + cc);
        if (rmask) {  // keep each bf16 half where its aux half is > 0: sign clear, 0 < |x| <= inf
          auto pos = [](uint32_t h) { return (h & 0x8000u) == 0 && (h & 0x7fffu) != 0 && (h & 0x7fffu) <= 0x7f80u; };
          auto keep = [&](uint32_t y, uint32_t x) {
            return y & ((pos(x & 0xffffu) ? 0x0000ffffu : 0u) | (pos(x >> 16) ? 0xffff0000u : 0u));
          };
          o.x = keep(o.x, am[p].x);
          o.y = keep(o.y, am[p].y);
          o.z = keep(o.z, am[p].z);
          o.w = keep(o.w, am[p].w);
        }
        *reinterpret_cast<uint4*>((u16*)a.y + m * a.ldy + n) = o;
      }
      epi_barrier();
      return;
    }
  }
  float* Cs = reinterpret_cast<float*>(smem);
  const bool out_bf16 = a.flags & FS2_EPI_OUT_BF16, aux_bf16 = a.flags & FS2_EPI_AUX_BF16;
  constexpr int TPR = BN / 8;            // threads per row
  constexpr int RPP = NWAVE * 64 / TPR;  // rows per pass
  constexpr int NP = (BM / 2) / RPP;     // passes per half
  const int cc = (tid % TPR) * 8;
  const int n = n0 + cc;
  // The bias (the same 8 columns in every pass) and a half's aux rows are loaded BEFORE the
  // half's LDS write: their latency then overlaps it.  Loaded inside each pass, they put a
  // dependent global load between the pass's LDS read and its store, four passes in series
  // (k = 1 QKV projection: 28.5 us with, 15.1 us without the epilogue; its LDS transpose
  // alone costs 2.4 us and its stores alone 4.1 us; profiles/r4_ab_experiments.txt).
  // (fp32 aux rows only where a half has at most two passes: four would cost 32 registers)
  constexpr bool PF32 = NP <= 2;
  const bool pf = !VOC && a.vec && n < a.N;
  const bool pf_aux = pf && (a.flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX)) &&
                      (aux_bf16 || PF32);
  f32x4 bz0 = f32x4{0.f, 0.f, 0.f, 0.f}, bz1 = bz0;
  if (pf && (a.flags & FS2_EPI_BIAS) && !skip) {
    bz0 = *reinterpret_cast<const f32x4*>(a.bias + n);
    bz1 = *reinterpret_cast<const f32x4*>(a.bias + n + 4);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint4 araw[NP][PF32 ? 2 : 1];  // aux rows of this half: bf16 in [p][0], fp32 in [p][0..1]
    if (pf_aux) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int64_t m = m0 + h * (BM / 2) + p * RPP + tid / TPR;
#pragma unroll
        for (int q = 0; q < (PF32 ? 2 : 1); ++q) araw[p][q] = uint4{0u, 0u, 0u, 0u};
        if (m < a.M) {
          if (aux_bf16) {
            araw[p][0] = *reinterpret_cast<const uint4*>((const u16*)a.aux + m * a.ld_aux + n);
          } else if constexpr (PF32) {
            const uint4* ap = reinterpret_cast<const uint4*>((const float*)a.aux + m * a.ld_aux + n);
            araw[p][0] = ap[0];
            araw[p][1] = ap[1];
          }
        }
      }
    }
    if (wm / WPH == h) {
      const int rb = (wm % WPH) * WR;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(rb + i * 16 + 4 * g + r) * EPI_LD + wn * (BN / WN) + j * 16 + r16] = acc[i][j][r];
    }
    epi_barrier();
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int rr = p * RPP + tid / TPR;
      const int64_t m = m0 + h * (BM / 2) + rr;
      if (m >= a.M || n >= a.N) continue;
      int rq = rr;
      if constexpr (SROW > 0) {  // row b + i + SROW * q of a band of 16 * SROW rows
        const int w = rr / WR, rw = rr % WR, bnd = rw / (16 * SROW), rb2 = rw % (16 * SROW);
        rq = w * WR + (bnd * SROW + rb2 % SROW) * 16 + rb2 / SROW;
      }
      float v[8];
      const f32x4 lo = *reinterpret_cast<const f32x4*>(Cs + rq * EPI_LD + cc);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(Cs + rq * EPI_LD + cc + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = lo[e];
        v[e + 4] = hi[e];
      }
      if (a.vec) {
        if ((a.flags & FS2_EPI_BIAS) && !skip) {
          const f32x4 b0 = pf ? bz0 : *reinterpret_cast<const f32x4*>(a.bias + n);
          const f32x4 b1 = pf ? bz1 : *reinterpret_cast<const f32x4*>(a.bias + n + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] += b0[e];
            v[e + 4] += b1[e];
          }
        }
        float av[8];
        if (pf_aux) {
          if (aux_bf16) {
            const uint4 raw = araw[p][0];
            const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              av[2 * e] = __uint_as_float(wv[e] << 16);
              av[2 * e + 1] = __uint_as_float(wv[e] & 0xffff0000u);
            }
          } else if constexpr (PF32) {
            const uint4 r0 = araw[p][0], r1 = araw[p][1];
            av[0] = __uint_as_float(r0.x); av[1] = __uint_as_float(r0.y);
            av[2] = __uint_as_float(r0.z); av[3] = __uint_as_float(r0.w);
            av[4] = __uint_as_float(r1.x); av[5] = __uint_as_float(r1.y);
            av[6] = __uint_as_float(r1.z); av[7] = __uint_as_float(r1.w);
          }
        } else if (a.flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX)) {
          if (aux_bf16) {
            const uint4 raw = *reinterpret_cast<const uint4*>((const u16*)a.aux + m * a.ld_aux + n);
            const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              av[2 * e] = __uint_as_float(wv[e] << 16);
              av[2 * e + 1] = __uint_as_float(wv[e] & 0xffff0000u);
            }
          } else {
            const float* ap = (const float*)a.aux + m * a.ld_aux + n;
            const f32x4 a0 = *reinterpret_cast<const f32x4*>(ap);
            const f32x4 a1 = *reinterpret_cast<const f32x4*>(ap + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              av[e] = a0[e];
              av[e + 4] = a1[e];
            }
          }
        }
        float yo[8];
        if (VOC && (a.flags & FS2_EPI_ACC_Y)) {
          if (out_bf16) {
            const uint4 raw = *reinterpret_cast<const uint4*>((const u16*)a.y + m * a.ldy + n);
            const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              yo[2 * e] = __uint_as_float(wv[e] << 16);
              yo[2 * e + 1] = __uint_as_float(wv[e] & 0xffff0000u);
            }
          } else {
            const float* yp = (const float*)a.y + m * a.ldy + n;
            const f32x4 y0 = *reinterpret_cast<const f32x4*>(yp);
            const f32x4 y1 = *reinterpret_cast<const f32x4*>(yp + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              yo[e] = y0[e];
              yo[e + 4] = y1[e];
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (a.flags & FS2_EPI_ADD_AUX) v[e] += av[e];
          if (VOC && (a.flags & FS2_EPI_ACC_Y)) v[e] = (v[e] + yo[e]) * a.scale;
          if (a.flags & FS2_EPI_RELU) v[e] = fmaxf(v[e], 0.f);
          if (VOC && (a.flags & FS2_EPI_LRELU)) v[e] = v[e] >= 0.f ? v[e] : a.alpha * v[e];
          if (a.flags & FS2_EPI_RELU_MASK_AUX) v[e] = av[e] > 0.f ? v[e] : 0.f;
        }
        if (VOC && (a.flags & FS2_EPI_Y2)) {
          float w2[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) w2[e] = v[e] >= 0.f ? v[e] : a.alpha2 * v[e];
          uint4 o;
          o.x = (uint32_t)fbv(w2[0]) | ((uint32_t)fbv(w2[1]) << 16);
          o.y = (uint32_t)fbv(w2[2]) | ((uint32_t)fbv(w2[3]) << 16);
          o.z = (uint32_t)fbv(w2[4]) | ((uint32_t)fbv(w2[5]) << 16);
          o.w = (uint32_t)fbv(w2[6]) | ((uint32_t)fbv(w2[7]) << 16);
          *reinterpret_cast<uint4*>(a.y2 + m * a.N + n) = o;
        }
        if (VOC && !a.y) continue;
        if (out_bf16) {
          uint4 o;
          o.x = (uint32_t)fbv(v[0]) | ((uint32_t)fbv(v[1]) << 16);
          o.y = (uint32_t)fbv(v[2]) | ((uint32_t)fbv(v[3]) << 16);
          o.z = (uint32_t)fbv(v[4]) | ((uint32_t)fbv(v[5]) << 16);
          o.w = (uint32_t)fbv(v[6]) | ((uint32_t)fbv(v[7]) << 16);
          *reinterpret_cast<uint4*>((u16*)a.y + m * a.ldy + n) = o;
        } else {
          float* yp = (float*)a.y + m * a.ldy + n;
          *reinterpret_cast<f32x4*>(yp) = f32x4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<f32x4*>(yp + 4) = f32x4{v[4], v[5], v[6], v[7]};
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (n + e >= a.N) break;
          float x = v[e];
          if ((a.flags & FS2_EPI_BIAS) && !skip) x += a.bias[n + e];
          float av = 0.f;
          if (a.flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX))
            av = aux_bf16 ? bfv(((const u16*)a.aux)[m * a.ld_aux + n + e])
                          : ((const float*)a.aux)[m * a.ld_aux + n + e];
          if (a.flags & FS2_EPI_ADD_AUX) x += av;
          if (VOC && (a.flags & FS2_EPI_ACC_Y))
            x = (x + (out_bf16 ? bfv(((const u16*)a.y)[m * a.ldy + n + e])
                               : ((const float*)a.y)[m * a.ldy + n + e])) * a.scale;
          if (a.flags & FS2_EPI_RELU) x = fmaxf(x, 0.f);
          if (VOC && (a.flags & FS2_EPI_LRELU)) x = x >= 0.f ? x : a.alpha * x;
          if (a.flags & FS2_EPI_RELU_MASK_AUX) x = av > 0.f ? x : 0.f;
          if (VOC && (a.flags & FS2_EPI_Y2)) a.y2[m * a.N + n + e] = fbv(x >= 0.f ? x : a.alpha2 * x);
          if (VOC && !a.y) continue;
          if (out_bf16) ((u16*)a.y)[m * a.ldy + n + e] = fbv(x);
          else ((float*)a.y)[m * a.ldy + n + e] = x;
        }
      }
    }
    epi_barrier();
  }
}

// K1: taps == 1 and K % 64 == 0 (the Linear / 1x1 projections) -- A and B stage through buffer
// descriptors based at the tile's first row: per-lane 32-bit offsets fixed over the k loop, the
// k-step in the scalar offset, rows past M / N out of the descriptors' range (zeros).
// (the K1 128 x 128 one-stage build, the projections' workhorse, is held to three blocks per CU)
template <int BM, int BN, int STAGES, bool TAPALIGNED, bool VOC, bool K1 = false>
__global__ __launch_bounds__(256, (K1 && BM == 128 && BN == 128 && STAGES == 1) ? 3 : 1) void
conv_gemm_nt_glds(GldsArgs a) {
  static_assert(!K1 || (TAPALIGNED && !VOC), "K1: taps == 1, K % 64 == 0, no vocoder epilogue");
  const int dil = VOC ? a.dil : 1;
  constexpr int BK = 64;
  constexpr int AW = BM / 32, BW = BN / 32;  // glds per wave per tile (8 rows each)
  constexpr int MI = BM / 32, NI = BN / 32;  // 16x16 fragments per wave (2x2 waves)
  constexpr int STAGE_E = (BM + BN) * BK;    // elements per stage
  constexpr int EPI_LD = BN + 4;             // fp32 epilogue row stride
  constexpr int EPI_E = (BM / 2) * EPI_LD * 2;
  constexpr int SMEM_E = STAGES * STAGE_E > EPI_E ? STAGES * STAGE_E : EPI_E;
  __shared__ __attribute__((aligned(1024))) u16 smem[SMEM_E];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;

  // XCD-aware bijective renumbering of the 1-D grid
  const int nwg = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  // tile order: groups of `group` n-tiles (a weight slice that stays L2-resident), m-tiles
  // within a group, n fastest -- each XCD's contiguous share streams its A rows once per group
  const int gfull = a.tiles_m * a.group;
  const int ng = wg / gfull, rem = wg - ng * gfull;
  const int gsz = a.tiles_n - ng * a.group < a.group ? a.tiles_n - ng * a.group : a.group;
  const int tm = m_interleave(rem / gsz, a.tiles_m, a.lens != nullptr);
  const int tn = ng * a.group + (rem - (rem / gsz) * gsz);
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const bool skip = a.lens && rows_all_padding(a.lens, a.T, m0, m0 + BM < a.M ? m0 + BM : a.M);

  // ---- per-lane source descriptors (fixed over the k loop)
  const int lrow = lane >> 3;  // row within the 8-row piece
  const u16* zero = reinterpret_cast<const u16*>(g_zero_line);
  int64_t a_base[AW];  // element offset of the row's utterance start (or -1: row invalid)
  int a_t[AW];         // frame index within the utterance
  int a_lc[AW];        // logical 16-B chunk this lane fetches
#pragma unroll
  for (int i = 0; i < AW; ++i) {
    const int R = (wave * AW + i) * 8 + lrow;
    const int64_t m = m0 + R;
    a_lc[i] = (lane & 7) ^ ((R >> 1) & 7);
    if (m < a.M) {
      const int64_t s = m / a.T;
      a_t[i] = (int)(m - s * a.T);
      a_base[i] = s * a.T;
    } else {
      a_t[i] = 0;
      a_base[i] = -1;
    }
  }
  const u16* b_src[BW];
  int b_lc[BW];
#pragma unroll
  for (int i = 0; i < BW; ++i) {
    const int R = (wave * BW + i) * 8 + lrow;
    const int n = n0 + R;
    b_lc[i] = (lane & 7) ^ ((R >> 1) & 7);
    b_src[i] = n < a.N ? a.w + (int64_t)n * a.K + b_lc[i] * 8 : nullptr;
  }

  const int nk = (a.K + BK - 1) / BK;
  // K1 staging: descriptors over the tile's BM rows of x / BN rows of w
  const auto x_rs = buf_rsrc(a.x + m0 * a.ldx, (a.M - m0 < BM ? a.M - m0 : BM) * a.ldx * 2);
  const auto w_rs = buf_rsrc(a.w + (int64_t)n0 * a.K, (int64_t)(a.N - n0 < BN ? a.N - n0 : BN) * a.K * 2);
  uint32_t a_vo[K1 ? AW : 1], b_vo[K1 ? BW : 1];
  if constexpr (K1) {
#pragma unroll
    for (int i = 0; i < AW; ++i)
      a_vo[i] = (uint32_t)((((wave * AW + i) * 8 + lrow) * a.ldx + a_lc[i] * 8) * 2);
#pragma unroll
    for (int i = 0; i < BW; ++i)
      b_vo[i] = (uint32_t)((((wave * BW + i) * 8 + lrow) * a.K + b_lc[i] * 8) * 2);
  }
  auto issue_k1 = [&](int kt, int stage) {
    u16* As = smem + stage * STAGE_E;
    u16* Bs = As + BM * BK;
    const uint32_t k0 = (uint32_t)(kt * BK * 2);
#pragma unroll
    for (int i = 0; i < AW; ++i) glds16_buf(x_rs, As + (wave * AW + i) * 8 * BK, a_vo[i], k0);
#pragma unroll
    for (int i = 0; i < BW; ++i) glds16_buf(w_rs, Bs + (wave * BW + i) * 8 * BK, b_vo[i], k0);
  };
  auto issue = [&](int kt, int stage) {
    u16* As = smem + stage * STAGE_E;
    u16* Bs = As + BM * BK;
    const int k0 = kt * BK;
    int j0 = 0, c0 = 0;
    if constexpr (TAPALIGNED) {
      j0 = k0 / a.Cin;
      c0 = k0 - j0 * a.Cin;
    }
#pragma unroll
    for (int i = 0; i < AW; ++i) {
      const u16* src = zero;
      int j = j0, c = c0 + a_lc[i] * 8;
      bool kok = true;
      if constexpr (!TAPALIGNED) {
        const int k = k0 + a_lc[i] * 8;
        kok = k < a.K;
        j = k / a.Cin;
        c = k - j * a.Cin;
      }
      const int tt = a_t[i] + j * dil - a.pad;
      if (kok && a_base[i] >= 0 && tt >= 0 && tt < a.T)
        src = a.x + (a_base[i] + tt) * a.ldx + c;
      glds16(src, As + (wave * AW + i) * 8 * BK);
    }
#pragma unroll
    for (int i = 0; i < BW; ++i) {
      const u16* src = zero;
      bool kok = true;
      if constexpr (!TAPALIGNED) kok = k0 + b_lc[i] * 8 < a.K;
      if (b_src[i] && kok) src = b_src[i] + k0;
      glds16(src, Bs + (wave * BW + i) * 8 * BK);
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment element offsets (swizzle depends only on r16 because row bases are 16-aligned)
  const int sw = (r16 >> 1) & 7;
  const int fo0 = r16 * BK + ((0 * 4 + g) ^ sw) * 8;
  const int fo1 = r16 * BK + ((1 * 4 + g) ^ sw) * 8;
  auto compute = [&](int stage) {
    const u16* As = smem + stage * STAGE_E + wm * (BM / 2) * BK;
    const u16* Bs = smem + stage * STAGE_E + BM * BK + wn * (BN / 2) * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int fo = ks ? fo1 : fo0;
      bf16x8g fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const bf16x8g*>(As + i * 16 * BK + fo);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const bf16x8g*>(Bs + j * 16 * BK + fo);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };

  if (!skip) {
    if constexpr (K1) kloop<STAGES, AW + BW>(nk, issue_k1, compute);
    else kloop<STAGES, AW + BW>(nk, issue, compute);
  }

  nt_epilogue<BM, BN, VOC, 4, 2, 2, 0, K1>(a, acc, smem, m0, n0, skip, tid, wm, wn, g, r16);
}

// ------------------------------------------------------------------------ halo variant
// Conv1d with taps > 1, Cin % 64 == 0 and T % BM == 0 (every row tile lies inside one
// utterance).  The reduction runs channel-block-major: for each 64-channel block the
// BM + taps - 1 input rows of the tile and its tap halo (zero outside the utterance) are
// staged in LDS ONCE, and tap j reads them at row offset j -- only the weight tile is
// re-staged per tap, through a 2-slot ring.  Against the tap-major kernel above this removes
// (taps-1)/taps of the A-operand LDS-DMA traffic: the k=9 FFN conv moves 18 KB instead of
// 32 KB per 64-deep step of a 128 x 128 tile.  LDS rows are swizzled chunk c -> c ^ (row & 7),
// which keeps the 16-row fragment reads conflict-free at every row offset.
template <int BM, int BN, int BST, int HX, bool VOC, int NWAVE = 4, bool PIPE = false>
__global__ __launch_bounds__(NWAVE * 64, NWAVE == 8 ? 1 : HX > 16 ? 2 : 3)
void conv_gemm_halo(GldsArgs a) {
  static_assert(BST == 2, "the 2-slot weight ring (1- and 3-slot rings measured slower, profiles/r2_ab_experiments.txt)");
  // NWAVE = 4: 2 x 2 waves; NWAVE = 8: 2 (rows) x 4 (columns) waves, one block per CU
  const int dil = VOC ? a.dil : 1;
  constexpr int BK = 64;
  constexpr int WN = NWAVE / 2;
  constexpr int MI = BM / 32, NI = BN / WN / 16;
  constexpr int HMAX = BM + HX;                     // halo rows allocated ((taps-1)*dil <= HX)
  constexpr int QMAX = (HMAX / 8 + NWAVE - 1) / NWAVE;  // 8-row halo pieces per wave
  constexpr int BW = BN / 8 / NWAVE;                // weight pieces per wave
  constexpr int A_E = HMAX * BK, B_E = BN * BK;
  // BST == 2: two halo slots -- channel block cb + 1's rows are staged while cb's taps run
  constexpr int NA = BST == 2 ? 2 : 1;
  constexpr int EPI_E = (BM / 2) * (BN + 4) * 2;
  constexpr int SMEM_E = NA * A_E + BST * B_E > EPI_E ? NA * A_E + BST * B_E : EPI_E;
  __shared__ __attribute__((aligned(1024))) u16 smem[SMEM_E];
  u16* As = smem;
  u16* Bs = smem + NA * A_E;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int g = lane >> 4, r16 = lane & 15;

  // kz > 1 (split-K over channel blocks): split z owns channel blocks [cb0, cb1) of every
  // tile; the splits are the outer index of the XCD-contiguous order
  const int kz = a.kz > 1 ? a.kz : 1;
  const int nwg = a.tiles_m * a.tiles_n, nall = nwg * kz;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nall >> 3, r8 = nall & 7;
  const int wga = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int z = wga / nwg, wg = wga - z * nwg;
  const int gfull = a.tiles_m * a.group;
  const int ng = wg / gfull, rem = wg - ng * gfull;
  const int gsz = a.tiles_n - ng * a.group < a.group ? a.tiles_n - ng * a.group : a.group;
  const int tm = m_interleave(rem / gsz, a.tiles_m, a.lens != nullptr);
  const int tn = ng * a.group + (rem - (rem / gsz) * gsz);
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const bool skip = a.lens && rows_all_padding(a.lens, a.T, m0, m0 + BM < a.M ? m0 + BM : a.M);
  // this wave's half of the tile (BM/2 rows) all padding: it stages its share of the tiles but
  // issues no MFMAs (those outputs are masked downstream; the 256-row forward tiles of the
  // decoder's k=9 conv hold ~13 % such rows)
  const int64_t hr0 = m0 + wm * (BM / 2), hr1 = hr0 + BM / 2 < a.M ? hr0 + BM / 2 : a.M;
  const bool half_pad = !VOC && (hr0 >= a.M || (a.lens && rows_all_padding(a.lens, a.T, hr0, hr1)));
  const int ncb_all = a.Cin / 64, cb0 = z * ncb_all / kz, cb1 = (z + 1) * ncb_all / kz;

  const int lrow = lane >> 3;
  const int HR = BM + (a.taps - 1) * dil, HP = (HR + 7) / 8;
  const int64_t u0 = (m0 / a.T) * a.T;
  // input rows past the utterance's length are zero in the FFT blocks (Layers.py:25,28) and in
  // the upstream gradients: read them from the zero line (no HBM traffic).  Vocoder lens are
  // row limits of another meaning: the whole padded utterance is staged there.
  const int64_t ulen = (!VOC && a.lens) ? (a.lens[m0 / a.T] < a.T ? a.lens[m0 / a.T] : a.T) : a.T;
  const int64_t u1 = u0 + ulen < a.M ? u0 + ulen : a.M;
  // this wave's 16-row fragments holding a row below the utterance's length (input rows past
  // it are staged as zeros; outputs past it are masked downstream of the FFT / variance-
  // predictor convs -- the only lens users of this kernel)
  int mi_act = MI;
  if (!VOC && a.lens) {
    const int64_t nv = u1 - (m0 + wm * (BM / 2));
    mi_act = nv <= 0 ? 0 : nv >= BM / 2 ? MI : (int)((nv + 15) / 16);
  }
  // halo piece p = wave + NWAVE q: rows h = 8 p + lrow, global row m0 - pad + h.  Buffer
  // descriptors based at the tile's first halo row / first weight row; a lane whose row lies
  // outside the utterance (or past N) carries an out-of-range offset and stages zeros.  The
  // channel block and tap advance in the scalar offset.
  const auto x_rs = buf_rsrc(a.x + (m0 - a.pad) * a.ldx + cb0 * BK, (int64_t)HMAX * a.ldx * 2);
  const auto w_rs = buf_rsrc(a.w + (int64_t)n0 * a.K + cb0 * BK, (int64_t)BN * a.K * 2);
  uint32_t h_vo[QMAX];
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int h = (wave + NWAVE * q) * 8 + lrow;
    const int64_t gr = m0 - a.pad + h;
    const int lc = (lane & 7) ^ (h & 7);
    h_vo[q] = (gr >= u0 && gr < u1) ? (uint32_t)((h * a.ldx + lc * 8) * 2) : kOOB;
  }
  uint32_t b_vo[BW];
#pragma unroll
  for (int i = 0; i < BW; ++i) {
    const int R = (wave * BW + i) * 8 + lrow;
    b_vo[i] = n0 + R < a.N ? (uint32_t)((R * a.K + ((lane & 7) ^ (R & 7)) * 8) * 2) : kOOB;
  }

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int a_row = wm * (BM / 2) + r16;
  const int b_row = wn * (BN / WN) + r16;
  const int b_off[2] = {b_row * BK + ((0 + g) ^ (b_row & 7)) * 8, b_row * BK + ((4 + g) ^ (b_row & 7)) * 8};
  // step s = cb * taps + j: weight tile (tap j, channel block cb) into ring slot s % BST; the
  // halo of channel block cb is staged at j == 0
  auto issue_a = [&](int cb, int aslot) {
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int pc = wave + NWAVE * q;
      if (pc < HP) glds16_buf(x_rs, As + aslot * A_E + pc * 8 * BK, h_vo[q], (uint32_t)(cb * BK * 2));
    }
  };
  int qa = 0;  // this wave's halo pieces (its LDS-DMA count per halo stage)
#pragma unroll
  for (int q = 0; q < QMAX; ++q) qa += (wave + NWAVE * q) < HP ? 1 : 0;
  auto issue_b = [&](int cb, int j, int slot) {
    const uint32_t k0 = (uint32_t)((j * a.Cin + cb * BK) * 2);
#pragma unroll
    for (int i = 0; i < BW; ++i) glds16_buf(w_rs, Bs + slot * B_E + (wave * BW + i) * 8 * BK, b_vo[i], k0);
  };
  // PIPE: one k-half (ks) of step (j, slot, aslot) into a register set, and its MFMAs
  // (nact: compile-time count of this wave's 16-row fragments that hold a valid row; the
  // others are neither read nor multiplied -- see mi_act below)
  auto frag_ld = [&](auto nact, int j, int slot, int aslot, int ks, bf16x8g (&fa)[MI],
                     bf16x8g (&fb)[NI]) {
    constexpr int NACT = decltype(nact)::value;
    const int ha = a_row + j * dil, sa = ha & 7;
    const u16* pa = As + aslot * A_E + ha * BK + ((ks * 4 + g) ^ sa) * 8;
    const u16* pb = Bs + slot * B_E + b_off[ks];
#pragma unroll
    for (int i = 0; i < NACT; ++i) fa[i] = *reinterpret_cast<const bf16x8g*>(pa + i * 16 * BK);
#pragma unroll
    for (int jj = 0; jj < NI; ++jj) fb[jj] = *reinterpret_cast<const bf16x8g*>(pb + jj * 16 * BK);
  };
  auto mfma_half = [&](auto nact, const bf16x8g (&fa)[MI], const bf16x8g (&fb)[NI]) {
    constexpr int NACT = decltype(nact)::value;
#pragma unroll
    for (int i = 0; i < NACT; ++i)
#pragma unroll
      for (int jj = 0; jj < NI; ++jj)
        acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[jj], acc[i][jj], 0, 0, 0);
  };
  auto compute = [&](int j, int slot, int aslot) {
    if (half_pad) return;
    // fragment rows differ by multiples of 16, so one swizzle serves all of them.  All 16
    // fragment reads of the step are issued before the first MFMA: the waits before the
    // MFMAs are then counted (the second k-half's reads land under the first half's MFMAs)
    const int ha = a_row + j * dil, sa = ha & 7;
    bf16x8g fa[2][MI], fb[2][NI];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const u16* pa = As + aslot * A_E + ha * BK + ((ks * 4 + g) ^ sa) * 8;
      const u16* pb = Bs + slot * B_E + b_off[ks];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[ks][i] = *reinterpret_cast<const bf16x8g*>(pa + i * 16 * BK);
#pragma unroll
      for (int jj = 0; jj < NI; ++jj) fb[ks][jj] = *reinterpret_cast<const bf16x8g*>(pb + jj * 16 * BK);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int jj = 0; jj < NI; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][i], fb[ks][jj], acc[i][jj], 0, 0, 0);
  };
  if (!skip) {
    const int ncb = cb1 - cb0;
    if constexpr (PIPE) {
      // Fragment-pipelined 2-slot loop.  Step s = (cb, j) reads weight slot s & 1 and halo slot
      // cb & 1 as two k-halves held in two register sets: set 1 (s, ks 1) is read while set 0's
      // MFMAs issue; then ONE barrier, after which set 0 is refilled with step s + 1's first
      // half under set 1's MFMAs -- a wave never waits on LDS right after the barrier.
      // At the barrier of step s every wave has retired all its reads of step s (lgkmcnt(0)),
      // so weight slot s & 1 takes tile s + 2 and, after cb's last tap, halo slot cb & 1 takes
      // channel block cb + 2.  Tile s + 1 (and its halo, issued earlier) must have landed:
      // it was issued at the previous barrier, followed at most by one halo (`pend` pieces of
      // this wave), and loads retire in issue order.  A wave whose rows are all padding runs
      // the same loads and barriers without fragments or MFMAs (a separate loop body, so the
      // compute body has no per-step branches for the wait-count analysis to merge).
      const int S = ncb * a.taps;
      issue_a(0, 0);
      issue_b(0, 0, 0);
      issue_b(0, 1, 1);  // taps >= 2: step 1 = (0, 1)
      int pend0 = 0;
      if (ncb > 1) {
        issue_a(1, 1);
        pend0 = qa;
      }
      vm_wait_n(BW + pend0);  // halo 0 and weight tile 0 landed
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      auto pipe_loop = [&](auto nact) {
        constexpr bool C = decltype(nact)::value > 0;
        bf16x8g fa0[MI], fb0[NI], fa1[MI], fb1[NI];
        if constexpr (C) frag_ld(nact, 0, 0, 0, 0, fa0, fb0);
        int cb = 0, j = 0, pend = pend0;
        // steps 0 .. S-2 (the last step, with no successor, is peeled below: a loop body whose
        // barrier half were conditional would merge two wait states before set 1's MFMAs)
        for (int s = 0; s + 1 < S; ++s) {
          const bool last_tap = j + 1 == a.taps;
          const int jn = last_tap ? 0 : j + 1, cbn = last_tap ? cb + 1 : cb;
          // set 0 landed under the previous step's second half (free wait).  The builtin form
          // (not inline asm) lets the compiler's wait-count pass see it: with 2 x 10 reads in
          // flight (beyond the 15-deep LDS counter) it would otherwise wait for set 1 as well
          // before set 0's MFMAs.
          __builtin_amdgcn_s_waitcnt(kLgkm0);
          if constexpr (C) {
            frag_ld(nact, j, s & 1, cb & 1, 1, fa1, fb1);
            mfma_half(nact, fa0, fb0);
          }
          __builtin_amdgcn_sched_barrier(0);
          vm_wait_n(pend);
          __builtin_amdgcn_s_waitcnt(kLgkm0);
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
          pend = 0;
          if (s + 2 < S) {
            const bool l2 = jn + 1 == a.taps;
            issue_b(l2 ? cbn + 1 : cbn, l2 ? 0 : jn + 1, s & 1);
          }
          if (last_tap && cb + 2 < ncb) {
            issue_a(cb + 2, cb & 1);
            pend = qa;
          }
          if constexpr (C) {
            frag_ld(nact, jn, (s + 1) & 1, cbn & 1, 0, fa0, fb0);
            mfma_half(nact, fa1, fb1);
          }
          __builtin_amdgcn_sched_barrier(0);
          cb = cbn;
          j = jn;
        }
        if constexpr (C) {
          __builtin_amdgcn_s_waitcnt(kLgkm0);
          frag_ld(nact, j, (S - 1) & 1, cb & 1, 1, fa1, fb1);
          mfma_half(nact, fa0, fb0);
          mfma_half(nact, fa1, fb1);
        }
      };
      // with lens, a wave whose rows past the first half of its fragments are all padding
      // runs the half-width body (their outputs are masked downstream, as for half_pad)
      if (half_pad) pipe_loop(std::integral_constant<int, 0>{});
      else if (mi_act <= MI / 2) pipe_loop(std::integral_constant<int, MI / 2>{});
      else pipe_loop(std::integral_constant<int, MI>{});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      // weight-tile ring of BST slots, BST-1 tiles ahead: step s = (cb, j) reads slot s % BST
      // while tiles s+1 .. s+BST-1 are in flight.  At a channel-block boundary the single
      // halo buffer is reloaded after a barrier (everyone finished the previous block).
      const int S = ncb * a.taps;
      issue_a(0, 0);
      for (int d = 0; d < BST - 1 && d < S; ++d) issue_b(d / a.taps, d % a.taps, d);
      int cb = 0, j = 0, slot = 0;
      for (int s = 0; s < S; ++s) {
        if (j == 0 && s > 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          issue_a(cb, 0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int sn = s + BST - 1;
        if (sn < S) {
          const int cbn = sn / a.taps;
          issue_b(cbn, sn - cbn * a.taps, sn % BST);
        }
        compute(j, slot, 0);
        slot = slot + 1 == BST ? 0 : slot + 1;
        if (++j == a.taps) {
          j = 0;
          ++cb;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  if (kz > 1) {  // raw fp32 partial product into slab z (halo_splitk_reduce applies the epilogue)
    GldsArgs e = a;
    e.flags = 0;
    e.y = a.slab + (int64_t)z * a.M * a.N;
    e.ldy = a.N;
    e.vec = 1;
    nt_epilogue<BM, BN, VOC, NWAVE, WN>(e, acc, smem, m0, n0, skip, tid, wm, wn, g, r16);
    return;
  }
  nt_epilogue<BM, BN, VOC, NWAVE, WN>(a, acc, smem, m0, n0, skip, tid, wm, wn, g, r16);
}

// Split-K epilogue of the halo kernel: y = epilogue(sum_z slab[z]) in split order, 8 columns
// per thread, with nt_epilogue's non-vocoder semantics (bias, aux add, ReLU / ReLU mask, bf16
// cast; tiles of BM rows that are all padding get no bias, as in the unsplit kernel).
template <int BM>
__global__ __launch_bounds__(256) void halo_splitk_reduce(GldsArgs a) {
  const int64_t n8 = a.N / 8, total = a.M * n8;
  const bool out_bf16 = a.flags & FS2_EPI_OUT_BF16, aux_bf16 = a.flags & FS2_EPI_AUX_BF16;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int64_t m = e / n8;
    const int n = (int)(e - m * n8) * 8;
    const float* sp = a.slab + m * a.N + n;
    f32x4 lo = ld4(sp), hi = ld4(sp + 4);
    for (int z = 1; z < a.kz; ++z) {
      const float* q = sp + (int64_t)z * a.M * a.N;
      lo += ld4(q);
      hi += ld4(q + 4);
    }
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const int64_t t0 = m / BM * BM;
    const bool skip = a.lens && rows_all_padding(a.lens, a.T, t0, t0 + BM < a.M ? t0 + BM : a.M);
    if ((a.flags & FS2_EPI_BIAS) && !skip) {
      const f32x4 b0 = ld4(a.bias + n), b1 = ld4(a.bias + n + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] += b0[i];
        v[i + 4] += b1[i];
      }
    }
    float av[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (a.flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX)) {
      if (aux_bf16) {
        const uint4 raw = *reinterpret_cast<const uint4*>((const u16*)a.aux + m * a.ld_aux + n);
        const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[2 * i] = __uint_as_float(wv[i] << 16);
          av[2 * i + 1] = __uint_as_float(wv[i] & 0xffff0000u);
        }
      } else {
        const float* ap = (const float*)a.aux + m * a.ld_aux + n;
        const f32x4 a0 = ld4(ap), a1 = ld4(ap + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[i] = a0[i];
          av[i + 4] = a1[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (a.flags & FS2_EPI_ADD_AUX) v[i] += av[i];
      if (a.flags & FS2_EPI_RELU) v[i] = fmaxf(v[i], 0.f);
      if (a.flags & FS2_EPI_RELU_MASK_AUX) v[i] = av[i] > 0.f ? v[i] : 0.f;
    }
    if (out_bf16) {
      uint4 o;
      o.x = (uint32_t)fbv(v[0]) | ((uint32_t)fbv(v[1]) << 16);
      o.y = (uint32_t)fbv(v[2]) | ((uint32_t)fbv(v[3]) << 16);
      o.z = (uint32_t)fbv(v[4]) | ((uint32_t)fbv(v[5]) << 16);
      o.w = (uint32_t)fbv(v[6]) | ((uint32_t)fbv(v[7]) << 16);
      *reinterpret_cast<uint4*>((u16*)a.y + m * a.ldy + n) = o;
    } else {
      float* yp = (float*)a.y + m * a.ldy + n;
      st4(yp, f32x4{v[0], v[1], v[2], v[3]});
      st4(yp + 4, f32x4{v[4], v[5], v[6], v[7]});
    }
  }
}

// fn(integral_constant<0>), ..., fn(integral_constant<N - 1>), in order
template <int N, typename Fn>
FS2_DEV void static_for(Fn&& fn) {
  if constexpr (N > 0) {
    static_for<N - 1>(fn);
    fn(std::integral_constant<int, N - 1>{});
  }
}

// ---------------------------------------------------------------- tap-register halo Conv1d
// conv_gemm_tapreg: the halo Conv1d (C_in % 64 == 0, taps > 1, undilated, every row tile inside
// one utterance) with each A fragment of a channel block read from LDS ONCE for all taps.
//
// A wave owns a band of 16 S rows x WC columns.  Its output fragment i (i < S) holds the band
// rows i + S m (m = 0..15), so tap j of fragment i needs the input rows i + j + S m: halo
// fragment F[i + j], where F[f] = rows f + S m of the band's halo (f < S + taps - 1).  The
// S + taps - 1 halo fragments of a channel block are each read from LDS once and held in a
// rolling register window (tap j uses F[j .. j + S - 1]: one new fragment per tap and k-half);
// per 64-channel block a 64 x 32 wave tile (S = 4, k = 9) reads 24 halo + 36 weight fragments
// for 144 MFMAs (0.42 per MFMA), the halo kernel's 128 x 32 wave tile 0.63.  Same MFMAs per output in the same (channel block, tap, k-half) order as the halo
// kernels: bitwise equal where both compute.
// LDS halo image: halo row h sits at position (h mod S) * RS + h / S, so every F[f] reads 16
// consecutive positions (chunk swizzle c ^ (h / S & 7): conflict-free ds_read_b128); the LDS-DMA
// source row of each position is fixed per block (zero line outside the utterance / length).
// Weight tiles (tap j, channel block cb) stream through a WS-slot ring, one barrier per tap;
// channel block cb + 1's halo is staged at tap 0 of block cb (two halo slots).
// Weight and halo registers rotate by k-half: after a tap's half-0 MFMAs the next tap's half-0
// weights and halo fragment (at the last tap the next block's first S halo fragments) are read
// under the half-1 MFMAs, and vice versa -- one register set of each.
// A wave whose band lies past the utterance's length stages its share but issues no MFMAs
// (those rows are masked downstream, as in conv_gemm_halo).
template <int BM, int BN, int WGM, int WGN, int S, int TAPS, int WS, int MINB>
__global__ __launch_bounds__(WGM * WGN * 64, MINB) void conv_gemm_tapreg(GldsArgs a) {
  constexpr int NW = WGM * WGN, BK = 64;
  constexpr int WR = 16 * S, WC = BN / WGN, NI = WC / 16;
  static_assert(BM == WGM * WR && WC % 16 == 0 && WGM % 2 == 0, "tile");
  constexpr int NF = S + TAPS - 1;
  constexpr int HR = BM + TAPS - 1, RS = (HR + S - 1) / S, HP = (S * RS + 7) / 8;
  constexpr int QMAX = (HP + NW - 1) / NW, BWP = BN / 8 / NW;
  static_assert(BN % (8 * NW) == 0, "weight pieces");
  constexpr int D = WS == 2 ? 2 : WS - 1;  // tile s + D is issued at step s
  static_assert(D <= 3 && TAPS >= D && (D - 2) * BWP + QMAX <= 8, "vmcnt bookkeeping");
  constexpr int A_E = HP * 8 * BK, B_E = BN * BK;
  constexpr int EPI_E = (BM / 2) * (BN + 4) * 2;
  constexpr int SMEM_E = 2 * A_E + WS * B_E > EPI_E ? 2 * A_E + WS * B_E : EPI_E;
  __shared__ __attribute__((aligned(1024))) u16 smem[SMEM_E];
  u16* As = smem;
  u16* Bs = smem + 2 * A_E;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int g = lane >> 4, r16 = lane & 15, lrow = lane >> 3;
  // block -> tile: XCD-contiguous runs, n fastest within a group (as conv_gemm_halo)
  const int nwg = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int gfull = a.tiles_m * a.group;
  const int ng = wg / gfull, rem = wg - ng * gfull;
  const int gsz = a.tiles_n - ng * a.group < a.group ? a.tiles_n - ng * a.group : a.group;
  const int tm = m_interleave(rem / gsz, a.tiles_m, a.lens != nullptr);
  const int tn = ng * a.group + (rem - (rem / gsz) * gsz);
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const bool skip = a.lens && rows_all_padding(a.lens, a.T, m0, m0 + BM < a.M ? m0 + BM : a.M);
  const int64_t u0 = (m0 / a.T) * a.T;
  const int64_t ulen = a.lens ? (a.lens[m0 / a.T] < a.T ? a.lens[m0 / a.T] : a.T) : a.T;
  const int64_t u1 = u0 + ulen < a.M ? u0 + ulen : a.M;
  const bool band_pad = m0 + wm * WR >= u1;

  // halo piece pc = wave + NW q: positions 8 pc + lrow, position P = res * RS + qq holds halo
  // row h = qq * S + res (global row m0 - pad + h)
  const auto x_rs = buf_rsrc(a.x + (m0 - a.pad) * a.ldx, (int64_t)HR * a.ldx * 2);
  const auto w_rs = buf_rsrc(a.w + (int64_t)n0 * a.K, (int64_t)BN * a.K * 2);
  uint32_t h_vo[QMAX];
  int qa = 0;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int pc = wave + NW * q, P = pc * 8 + lrow;
    const int res = P / RS, qq = P - res * RS, h = qq * S + res;
    const int64_t gr = m0 - a.pad + h;
    const int lc = (lane & 7) ^ (qq & 7);
    h_vo[q] = (pc < HP && res < S && h < HR && gr >= u0 && gr < u1)
                  ? (uint32_t)((h * a.ldx + lc * 8) * 2) : kOOB;
    qa += pc < HP ? 1 : 0;
  }
  uint32_t b_vo[BWP];
#pragma unroll
  for (int i = 0; i < BWP; ++i) {
    const int R = (wave * BWP + i) * 8 + lrow;
    b_vo[i] = n0 + R < a.N ? (uint32_t)((R * a.K + ((lane & 7) ^ (R & 7)) * 8) * 2) : kOOB;
  }
  auto issue_a = [&](int cb, int slot) {
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int pc = wave + NW * q;
      if (pc < HP) glds16_buf(x_rs, As + slot * A_E + pc * 8 * BK, h_vo[q], (uint32_t)(cb * BK * 2));
    }
  };
  auto issue_b = [&](int t) {  // weight tile t = (channel block t / TAPS, tap t % TAPS)
    const int cb = t / TAPS, j = t - cb * TAPS;
    const uint32_t k0 = (uint32_t)((j * a.Cin + cb * BK) * 2);
    u16* dst = Bs + (t % WS) * B_E + wave * BWP * 8 * BK;
#pragma unroll
    for (int i = 0; i < BWP; ++i) glds16_buf(w_rs, dst + i * 8 * BK, b_vo[i], k0);
  };

  f32x4 acc[S][NI];
#pragma unroll
  for (int i = 0; i < S; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8g F[NF][2], Bw[NI][2];
  // F[f] of this lane: position (f % S) * RS + wm * 16 + f / S + r16, swizzle key = its offset
  // within the residue class mod 8 = (r16 + f / S) & 7 -- one of (NF - 1) / S + 1 lane patterns
  // per k-half (the rest of the address is a compile-time offset)
  constexpr int NQ = (NF - 1) / S + 1;
  const u16* fa[NQ][2];
#pragma unroll
  for (int d = 0; d < NQ; ++d)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      fa[d][ks] = As + (r16 + wm * 16 + d) * BK + (((ks * 4 + g) ^ ((r16 + d) & 7)) * 8);
  const int b_row = wn * WC + r16;
  const u16* fb[2] = {Bs + b_row * BK + ((g ^ (b_row & 7)) * 8),
                      Bs + b_row * BK + (((4 + g) ^ (b_row & 7)) * 8)};
  auto rd_f = [&](int cb, int f, int ks) {
    F[f][ks] = *reinterpret_cast<const bf16x8g*>(fa[f / S][ks] + (cb & 1) * A_E + (f % S) * RS * BK);
  };
  auto rd_b = [&](int t, int ks) {
    const int so = (t % WS) * B_E;
#pragma unroll
    for (int jj = 0; jj < NI; ++jj) Bw[jj][ks] = *reinterpret_cast<const bf16x8g*>(fb[ks] + so + jj * 16 * BK);
  };
  auto mfma_half = [&](auto jc, int ks) {
    constexpr int J = decltype(jc)::value;
#pragma unroll
    for (int i = 0; i < S; ++i)
#pragma unroll
      for (int jj = 0; jj < NI; ++jj)
        acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[i + J][ks], Bw[jj][ks], acc[i][jj], 0, 0, 0);
  };

  if (!skip) {
    const int ncb = a.Cin / BK, Stot = ncb * TAPS;
    // prologue: halo 0, tiles 0 .. D-1
    issue_a(0, 0);
    issue_b(0);
    int pend = 0;
#pragma unroll
    for (int d = 1; d < D; ++d)
      if (d < Stot) {
        issue_b(d);
        pend += BWP;
      }
    vm_wait_n(pend);  // halo 0 and tile 0 landed
    __builtin_amdgcn_s_barrier();
    auto run = [&](auto cc) {
      constexpr bool C = decltype(cc)::value;
      if constexpr (C) {
#pragma unroll
        for (int f = 0; f < S; ++f) {
          rd_f(0, f, 0);
          rd_f(0, f, 1);
        }
        rd_b(0, 0);
        rd_b(0, 1);
      }
      for (int cb = 0; cb < ncb; ++cb) {
        const bool more = cb + 1 < ncb;
        auto step = [&](auto jc) {
          constexpr int J = decltype(jc)::value;
          const int s = cb * TAPS + J;
          // tile s + 1 landed (this wave's pieces); later DMA may stay in flight: tiles
          // s + 2 .. s + D - 1 and the halo issued at tap 0 when that came after tile s + 1
          int n = 0;
          if (D == 3 && s + 2 < Stot) n += BWP;
          if (J >= 1 && J <= D - 1 && more) n += qa;
          vm_wait_n(n);
          if constexpr (WS == 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
          if (s + D < Stot) issue_b(s + D);
          // block cb + 1's halo into the slot block cb - 1 used (its last reads, at tap
          // TAPS - 2, were consumed by the MFMAs of tap TAPS - 1: done before this barrier)
          if (J == 0 && more) issue_a(cb + 1, (cb + 1) & 1);
          if constexpr (C) {
            // tap J uses F[J .. J + S - 1]; F[J] is dead after it, F[J + S] is new at J + 1
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              mfma_half(jc, ks);
              __builtin_amdgcn_sched_barrier(0);
              if (s + 1 < Stot) rd_b(s + 1, ks);
              if constexpr (J + 1 < TAPS) {
                rd_f(cb, J + S, ks);
              } else if (more) {
#pragma unroll
                for (int f = 0; f < S; ++f) rd_f(cb + 1, f, ks);
              }
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        };
        static_for<TAPS>(step);
      }
    };
    if (band_pad) run(std::false_type{});
    else run(std::true_type{});
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  nt_epilogue<BM, BN, false, NW, WGN, WGM, S, true>(a, acc, smem, m0, n0, skip, tid, wm, wn, g, r16);
}

// ------------------------------------------------------------------------ weight gradient
//   slab[z][o][kk] = sum_{m in split z} dy[m, o] * x~[m, kk],  x~[m, j*Cin + c] = x[m + j - pad, c]
//   bslab[z][o]    = sum_{m in split z} dy[m, o]            (bias gradient, optional)
//
// Both operands are k-major ([reduction rows][channels]).  Tiles 128 (o) x 128 (kk) x 64
// rows; each operand's LDS image is [64 rows][128] bf16 (256-B rows), filled lane-linearly by
// glds (4 rows per wave-instruction) with the 16-B chunk swizzle c ^ ((R & 7) << 1) on the
// source, and read with ds_read_b64_tr_b16: a fragment's 8 k come from rows {4g+q} and
// {16+4g+q} of the 32-row k-step, so each 32-lane half reads 8 distinct rows x 2 chunks =
// 16 distinct bank slots.  The frame index of each staged row is carried incrementally
// across k-tiles (no division in the loop).  The bias gradient rides on the same A
// fragments: the waves of the first kk column tile multiply them by a ones fragment.
struct WgradGlds {
  const u16* dy;
  int64_t ldy;
  const u16* x;
  int64_t ldx;
  float* slab;
  float* bslab;
  int64_t M, T;
  int Cin, Cout, taps, pad, Kp;
  int64_t rows_per_split;
  int tiles_o, tiles_k, splits;
  const int64_t* lens;  // optional: 64-row k-tiles made only of padding rows are skipped
};

typedef short s16x4g __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4g lds_s16x4g;

// ds_read_b64_tr_b16 as inline asm.  The builtin's memory operand carries no alias scope, so
// hipcc's wait-count pass makes every such read wait for ALL LDS-DMA in flight (vmcnt(0)):
// issued after the next k-tile's DMA it drained the prefetch every k-tile, serialising the
// weight-gradient loops on one global round trip.  The asm read is invisible to that pass:
// the caller orders it after the DMA of the tile it reads (counted vmcnt + barrier, as the
// k-loops do) and waits for its result with lgkm_wait<N>() before use.
FS2_DEV s16x4g ds_tr16(const u16* p) {
  s16x4g r;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) u16*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// s_waitcnt lgkmcnt(N), then a scheduling fence: register-only MFMAs must not be hoisted
// above the wait (the asm reads' results are unknown to the compiler)
template <int N>
FS2_DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int BT, int STAGES>
__global__ __launch_bounds__(256) void conv_wgrad_tn_glds(WgradGlds a) {
  constexpr int BM = BT, BN = BT, BK = 64;  // BT = 128 or 64 (o and kk tile widths)
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int NCH = BT / 8;               // 16-B chunks per image row
  constexpr int RPI = 64 / NCH;             // image rows per glds wave-instruction
  constexpr int IPW = BK / RPI / 4;         // glds per wave per operand per tile
  constexpr int IMG = BK * BT;              // elements per operand image
  constexpr int STAGE_E = 2 * IMG;
  constexpr int EPI_LD = BN + 4;
  constexpr int EPI_E = (BM / 2) * EPI_LD * 2;
  constexpr int SMEM_E = STAGES * STAGE_E > EPI_E ? STAGES * STAGE_E : EPI_E;
  constexpr int MAXKT = 1024;  // k-tile list (skipping all-padding tiles) lives after the ring
  __shared__ __attribute__((aligned(1024))) u16 smem[SMEM_E + MAXKT + 64];
  short* ktl = reinterpret_cast<short*>(smem + SMEM_E);
  int* wcnt = reinterpret_cast<int*>(smem + SMEM_E + MAXKT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r16 = lane & 15;

  const int per_split = a.tiles_o * a.tiles_k;
  const int nwg = per_split * a.splits;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int z = wg / per_split, rem = wg - z * per_split;
  const int tk = rem % a.tiles_k, to = rem / a.tiles_k;
  const int o0 = to * BM, n0 = tk * BN;
  const int64_t r_begin = (int64_t)z * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.M) r_end = a.M;
  const int nk_all = r_end > r_begin ? (int)((r_end - r_begin + BK - 1) / BK) : 0;
  // ordered list of the split's k-tiles that hold at least one real row (wave ballots +
  // prefix popcounts; skipped tiles add exact zeros, so the sums are unchanged bitwise)
  const bool use_list = a.lens != nullptr && nk_all <= MAXKT;
  int nk = nk_all;
  if (use_list) {
    int total = 0;
    for (int c0 = 0; c0 < nk_all; c0 += 256) {
      const int kt = c0 + tid;
      bool v = false;
      if (kt < nk_all) {
        const int64_t q0 = r_begin + (int64_t)kt * BK;
        v = !rows_all_padding(a.lens, a.T, q0, q0 + BK < r_end ? q0 + BK : r_end);
      }
      const uint64_t mask = __ballot(v);
      if (lane == 0) wcnt[wave] = __popcll(mask);
      __syncthreads();
      int before = total;
      for (int w = 0; w < wave; ++w) before += wcnt[w];
      const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
      if (v) ktl[before + below] = (short)kt;
      for (int w = 0; w < 4; ++w) total += wcnt[w];
      __syncthreads();
    }
    nk = total;
  }

  // per-lane staging descriptors: instruction i stages rows RPI*(wave*IPW+i) + lane/NCH.
  // Chunk swizzle f(R): 256-B rows (BT 128) (R & 7) << 1; 128-B rows (BT 64)
  // ((R >> 1) & 3) << 1 -- either way a 32-lane transposed read (8 rows x 2 chunks) hits
  // 16 distinct 16-B bank slots.
  auto swz_of = [](int R) { return BT == 128 ? (R & 7) << 1 : ((R >> 1) & 3) << 1; };
  const u16* zero = reinterpret_cast<const u16*>(g_zero_line);
  const int pc = lane % NCH;
  int R[IPW], t_i[IPW], a_col[IPW], b_j[IPW], b_c[IPW];
  int64_t base_i[IPW];
  bool a_ok[IPW], b_ok[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    R[i] = (wave * IPW + i) * RPI + lane / NCH;
    const int lc = pc ^ swz_of(R[i]);
    a_col[i] = o0 + lc * 8;
    a_ok[i] = a_col[i] < a.Cout;
    const int kk = n0 + lc * 8;
    b_ok[i] = kk < a.Kp;
    b_j[i] = kk / a.Cin;
    b_c[i] = kk - b_j[i] * a.Cin;
    const int64_t m = r_begin + R[i];
    const int64_t s = m / a.T;
    t_i[i] = (int)(m - s * a.T);
    base_i[i] = s * a.T;
  }

  int cur_tile = 0;  // the k-tile whose rows t_i / base_i describe
  auto issue = [&](int kt, int stage) {
    u16* As = smem + stage * STAGE_E;
    u16* Bs = As + IMG;
    const int tile = use_list ? (int)ktl[kt] : kt;
    const int adv = (tile - cur_tile) * BK;
    cur_tile = tile;
    const int64_t k0 = r_begin + (int64_t)tile * BK;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      t_i[i] += adv;
      while (t_i[i] >= a.T) {
        t_i[i] -= (int)a.T;
        base_i[i] += a.T;
      }
      const int64_t m = k0 + R[i];
      const bool mok = m < r_end;
      const u16* sa = (mok && a_ok[i]) ? a.dy + m * a.ldy + a_col[i] : zero;
      glds16(sa, As + (wave * IPW + i) * RPI * BT);
      const int tt = t_i[i] + b_j[i] - a.pad;
      const u16* sb = (mok && b_ok[i] && tt >= 0 && tt < a.T)
                          ? a.x + (base_i[i] + tt) * a.ldx + b_c[i] : zero;
      glds16(sb, Bs + (wave * IPW + i) * RPI * BT);
    }
  };

  f32x4 acc[MI][NI], accb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool do_bias = a.bslab != nullptr && tk == 0 && wn == 0;  // wave-uniform
  bf16x8g ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // transposed fragment: 16 columns at col0, k-step ks; rows {4g+q} and {16+4g+q}
  const int swz = swz_of(4 * g + q);
  // transposed fragment halves (asm reads, see ds_tr16): rows ks*32 + {4g+q} and + 16
  auto tr_lo = [&](const u16* img, int col0, int ks, int hi) -> s16x4g {
    const int lc = (col0 >> 3) + (p >> 1);
    const int off = (ks * 32 + 4 * g + q + 16 * hi) * BT + ((lc ^ swz) << 3) + ((p & 1) << 2);
    return ds_tr16(img + off);
  };
  auto cat = [](s16x4g lo, s16x4g hi) {
    return __builtin_bit_cast(bf16x8g, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  // both k-halves' fragment reads issued up front; the first half's MFMAs start once its reads
  // (the older 2 (MI + NI)) landed
  auto compute = [&](int stage) {
    const u16* As = smem + stage * STAGE_E;
    const u16* Bs = As + IMG;
    s16x4g ra[2][MI][2], rb[2][NI][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) ra[ks][i][h] = tr_lo(As, wm * (BM / 2) + i * 16, ks, h);
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) rb[ks][j][h] = tr_lo(Bs, wn * (BN / 2) + j * 16, ks, h);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0) lgkm_wait<(2 * (MI + NI) < 15 ? 2 * (MI + NI) : 15)>();  // 4-bit counter
      else lgkm_wait<0>();
      bf16x8g fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = cat(ra[ks][i][0], ra[ks][i][1]);
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = cat(rb[ks][j][0], rb[ks][j][1]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
          accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb[i], 0, 0, 0);
      }
    }
  };

  kloop<STAGES, 2 * IPW>(nk, issue, compute);

  if (do_bias && r16 == 0) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + wm * (BM / 2) + i * 16 + 4 * g + r;
        if (o < a.Cout) a.bslab[(int64_t)z * a.Cout + o] = accb[i][r];
      }
  }
  // slab tile through LDS: rows o, 8 consecutive kk per thread (32-B stores)
  float* Cs = reinterpret_cast<float*>(smem);
  float* slab = a.slab + (int64_t)z * a.Cout * a.Kp;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(i * 16 + 4 * g + r) * EPI_LD + wn * (BN / 2) + j * 16 + r16] = acc[i][j][r];
    }
    __syncthreads();
    constexpr int TPR = BN / 8, RPP = 256 / TPR;
    const int cc = (tid % TPR) * 8;
    const int kk = n0 + cc;
#pragma unroll
    for (int pp = 0; pp < (BM / 2) / RPP; ++pp) {
      const int rr = pp * RPP + tid / TPR;
      const int o = o0 + h * (BM / 2) + rr;
      if (o < a.Cout && kk < a.Kp) {
        float* dst = slab + (int64_t)o * a.Kp + kk;
        *reinterpret_cast<f32x4*>(dst) = *reinterpret_cast<const f32x4*>(Cs + rr * EPI_LD + cc);
        *reinterpret_cast<f32x4*>(dst + 4) = *reinterpret_cast<const f32x4*>(Cs + rr * EPI_LD + cc + 4);
      }
    }
    __syncthreads();
  }
}

// Halo weight gradient for Conv1d with 2 <= taps <= 9 (C_in, C_out multiples of 64, T a
// multiple of 64), the split-K path for grids that conv_wgrad_band (wgrad.hip) cannot fill:
// a block owns a 64 (o) x 64 (c) tile for ALL taps.  Per 64-row k-tile it stages the dy tile
// (64 x 64) and the x rows of the tile plus the tap halo (64 + taps - 1 rows, zero outside the
// utterance) ONCE, and tap j reads the x image at row offset j.  Both images are [rows][64]
// bf16 (128-B rows) filled by LDS-DMA with the chunk swizzle ((R >> 1) & 3) << 1 and read with
// ds_read_b64_tr_b16 (rows {4g+q} u {16+4g+q} of a 32-row step).  Each wave owns 64 (o) x 16
// (c) for all taps: the dy fragments (4 per k-step) are read once and reused by every tap, a
// tap costs ONE shifted x fragment for 4 MFMAs, and the next taps' x fragments are read under
// the current tap's MFMAs.  Each wave also carries the bias gradient of its 16 o rows.
// Output: the split-K slab layout (and bias slab) of conv_wgrad_tn_glds.
template <int TAPS>
__global__ __launch_bounds__(256, 2) void conv_wgrad_halo(WgradGlds a) {
  constexpr int BO = 64, BC = 64, BK = 64, STAGES = 2;
  constexpr int HX = 8;                      // halo rows allocated (taps <= 9)
  constexpr int A_E = BK * BO;               // dy image
  constexpr int X_E = (BK + HX) * BC;        // x halo image
  constexpr int STAGE_E = A_E + X_E;
  constexpr int MAXKT = 1024;
  __shared__ __attribute__((aligned(1024))) u16 smem[STAGES * STAGE_E + MAXKT + 64];
  short* ktl = reinterpret_cast<short*>(smem + STAGES * STAGE_E);
  int* wcnt = reinterpret_cast<int*>(smem + STAGES * STAGE_E + MAXKT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r16 = lane & 15;

  const int per_split = a.tiles_o * a.tiles_k;  // tiles_k = C_in / 64 here
  const int nwg = per_split * a.splits;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int z = wg / per_split, rem = wg - z * per_split;
  const int tc = rem % a.tiles_k, to = rem / a.tiles_k;
  const int o0 = to * BO, c0 = tc * BC;
  const int64_t r_begin = (int64_t)z * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.M) r_end = a.M;
  const int nk_all = r_end > r_begin ? (int)((r_end - r_begin + BK - 1) / BK) : 0;
  const bool use_list = a.lens != nullptr && nk_all <= MAXKT;
  int nk = nk_all;
  if (use_list) {  // ordered list of k-tiles holding a real row (as conv_wgrad_tn_glds)
    int total = 0;
    for (int cc0 = 0; cc0 < nk_all; cc0 += 256) {
      const int kt = cc0 + tid;
      bool v = false;
      if (kt < nk_all) {
        const int64_t k0 = r_begin + (int64_t)kt * BK;
        v = !rows_all_padding(a.lens, a.T, k0, k0 + BK < r_end ? k0 + BK : r_end);
      }
      const uint64_t mask = __ballot(v);
      if (lane == 0) wcnt[wave] = __popcll(mask);
      __syncthreads();
      int before = total;
      for (int w = 0; w < wave; ++w) before += wcnt[w];
      const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
      if (v) ktl[before + below] = (short)kt;
      for (int w = 0; w < 4; ++w) total += wcnt[w];
      __syncthreads();
    }
    nk = total;
  }

  auto swz = [](int R) { return ((R >> 1) & 3) << 1; };
  const u16* zero = reinterpret_cast<const u16*>(g_zero_line);
  const int lrow = lane >> 3, lch = lane & 7;
  const int HR = BK + a.taps - 1, HP = (HR + 7) / 8;  // x halo rows / 8-row pieces
  auto issue = [&](int kt, int stage) {
    u16* As = smem + stage * STAGE_E;
    u16* Xs = As + A_E;
    const int tile = use_list ? (int)ktl[kt] : kt;
    const int64_t k0 = r_begin + (int64_t)tile * BK;
    // the 64 rows of a k-tile lie in one utterance (T % 64 == 0, splits are 64-row aligned)
    const int64_t u0 = (k0 / a.T) * a.T, u1 = u0 + a.T < a.M ? u0 + a.T : a.M;
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // dy: 8 pieces of 8 rows, 2 per wave
      const int R = (wave * 2 + i) * 8 + lrow;
      const int64_t m = k0 + R;
      const u16* src = m < r_end ? a.dy + m * a.ldy + o0 + ((lch ^ swz(R)) << 3) : zero;
      glds16(src, As + (wave * 2 + i) * 8 * BO);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // x halo: up to 9 pieces, wave + 4 i
      const int pc = wave + 4 * i;
      if (pc < HP) {
        const int h = pc * 8 + lrow;
        const int64_t gr = k0 - a.pad + h;
        // rows past the split's end only meet zero dy rows; only the utterance matters
        const u16* src = (gr >= u0 && gr < u1) ? a.x + gr * a.ldx + c0 + ((lch ^ swz(h)) << 3)
                                               : zero;
        glds16(src, Xs + pc * 8 * BC);
      }
    }
  };

  f32x4 acc[TAPS][4], accb = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < TAPS; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.bslab != nullptr && tc == 0;  // block-uniform
  bf16x8g ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // transposed fragment (asm reads, see ds_tr16; the caller waits with lgkm_wait): 16 columns
  // at col0, rows rb + {4g+q} and rb + {16+4g+q}
  auto tr_frag = [&](const u16* img, int rb, int col0) -> bf16x8g {
    const int R = rb + 4 * g + q;
    const int lc = (col0 >> 3) + (p >> 1);
    const int off = R * 64 + ((lc ^ swz(R)) << 3) + ((p & 1) << 2);
    const s16x4g lo = ds_tr16(img + off);
    const s16x4g hi = ds_tr16(img + off + 16 * 64);
    return __builtin_bit_cast(bf16x8g, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto compute = [&](int stage) {
    const u16* As = smem + stage * STAGE_E;
    const u16* Xs = As + A_E;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // x fragments two taps ahead in a ring of three: tap j's MFMAs wait only for the reads
      // up to its fragment (the LDS latency exceeds one tap's 4 MFMAs)
      bf16x8g fa[4], fb[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = tr_frag(As, ks * 32, i * 16);
      fb[0] = tr_frag(Xs, ks * 32, wave * 16);
      if (TAPS > 1) fb[1] = tr_frag(Xs, ks * 32 + 1, wave * 16);
#pragma unroll
      for (int j = 0; j < TAPS; ++j) {
        if (j + 2 < TAPS) {
          fb[(j + 2) % 3] = tr_frag(Xs, ks * 32 + j + 2, wave * 16);
          lgkm_wait<4>();  // all but the x fragments of taps j + 1, j + 2 landed
        } else if (j + 1 < TAPS) {
          lgkm_wait<2>();
        } else {
          lgkm_wait<0>();
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j % 3], acc[j][i], 0, 0, 0);
      }
      if (do_bias) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i == wave) accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb, 0, 0, 0);
      }
    }
  };

  kloop<STAGES, 5>(nk, issue, compute);  // per-wave DMA count varies (<= 5): vmcnt(0)-style

  if (do_bias && r16 == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) a.bslab[(int64_t)z * a.Cout + o0 + wave * 16 + 4 * g + r] = accb[r];
  }
  // slab[z][o][j*Cin + c]: 16 consecutive c per row group (64-B runs)
  float* slab = a.slab + (int64_t)z * a.Cout * a.Kp;
#pragma unroll
  for (int j = 0; j < TAPS; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = o0 + i * 16 + 4 * g + r;
        const int c = c0 + wave * 16 + r16;
        slab[(int64_t)o * a.Kp + (int64_t)j * a.Cin + c] = acc[j][i][r];
      }
}

// dw[o][c][j] (+)= sum_z slab[z][o][j*Cin + c]; db[o] += sum_z bslab[z][o].  Split order is
// fixed (bitwise reproducible).  taps == 1: the layouts coincide, 4 consecutive elements per
// thread.  taps > 1: one block per (o, 64-channel chunk); slab rows are read as 256-B runs
// per tap and the [c][j] block is written contiguously.
__global__ __launch_bounds__(256) void wgrad_reduce_k1(const float* __restrict__ slab,
                                                       const float* __restrict__ bslab, int splits,
                                                       int Cout, int64_t total, float* dw, float* db) {
  // 64 float4 columns x 4 split groups: group y sums splits y, y+4, ... in order, then the
  // 4 group sums are added in group order (fixed order, bitwise reproducible)
  __shared__ f32x4 red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t i4 = ((int64_t)blockIdx.x * 64 + tx) * 4;
  f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
  if (i4 < total) {
#pragma unroll 4
    for (int zz = ty; zz < splits; zz += 4) s += ld4(slab + zz * total + i4);
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && i4 < total)
    st4(dw + i4, ld4(dw + i4) + (((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]));
  // bias: one output per thread over the first blocks (block 0 looping over every output
  // made the launch's tail), split loads four at a time, summed in split order
  const int ob = blockIdx.x * 256 + threadIdx.x;
  if (db && ob < Cout) {
    float b = 0.f;
    int zz = 0;
    for (; zz + 3 < splits; zz += 4) {
      const float v0 = bslab[(int64_t)zz * Cout + ob], v1 = bslab[(int64_t)(zz + 1) * Cout + ob];
      const float v2 = bslab[(int64_t)(zz + 2) * Cout + ob], v3 = bslab[(int64_t)(zz + 3) * Cout + ob];
      b += v0;
      b += v1;
      b += v2;
      b += v3;
    }
    for (; zz < splits; ++zz) b += bslab[(int64_t)zz * Cout + ob];
    db[ob] += b;
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_taps(const float* __restrict__ slab,
                                                         const float* __restrict__ bslab,
                                                         int splits, int Cout, int Cin, int taps,
                                                         float* dw, float* db) {
  __shared__ float tile[64 * 33];
  const int o = blockIdx.y, c0 = blockIdx.x * 64;
  const int64_t Kp = (int64_t)taps * Cin, total = (int64_t)Cout * Kp;
  const int nc = Cin - c0 < 64 ? Cin - c0 : 64;
  for (int jb = 0; jb < taps; jb += 32) {
    const int nj = taps - jb < 32 ? taps - jb : 32;
    // 16-B loads: thread e owns 4 consecutive channels of one tap row (nc and every offset
    // are multiples of 4); split slabs four at a time, summed in split order
    for (int e = threadIdx.x; e < 16 * nj; e += 256) {
      const int jj = e >> 4, c = (e & 15) * 4;
      if (c < nc) {
        const int64_t off = (int64_t)o * Kp + (int64_t)(jb + jj) * Cin + c0 + c;
        f32x4 s = ld4(slab + off);
        int zz = 1;
        for (; zz + 3 < splits; zz += 4) {
          const f32x4 v0 = ld4(slab + zz * total + off), v1 = ld4(slab + (zz + 1) * total + off);
          const f32x4 v2 = ld4(slab + (zz + 2) * total + off), v3 = ld4(slab + (zz + 3) * total + off);
          s += v0;
          s += v1;
          s += v2;
          s += v3;
        }
        for (; zz < splits; ++zz) s += ld4(slab + zz * total + off);
        tile[(c + 0) * 33 + jj] = s.x;
        tile[(c + 1) * 33 + jj] = s.y;
        tile[(c + 2) * 33 + jj] = s.z;
        tile[(c + 3) * 33 + jj] = s.w;
      }
    }
    __syncthreads();
    float* out = dw + ((int64_t)o * Cin + c0) * taps;
    for (int e = threadIdx.x; e < nc * nj; e += 256) {
      const int c = e / nj, jj = e - c * nj;
      out[(int64_t)c * taps + jb + jj] += tile[c * 33 + jj];
    }
    __syncthreads();
  }
  if (db && blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f;
    for (int zz = 0; zz < splits; ++zz) s += bslab[(int64_t)zz * Cout + o];
    db[o] += s;
  }
}

// taps > 1, one workgroup per output row o: the S slab rows (taps * Cin contiguous floats each)
// are summed in split order with 16-B loads, S loads in flight per chunk, into LDS, then added
// to dw[o][c][j] in output order (the [j][c] -> [c][j] transpose through LDS; coalesced 4-B
// read-modify-writes).  Same split order as wgrad_reduce_taps (bitwise equal), a quarter of its
// workgroups, every slab row read as one contiguous run.
constexpr int RROW_MAX = 9 * 1024;
__global__ __launch_bounds__(256) void wgrad_reduce_rows(const float* __restrict__ slab,
                                                         const float* __restrict__ bslab,
                                                         int splits, int Cout, int Cin, int taps,
                                                         float* dw, float* db) {
  __shared__ float row[RROW_MAX];
  const int o = blockIdx.x, Kp = taps * Cin;
  const int64_t total = (int64_t)Cout * Kp;
  const float* src = slab + (int64_t)o * Kp;
  for (int e4 = threadIdx.x; e4 < Kp / 4; e4 += 256) {
    f32x4 s = ld4(src + 4 * e4);
    for (int z = 1; z < splits; ++z) s += ld4(src + z * total + 4 * e4);
    *reinterpret_cast<f32x4*>(row + 4 * e4) = s;
  }
  __syncthreads();
  float* out = dw + (int64_t)o * Kp;
  for (int e = threadIdx.x; e < Kp; e += 256) {
    const int c = e / taps, j = e - c * taps;
    out[e] += row[j * Cin + c];
  }
  if (db && threadIdx.x == 0) {
    float b = 0.f;
    for (int z = 0; z < splits; ++z) b += bslab[(int64_t)z * Cout + o];
    db[o] += b;
  }
}

int conv_wgrad_glds_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                           float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out,
                           int taps, int pad, const int64_t* lens, int splits, int tile, float* ws,
                           hipStream_t st) {
  FS2_CHECK_ARG(c_in % 8 == 0 && c_out % 8 == 0 && ldx % 8 == 0 && ldy % 8 == 0 &&
                    ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0,
                "fs2_conv_wgrad(bf16): channel counts / strides must be multiples of 8, operands 16-B aligned");
  int64_t rps = (rows + splits - 1) / splits;
  rps = (rps + 63) / 64 * 64;
  const int64_t Kp = taps * c_in;
  float* bslab = db ? ws + splits * c_out * Kp : nullptr;
  WgradGlds a{(const u16*)dy, ldy, (const u16*)x, ldx, ws, bslab, rows, seq_len, (int)c_in,
              (int)c_out, taps, pad, (int)Kp, rps, (int)((c_out + tile - 1) / tile),
              (int)((Kp + tile - 1) / tile), splits, lens};
  if (taps > 1 && g_tune[FS2_TUNE_WGRAD_HALO] == 0) {
    // 64 x 64 x taps tiles shared by eight waves (conv_wgrad_wide, wgrad.hip)
    const int rcw = conv_wgrad_wide_launch(dy, ldy, x, ldx, dw, db, rows, seq_len, c_in, c_out,
                                           taps, pad, lens, ws, st);
    if (rcw != kNotEligible) return rcw;
  }
  if (taps > 1 && g_tune[FS2_TUNE_WGRAD_HALO] == 0) {
    // no split slabs where the output tiles fill the chip (conv_wgrad_band, wgrad.hip)
    const int rc = conv_wgrad_band_launch(dy, ldy, x, ldx, dw, db, rows, seq_len, c_in, c_out,
                                          taps, pad, lens, st);
    if (rc != kNotEligible) return rc;
  }
  const bool halo = taps >= 2 && taps <= 9 && (taps == 3 || taps == 5 || taps == 9) &&
                    c_in % 64 == 0 && c_out % 64 == 0 && seq_len % 64 == 0 &&
                    g_tune[FS2_TUNE_WGRAD_HALO] >= 0;
  if (halo) {
    a.tiles_o = (int)(c_out / 64);
    a.tiles_k = (int)(c_in / 64);
    const unsigned hgrid = (unsigned)(a.tiles_o * a.tiles_k * splits);
    if (taps == 9) conv_wgrad_halo<9><<<hgrid, 256, 0, st>>>(a);
    else if (taps == 5) conv_wgrad_halo<5><<<hgrid, 256, 0, st>>>(a);
    else conv_wgrad_halo<3><<<hgrid, 256, 0, st>>>(a);
  }
  const unsigned grid = (unsigned)(a.tiles_o * a.tiles_k * splits);
  const int stages = g_tune[FS2_TUNE_WGRAD_STAGES] >= 1 && g_tune[FS2_TUNE_WGRAD_STAGES] <= 4
                         ? g_tune[FS2_TUNE_WGRAD_STAGES] : (tile == 128 ? 1 : 2);
#define FS2_WG(BT, S) conv_wgrad_tn_glds<BT, S><<<grid, 256, 0, st>>>(a)
  if (halo) {
  } else if (tile == 128) {
    switch (stages) {
      case 2: FS2_WG(128, 2); break;
      case 3: FS2_WG(128, 3); break;
      case 4: FS2_WG(128, 4); break;
      default: FS2_WG(128, 1);
    }
  } else {
    switch (stages) {
      case 2: FS2_WG(64, 2); break;
      case 3: FS2_WG(64, 3); break;
      case 4: FS2_WG(64, 4); break;
      default: FS2_WG(64, 1);
    }
  }
#undef FS2_WG
  if (taps == 1) {
    const int64_t total = c_out * c_in;  // multiple of 64 (both channel counts % 8 == 0)
    wgrad_reduce_k1<<<(unsigned)((total / 4 + 63) / 64), 256, 0, st>>>(ws, bslab, splits,
                                                                     (int)c_out, total, dw, db);
  } else if (taps * c_in <= RROW_MAX && c_in % 4 == 0) {
    wgrad_reduce_rows<<<(unsigned)c_out, 256, 0, st>>>(ws, bslab, splits, (int)c_out, (int)c_in,
                                                       taps, dw, db);
  } else {
    dim3 rg((unsigned)((c_in + 63) / 64), (unsigned)c_out);
    wgrad_reduce_taps<<<rg, 256, 0, st>>>(ws, bslab, splits, (int)c_out, (int)c_in, taps, dw, db);
  }
  return launch_status("fs2_conv_wgrad(bf16)");
}


static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

template <int BM, int BN, int S>
static void launch_nt(GldsArgs a, bool tapaligned, bool voc, hipStream_t st) {
  // n-tiles per group: all of them by default (measured: smaller weight-slice groups did not
  // pay on the step's shapes and multiplied the A re-reads of the long-K data gradient)
  const int g = g_tune[FS2_TUNE_NT_GROUP] > 0 ? g_tune[FS2_TUNE_NT_GROUP] : a.tiles_n;
  a.group = g > a.tiles_n ? a.tiles_n : g;
  const unsigned grid = (unsigned)(a.tiles_m * a.tiles_n);
  if (voc) {  // vocoder convs: one pipeline depth, dilation + the extended epilogue
    if (tapaligned) conv_gemm_nt_glds<BM, BN, 2, true, true><<<grid, 256, 0, st>>>(a);
    else conv_gemm_nt_glds<BM, BN, 2, false, true><<<grid, 256, 0, st>>>(a);
  } else if (tapaligned && a.taps == 1 && g_tune[FS2_TUNE_NT_K1] >= 0) {
    conv_gemm_nt_glds<BM, BN, S, true, false, true><<<grid, 256, 0, st>>>(a);
  } else if (tapaligned) {
    conv_gemm_nt_glds<BM, BN, S, true, false><<<grid, 256, 0, st>>>(a);
  } else {
    conv_gemm_nt_glds<BM, BN, S, false, false><<<grid, 256, 0, st>>>(a);
  }
}

// Split-K choice + workspace for the 64x64 halo kernel.  A grid below ~3 blocks per CU with a
// long channel loop (the encoder's k=9 data gradient: 384 tiles, 16 channel blocks x 9 taps
// each) leaves CUs with one block and the rest with two; splitting the channel blocks kz ways
// fills the chip and halves each block's serial loop, at the cost of kz fp32 partial products
// summed by halo_splitk_reduce.
//
// The decomposition is a function of the shape alone (halo_splitk_count): no stream, capture
// or allocation state can change it, so every call of a shape sums in one fp32 order.  The
// partials live in process-wide buffers (halo_splitk_slab), one for eager calls and one for
// calls recorded into a graph (a replay must not share scratch with eager work on another
// stream); both grow together, outside capture only.  Any failure to provide them -- a capture
// needing more than an earlier eager call sized, an event or allocation error -- is an error
// of the call, never a silent switch to the unsplit launch.  (Rounds 4 / 5 fell back to the
// unsplit kernel, a different summation order, on such failures: a process-history-dependent
// result.)  Stream order between eager users: each eager split launch pair records one event
// after its reduce (halo_splitk_done) and the next eager user's stream always waits on it.
// A graph buffer is never freed while a graph may still replay it (retired on growth).
static std::mutex g_splitk_mu;
static hipEvent_t g_splitk_ev = nullptr;
static bool g_splitk_recorded = false;
static float* g_slab[2] = {nullptr, nullptr};  // [0] eager calls, [1] captured calls
static size_t g_slab_cap = 0;
static bool g_slab_captured = false;  // g_slab[1] is referenced by a captured graph
static void halo_splitk_done(hipStream_t st) {
  std::lock_guard<std::mutex> lock(g_splitk_mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  if (g_splitk_ev && hipEventRecord(g_splitk_ev, st) == hipSuccess) g_splitk_recorded = true;
}
static int halo_splitk_count(const GldsArgs& a, unsigned grid, bool voc, bool hx64) {
  const int knob = g_tune[FS2_TUNE_HALO_SPLITK];
  const int ncb = a.Cin / 64;
  const int keep = FS2_EPI_BIAS | FS2_EPI_RELU | FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX |
                   FS2_EPI_OUT_BF16 | FS2_EPI_AUX_BF16;
  if (knob == -1 || voc || hx64 || !a.vec || (a.flags & ~keep) || a.N % 8) return 1;
  int kz = knob > 0 ? knob : (grid < 512 && ncb >= 8 ? (int)((768 + grid - 1) / grid) : 1);
  if (kz > ncb / 4) kz = ncb / 4;
  return kz < 2 ? 1 : kz;
}
static int halo_splitk_slab(GldsArgs& a, int kz, hipStream_t st) {
  const size_t need = (size_t)kz * (size_t)a.M * (size_t)a.N * sizeof(float);
  std::lock_guard<std::mutex> lock(g_splitk_mu);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
    set_error("fs2_conv_gemm: split-K: stream capture query failed");
    return FS2_ERR_LAUNCH;
  }
  const bool capturing = cs != hipStreamCaptureStatusNone;
  if (capturing) {
    if (g_slab_cap < need) {
      set_error("fs2_conv_gemm: split-K partials of %zu bytes needed during graph capture; run the "
                "same shapes eagerly once before capturing (%zu bytes sized)", need, g_slab_cap);
      return FS2_ERR_LAUNCH;
    }
    g_slab_captured = true;
    a.slab = g_slab[1];
  } else {
    if (!g_splitk_ev && hipEventCreateWithFlags(&g_splitk_ev, hipEventDisableTiming) != hipSuccess) {
      g_splitk_ev = nullptr;
      set_error("fs2_conv_gemm: split-K: event creation failed");
      return FS2_ERR_LAUNCH;
    }
    // the previous eager user's reduce has read the buffer before this stream writes it
    if (g_splitk_recorded && hipStreamWaitEvent(st, g_splitk_ev, 0) != hipSuccess) {
      set_error("fs2_conv_gemm: split-K: stream wait failed");
      return FS2_ERR_LAUNCH;
    }
    if (g_slab_cap < need) {
      if (hipDeviceSynchronize() != hipSuccess) {
        set_error("fs2_conv_gemm: split-K: device synchronisation failed");
        return FS2_ERR_LAUNCH;
      }
      (void)hipFree(g_slab[0]);
      if (!g_slab_captured) (void)hipFree(g_slab[1]);  // else retired: a graph may replay it
      g_slab[0] = g_slab[1] = nullptr;
      g_slab_cap = 0;
      g_slab_captured = false;
      void *p0 = nullptr, *p1 = nullptr;
      if (hipMalloc(&p0, need) != hipSuccess || hipMalloc(&p1, need) != hipSuccess) {
        (void)hipFree(p0);
        set_error("fs2_conv_gemm: split-K: hipMalloc of %zu bytes failed", need);
        return FS2_ERR_LAUNCH;
      }
      g_slab[0] = static_cast<float*>(p0);
      g_slab[1] = static_cast<float*>(p1);
      g_slab_cap = need;
    }
    a.slab = g_slab[0];
  }
  poison(a.slab, (int64_t)need, st);
  return FS2_OK;
}

// n-tiles per tile group of the halo kernels (FS2_TUNE_NT_GROUP; default: all of them)
static int halo_group(int tiles_n) {
  const int g = g_tune[FS2_TUNE_NT_GROUP];
  return g > 0 && g < tiles_n ? g : tiles_n;
}

// fs2_conv_gemm_ln: the tap-major kernel on 64 x 256 tiles (whole 256-wide rows; 128 x 256
// with FS2_TUNE_LN_TILE = 1) with the LayerNorm epilogue
int conv_gemm_ln_glds_launch(const void* x, int64_t ldx, const void* wk, int64_t rows,
                             int64_t seq_len, int64_t c_in, int taps, int pad, const int64_t* lens,
                             const float* bias, const float* res, const float* gamma,
                             const float* beta, float* out, void* out_t, float* xhat, float* rstd,
                             float p_in, const uint64_t* seed, uint64_t site_in, hipStream_t st) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  FS2_CHECK_ARG(c_in % 8 == 0 && ldx % 8 == 0 && al16(x) && al16(wk),
                "fs2_conv_gemm_ln: c_in/ldx must be multiples of 8 and operands 16-B aligned");
  FS2_CHECK_ARG(al16(out) && al16(xhat) && al16(gamma) && al16(beta) && al16(res) && al16(bias) &&
                    al16(out_t),
                "fs2_conv_gemm_ln: LayerNorm tensors must be 16-B aligned");
  GldsArgs a{(const u16*)x, ldx, (const u16*)wk, nullptr, 256, rows, seq_len, (int)c_in, 256,
             taps, pad, (int)(taps * c_in), bias, bias ? FS2_EPI_BIAS : 0, nullptr, 0, 0, 0, 1, 1,
             lens, 1, 0.f, 1.f, nullptr, 0.f};
  a.ln_res = res;
  a.ln_gamma = gamma;
  a.ln_beta = beta;
  a.ln_out = out;
  a.ln_out_t = (u16*)out_t;
  a.ln_xhat = xhat;
  a.ln_rstd = rstd;
  a.ln_seed = p_in > 0.f ? seed : nullptr;
  a.ln_site = site_in;
  a.ln_p = p_in;
  const bool wide = g_tune[FS2_TUNE_LN_TILE] == 1;
  const int bm = wide ? 128 : 64;
  a.tiles_m = (int)((rows + bm - 1) / bm);
  a.tiles_n = 1;
  const unsigned grid = (unsigned)a.tiles_m;
  const bool tapaligned = c_in % 64 == 0;
  const bool k1 = tapaligned && taps == 1 && g_tune[FS2_TUNE_NT_K1] >= 0;
  if (wide) {
    if (tapaligned) conv_gemm_nt_glds<128, 256, 2, true, false><<<grid, 256, 0, st>>>(a);
    else conv_gemm_nt_glds<128, 256, 2, false, false><<<grid, 256, 0, st>>>(a);
  } else {
    if (k1) conv_gemm_nt_glds<64, 256, 2, true, false, true><<<grid, 256, 0, st>>>(a);
    else if (tapaligned) conv_gemm_nt_glds<64, 256, 2, true, false><<<grid, 256, 0, st>>>(a);
    else conv_gemm_nt_glds<64, 256, 2, false, false><<<grid, 256, 0, st>>>(a);
  }
  return launch_status("fs2_conv_gemm_ln");
}

// fs2_conv_gemm_ln_bwd: the tap-major kernel on 64 x 256 tiles with the LayerNorm-backward
// epilogue (ws = fs2_ln_bwd's partial layout; the caller runs fs2_ln_bwd_final)
int conv_gemm_lnbwd_glds_launch(const void* x, int64_t ldx, const void* wk, int64_t rows,
                                int64_t seq_len, int64_t c_in, int taps, int pad,
                                const int64_t* lens, const float* aux, const float* xhat,
                                const float* rstd, const float* gamma, float p_in,
                                const uint64_t* seed, uint64_t site_in, float* dres, int dres_add,
                                void* dy_t, float* ws, hipStream_t st) {
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  FS2_CHECK_ARG(c_in % 8 == 0 && ldx % 8 == 0 && al16(x) && al16(wk),
                "fs2_conv_gemm_ln_bwd: c_in/ldx must be multiples of 8 and operands 16-B aligned");
  FS2_CHECK_ARG(al16(aux) && al16(xhat) && al16(gamma) && al16(dres) && al16(dy_t) && al16(ws),
                "fs2_conv_gemm_ln_bwd: LayerNorm tensors must be 16-B aligned");
  GldsArgs a{(const u16*)x, ldx, (const u16*)wk, nullptr, 256, rows, seq_len, (int)c_in, 256,
             taps, pad, (int)(taps * c_in), nullptr, aux ? FS2_EPI_ADD_AUX : 0, aux, 256, 0, 0, 1,
             1, lens, 1, 0.f, 1.f, nullptr, 0.f};
  a.ln_gamma = gamma;
  a.ln_out = dres;
  a.ln_out_t = (u16*)dy_t;
  a.ln_xhat = const_cast<float*>(xhat);
  a.ln_rstd = const_cast<float*>(rstd);
  a.ln_seed = p_in > 0.f ? seed : nullptr;
  a.ln_site = site_in;
  a.ln_p = p_in;
  a.ln_mode = 1;
  a.ln_dres_add = dres_add;
  a.ln_part = ws;
  a.ln_nblk = (rows + 31) / 32;
  a.tiles_m = (int)((rows + 63) / 64);
  a.tiles_n = 1;
  const unsigned grid = (unsigned)a.tiles_m;
  if (c_in % 64 == 0 && taps == 1 && g_tune[FS2_TUNE_NT_K1] >= 0)
    conv_gemm_nt_glds<64, 256, 2, true, false, true><<<grid, 256, 0, st>>>(a);
  else if (c_in % 64 == 0) conv_gemm_nt_glds<64, 256, 2, true, false><<<grid, 256, 0, st>>>(a);
  else conv_gemm_nt_glds<64, 256, 2, false, false><<<grid, 256, 0, st>>>(a);
  return launch_status("fs2_conv_gemm_ln_bwd");
}

int conv_gemm_glds_launch(const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                          int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                          int pad, const int64_t* lens, const float* bias, int flags,
                          const void* aux, int64_t ld_aux, const VocEpi& ve, hipStream_t st) {
  FS2_CHECK_ARG(c_in % 8 == 0 && ldx % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)wk & 15) == 0,
                "fs2_conv_gemm(bf16): c_in/ldx must be multiples of 8 and operands 16-B aligned");
  const int K = (int)(taps * c_in);
  // LDS stages (scripts/nt_sweep.py): 128x128 tiles run 3-4 blocks per CU and overlap one
  // another's load phase with one stage; the smaller-grid tilings prefetch (2 stages, 4 for
  // 64x64 tiles with K >= 4096, where each block walks 144 k-tiles)
  const int tune = g_tune[FS2_TUNE_GEMM_STAGES];
  const bool uses_aux = flags & (FS2_EPI_ADD_AUX | FS2_EPI_RELU_MASK_AUX);
  const int vec = c_out % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)y % 16) == 0 &&
                  (!(flags & FS2_EPI_BIAS) || ((uintptr_t)bias % 16) == 0) &&
                  (!uses_aux || (ld_aux % 8 == 0 && ((uintptr_t)aux % 16) == 0)) &&
                  (!(flags & FS2_EPI_Y2) || ((uintptr_t)ve.y2 % 16) == 0);
  GldsArgs a{(const u16*)x, ldx, (const u16*)wk, y, ldy, rows, seq_len, (int)c_in, (int)c_out,
             taps, pad, K, bias, flags, aux, ld_aux, 0, 0, vec, 1, lens,
             ve.dil, ve.alpha, ve.scale, (u16*)ve.y2, ve.alpha2};
  const bool tapaligned = c_in % 64 == 0;
  const bool voc = ve.dil != 1 || (flags & (FS2_EPI_LRELU | FS2_EPI_ACC_Y | FS2_EPI_Y2)) || !y;
  const int64_t big = ((rows + 127) / 128) * ((c_out + 127) / 128);
#define FS2_NT(BM_, BN_)                                                  \
  switch (stages) {                                                       \
    case 2: launch_nt<BM_, BN_, 2>(a, tapaligned, voc, st); break;        \
    case 3: launch_nt<BM_, BN_, 3>(a, tapaligned, voc, st); break;        \
    case 4: launch_nt<BM_, BN_, 4>(a, tapaligned, voc, st); break;        \
    default: launch_nt<BM_, BN_, 1>(a, tapaligned, voc, st);              \
  }
  // narrow vocoder convs (HiFi-GAN's 64- and 32-channel stages, millions of rows): the
  // n-tile matches c_out instead of wasting 1/2-3/4 of a 128-wide tile's MFMAs
  if (voc && c_out <= 64 && big >= 128) {
    a.tiles_m = (int)((rows + 127) / 128);
    a.tiles_n = 1;
    a.group = 1;
    const unsigned grid = (unsigned)a.tiles_m;
    if (c_out <= 32) {
      launch_nt<128, 32, 2>(a, tapaligned, true, st);
    } else if (taps > 1 && (taps - 1) * ve.dil <= 64 && tapaligned && seq_len % 128 == 0 &&
               g_tune[FS2_TUNE_NT_HALO] >= 0) {
      if ((taps - 1) * ve.dil > 16) conv_gemm_halo<128, 64, 2, 64, true><<<grid, 256, 0, st>>>(a);
      else conv_gemm_halo<128, 64, 2, 16, true><<<grid, 256, 0, st>>>(a);
    } else {
      launch_nt<128, 64, 2>(a, tapaligned, true, st);
    }
    return launch_status("fs2_conv_gemm(bf16)");
  }
  // tap-register halo kernel (conv_gemm_tapreg): 4-wave 128 x 64 tiles at 3 blocks per CU when
  // they fill at least one round of the CUs (decoder k=9 forward, encoder k=9 forward, PostNet
  // 512 -> 512; smaller grids keep the halo kernels' split-K / 64-row paths).  Alone, decoder
  // k=9 forward: 89.7 us vs 94.4 (128 x 128, 2 blocks per CU) and 97.7 (8-wave 256 x 128, one
  // block per CU): independent blocks overlap one another's barrier / DMA phases.  Narrow
  // outputs (c_out <= 256: the decoder k=9 data gradient, which runs beside the side stream's
  // k=9 weight gradient) take the 128 x 128 tiles at 2 blocks per CU: slower alone (109 vs
  // 87 us) but the dgrad||wgrad pair is 181 vs 191 us and the step 7.40 vs 7.55 ms
  const int trk = g_tune[FS2_TUNE_TAPREG];
  if (trk >= 0 && !voc && tapaligned && (taps == 5 || taps == 9) && pad >= 0 && pad < taps) {
    const int cu = cu_count();
    const int64_t t4 = (rows / 128) * ((c_out + 63) / 64);
    const bool ok4 = seq_len % 128 == 0 && rows % 128 == 0 && rows % seq_len == 0;
    int pick = 0;
    if (trk == 1) pick = ok4 ? 4 : 0;                  // force 128 x 64
    else if (trk == 3) pick = ok4 ? 3 : 0;             // force 128 x 128
    else if (ok4 && c_out <= 256 && t4 >= 3 * cu) pick = 3;
    else if (ok4 && t4 >= 3 * cu) pick = 4;
    if (pick) {
      a.tiles_m = (int)(rows / 128);
      const bool n64 = pick == 4;
      a.tiles_n = (int)((c_out + (n64 ? 63 : 127)) / (n64 ? 64 : 128));
      // tile group: the n-tiles whose weight slice (~1.25 MB) an XCD's resident blocks share in
      // its 4 MB L2 while they walk the m-tiles (all 16 n-tiles of the decoder k=9 forward, a
      // 4.7 MB weight, re-fetched it past L2: 187 MB per launch; groups of 4: 92 -> 85 us)
      if (g_tune[FS2_TUNE_NT_GROUP] > 0) {
        a.group = halo_group(a.tiles_n);
      } else {
        const int64_t slice = (int64_t)(n64 ? 64 : 128) * K * 2;
        int gr = (int)(((int64_t)5 << 18) / slice);
        a.group = gr < 1 ? 1 : gr > a.tiles_n ? a.tiles_n : gr;
      }
      const unsigned grid = (unsigned)(a.tiles_m * a.tiles_n);
      if (pick == 3) {  // 4-wave 128 x 128 tiles, 2 blocks per CU
        if (taps == 9) conv_gemm_tapreg<128, 128, 2, 2, 4, 9, 2, 2><<<grid, 256, 0, st>>>(a);
        else conv_gemm_tapreg<128, 128, 2, 2, 4, 5, 2, 2><<<grid, 256, 0, st>>>(a);
      } else {
        if (taps == 9) conv_gemm_tapreg<128, 64, 2, 2, 4, 9, 2, 3><<<grid, 256, 0, st>>>(a);
        else conv_gemm_tapreg<128, 64, 2, 2, 4, 5, 2, 3><<<grid, 256, 0, st>>>(a);
      }
      return launch_status("fs2_conv_gemm(bf16)");
    }
  }
  // halo kernel (tile sizes as the tap-major choice below: 128x128 / 128x64 / 64x64 by grid;
  // FS2_TUNE_NT_HALO = 2 forces 128 x 128).  Every row tile must lie inside one utterance.
  const bool halo_wide = big >= 512 || g_tune[FS2_TUNE_NT_HALO] == 2;
  int halo_bm = halo_wide || big >= 128 ? 128 : 64;
  // utterances a multiple of 64 rows only (the vocoder's 64-rows-per-frame stage over an odd
  // frame count): 64-row tiles keep the halo kernel (the tap-major one re-stages A per tap)
  if (halo_bm == 128 && seq_len % 128 != 0 && seq_len % 64 == 0) halo_bm = 64;
  // 8-wave 256 x 128 halo tiles, one block per CU with the weight prefetch in flight across the
  // barrier, for the wide forward shapes (c_in <= 256, >= 512 128x128 tiles, T % 256 == 0) that
  // the tap-register kernel does not take (k=9 decoder forward 114 -> 102 us alone,
  // scripts/halo_check.py; FS2_TUNE_NT_HALO 1 disables it).  C_in 512 (the PostNet convs) ran
  // faster on the 4-wave 128 x 128 tiles (78 -> 73 / 84 -> 77 us: the 8-wave grid of 384 blocks
  // is 1.5 rounds of the CUs there).  Deeper rings and 128 x 128 8-wave tiles measured slower.
  if (g_tune[FS2_TUNE_NT_HALO] == 0 && big >= 512 && c_in <= 256 && taps > 1 &&
      (taps - 1) * ve.dil <= 16 && tapaligned && !voc && seq_len % 256 == 0) {
    a.tiles_m = (int)((rows + 255) / 256);
    a.tiles_n = (int)((c_out + 127) / 128);
    a.group = halo_group(a.tiles_n);
    const unsigned grid = (unsigned)(a.tiles_m * a.tiles_n);
    conv_gemm_halo<256, 128, 2, 16, false, 8, true><<<grid, 512, 0, st>>>(a);
    return launch_status("fs2_conv_gemm(bf16)");
  }
  if (taps > 1 && (taps - 1) * ve.dil <= 64 && tapaligned && seq_len % halo_bm == 0 &&
      g_tune[FS2_TUNE_NT_HALO] >= 0) {
    a.tiles_m = (int)((rows + halo_bm - 1) / halo_bm);
    a.tiles_n = (int)((c_out + (halo_wide ? 127 : 63)) / (halo_wide ? 128 : 64));
    a.group = halo_group(a.tiles_n);
    const unsigned grid = (unsigned)(a.tiles_m * a.tiles_n);
    // HX: halo rows beyond the tile, 16 (taps <= 17 undilated: the FFT/PostNet/VP convs) or
    // 64 (dilated vocoder convs; the larger A image leaves 2 blocks per CU)
    const bool hx64 = (taps - 1) * ve.dil > 16;
#define FS2_HALO2(BM_, BN_)                                                                  \
  if (hx64) conv_gemm_halo<BM_, BN_, 2, 64, true><<<grid, 256, 0, st>>>(a);                  \
  else if (voc) conv_gemm_halo<BM_, BN_, 2, 16, true><<<grid, 256, 0, st>>>(a);              \
  else conv_gemm_halo<BM_, BN_, 2, 16, false, 4, true><<<grid, 256, 0, st>>>(a);
    {
      if (halo_wide && halo_bm == 128) {
        const int kz = g_tune[FS2_TUNE_HALO_SPLITK] > 0 ? halo_splitk_count(a, grid, voc, hx64) : 1;
        if (kz > 1) {  // forced split of 128x128 tiles (experiments)
          if (int rc = halo_splitk_slab(a, kz, st)) return rc;
          a.kz = kz;
          conv_gemm_halo<128, 128, 2, 16, false><<<grid * kz, 256, 0, st>>>(a);
          const int64_t n8 = rows * (c_out / 8);
          halo_splitk_reduce<128><<<(unsigned)((n8 + 255) / 256 < 2048 ? (n8 + 255) / 256 : 2048),
                                    256, 0, st>>>(a);
          halo_splitk_done(st);
        } else {
          FS2_HALO2(128, 128)
        }
      } else if (halo_wide) { FS2_HALO2(64, 128) }
      else if (halo_bm == 128) {
        // a forced split count (FS2_TUNE_HALO_SPLITK > 0) also applies to full 128x64 grids
        const int kz = g_tune[FS2_TUNE_HALO_SPLITK] > 0 ? halo_splitk_count(a, grid, voc, hx64) : 1;
        if (kz > 1) {
          if (int rc = halo_splitk_slab(a, kz, st)) return rc;
          a.kz = kz;
          conv_gemm_halo<128, 64, 2, 16, false, 4, true><<<grid * kz, 256, 0, st>>>(a);
          const int64_t n8 = rows * (c_out / 8);
          halo_splitk_reduce<128><<<(unsigned)((n8 + 255) / 256 < 2048 ? (n8 + 255) / 256 : 2048),
                                    256, 0, st>>>(a);
          halo_splitk_done(st);
        } else {
          FS2_HALO2(128, 64)
        }
      } else {
        // under-filled 64x64 grid: with 128-row utterance multiples, 128x64 tiles split kz ways
        // (half the weight-tile re-staging per output row of 64x64 tiles); else 64x64 split
        GldsArgs a2 = a;
        a2.tiles_m = (int)((rows + 127) / 128);
        const unsigned grid2 = (unsigned)(a2.tiles_m * a2.tiles_n);
        const int kz2 = seq_len % 128 == 0 && g_tune[FS2_TUNE_HALO_SPLITK] != -2
                            ? halo_splitk_count(a2, grid2, voc, hx64) : 1;
        const int kz = kz2 > 1 ? 1 : halo_splitk_count(a, grid, voc, hx64);
        if (kz2 > 1) {
          if (int rc = halo_splitk_slab(a2, kz2, st)) return rc;
          a2.kz = kz2;
          conv_gemm_halo<128, 64, 2, 16, false, 4, true><<<grid2 * kz2, 256, 0, st>>>(a2);
          const int64_t n8 = rows * (c_out / 8);
          halo_splitk_reduce<128><<<(unsigned)((n8 + 255) / 256 < 2048 ? (n8 + 255) / 256 : 2048),
                                    256, 0, st>>>(a2);
          halo_splitk_done(st);
        } else if (kz > 1) {
          if (int rc = halo_splitk_slab(a, kz, st)) return rc;
          a.kz = kz;
          conv_gemm_halo<64, 64, 2, 16, false, 4, true><<<grid * kz, 256, 0, st>>>(a);
          const int64_t n8 = rows * (c_out / 8);
          halo_splitk_reduce<64><<<(unsigned)((n8 + 255) / 256 < 2048 ? (n8 + 255) / 256 : 2048),
                                   256, 0, st>>>(a);
          halo_splitk_done(st);
        } else {
          FS2_HALO2(64, 64)
        }
      }
    }
#undef FS2_HALO2
  } else if ((big >= 512 && g_tune[FS2_TUNE_NT_TILE] == 0) || g_tune[FS2_TUNE_NT_TILE] == 1) {
    a.tiles_m = (int)((rows + 127) / 128);
    a.tiles_n = (int)((c_out + 127) / 128);
    const int stages = tune ? tune : 1;
    FS2_NT(128, 128)
  } else if ((big >= 128 && g_tune[FS2_TUNE_NT_TILE] == 0) || g_tune[FS2_TUNE_NT_TILE] == 2) {
    a.tiles_m = (int)((rows + 127) / 128);
    a.tiles_n = (int)((c_out + 63) / 64);
    const int stages = tune ? tune : 2;
    FS2_NT(128, 64)
  } else {
    a.tiles_m = (int)((rows + 63) / 64);
    a.tiles_n = (int)((c_out + 63) / 64);
    const int stages = tune ? tune : (K >= 4096 ? 4 : 2);
    FS2_NT(64, 64)
  }
#undef FS2_NT
  return launch_status("fs2_conv_gemm(bf16)");
}

}  // namespace fs2
