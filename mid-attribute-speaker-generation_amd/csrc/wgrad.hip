// Conv1d weight gradient without split-K slabs: conv_wgrad_band.
//
//   dw[o, c, j] += sum_r dy[r, o] * x[r + j - pad, c]        (taps 3 / 5 / 9)
//   db[o]       += sum_r dy[r, o]
//
// Replaces the weight half of ConvolutionBackward for the FFT-block Conv1d FFN
// (transformer/SubLayers.py:85-93), the PostNet convs (transformer/Layers.py:129-137) and the
// variance-predictor convs (model/modules.py:209-250).
//
// The product is a tall reduction: 24,576 rows against a 1,024 x 2,304 output for the decoder
// FFN.  The round-3 kernel split the rows over 8 blocks per output tile and round-tripped eight
// fp32 slabs (72 MB written, 81 MB read back by a reduce launch, for a 9.4 MB result).  Here
// one block owns a 32 (o) x 32 (c) x taps output tile for ALL rows, so the grid is the output
// tiles (256 blocks for the decoder / encoder FFN and the PostNet 512 x 512 convs) and no slab
// exists: the four waves of a block each take every fourth band of rows, hold the whole tile
// in registers (taps x 2 x 2 fragments of v_mfma_f32_16x16x32_bf16), and are summed in a fixed
// order through LDS at the end ((w0 + w2) + (w1 + w3): bitwise reproducible), then added
// straight into dw / db.
//
// Bands.  A band is 32 S consecutive rows inside one utterance (T % 32 S == 0).  Its step s
// (s < S) is the 32-deep MFMA reduction over the rows s + S m (m = 0..31), so tap j of step s
// needs the input rows s + j + S m of the band's halo: halo fragment F[s + j], where F[f] are
// the halo rows f + S m (f < S + taps - 1).  Each halo fragment is read from LDS ONCE and feeds
// every (s, j) with s + j = f -- the tap-register idea of conv_gemm_tapreg applied to the
// reduction dimension (rows may be paired with MFMA k-slots in any order, as long as dy and x
// use the same one).  The dy image stores band row h at position (h mod S) * 32 + h / S and the
// x image halo row h at (h mod S) * RS + h / S, so every fragment is 32 consecutive positions.
// Positions are 64-B rows (32 bf16 columns); the 32-B halves swap at (P >> 2) & 1, which makes
// the ds_read_b64_tr_b16 fragment reads conflict-free at any starting position.
//
// Each wave stages its own bands through its own ST-slot LDS ring by LDS-DMA and waits only for
// its own loads (counted vmcnt): there is no barrier in the main loop.  Rows past an
// utterance's length (lens given) are staged from the zero line, and bands made only of them
// are not visited.  The bias gradient rides on the dy fragments of the blocks of the first c
// tile (an MFMA against a ones fragment).
#include <type_traits>

#include "common.hpp"

namespace fs2 {

typedef unsigned short u16;
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef short s16x4w __attribute__((ext_vector_type(4)));


struct WgradBand {
  const u16* dy;
  int64_t ldy;
  const u16* x;
  int64_t ldx;
  float* dw;
  float* db;
  int64_t M, T;
  int Cin, Cout, pad;
  int tiles_o, tiles_c;
  const int64_t* lens;
};

namespace {

FS2_DEV void wb_glds16(const void* src, u16* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// ds_read_b64_tr_b16 as inline asm (invisible to the compiler's wait-count pass, which would
// otherwise make every read wait for all LDS-DMA in flight); waited for with wb_lgkm<N>
FS2_DEV s16x4w wb_tr16(const u16* p) {
  s16x4w r;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) u16*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
template <int N>
FS2_DEV void wb_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
FS2_DEV void wb_vm(int ahead) {  // at most `ahead` bands of N LDS-DMA instructions in flight
  if (ahead <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * N) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * N) : "memory");
}

}  // namespace

namespace {
template <int N, typename Fn>
FS2_DEV void ww_static_for(Fn&& fn) {
  if constexpr (N > 0) {
    ww_static_for<N - 1>(fn);
    fn(std::integral_constant<int, N - 1>{});
  }
}
// ds_read_b64_tr_b16 at a per-lane base + a compile-time byte offset (the instruction's
// 16-bit immediate): every fragment address of a main loop is one of a few per-lane bases
template <int OFF>
FS2_DEV s16x4w ww_tr(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  s16x4w r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}
FS2_DEV bf16x8w ww_cat(s16x4w lo, s16x4w hi) {
  return __builtin_bit_cast(bf16x8w, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
}  // namespace

template <int TAPS, int S, int ST, int W>
__global__ __launch_bounds__(64 * W, W == 8 ? 1 : 2) void conv_wgrad_band(WgradBand a) {
  constexpr int BO = 32, BC = 32, BR = 32 * S, NT = 64 * W;
  constexpr int HR = BR + TAPS - 1, RS = (HR + S - 1) / S, NF = S + TAPS - 1;
  constexpr int PB = 64;                                     // bytes per image position
  constexpr int DPOS = BR, XPOS = (S * RS + 15) / 16 * 16;  // image positions
  constexpr int NQD = DPOS / 16, NQX = XPOS / 16, NQ = NQD + NQX;  // LDS-DMA per band
  constexpr int STAGE_B = (DPOS + XPOS) * PB;                     // bytes per ring slot
  constexpr int RING_B = W * ST * STAGE_B;
  static_assert(RING_B < 65536 + W * ST * STAGE_B, "offsets");
  constexpr int QLD = BC * TAPS + 4;  // fp32 row stride of a dW-layout partial tile
  constexpr int RED_B = (W / 2) * (BO * QLD * 4 + 2 * 64 * 16);  // W / 2 partial tiles + bias
  static_assert(TAPS * 16 * 64 <= BO * QLD, "native partial fits a region");
  constexpr int MAXB = 1024;
  // the band list sits behind the ring, inside the reduction region (used after the main loop):
  // 77 KB in all, two blocks per CU
  constexpr int LIST_B = RING_B + 4 * MAXB + 64;
  constexpr int SMEM_B = LIST_B > RED_B ? LIST_B : RED_B;
  constexpr int LOOK = 2;  // halo fragments read ahead of their MFMAs
  static_assert(NQ * (ST - 2 > 0 ? ST - 2 : 1) <= 63 && ST == 2, "vmcnt bookkeeping / the unrolled ring");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM_B];
  short* blist = reinterpret_cast<short*>(smem + RING_B);          // band index
  short* brem = reinterpret_cast<short*>(smem + RING_B + 2 * MAXB);  // its rows below the length
  int* wcnt = reinterpret_cast<int*>(smem + RING_B + 4 * MAXB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r16 = lane & 15;

  // output tile: XCD-contiguous runs, c fastest (an XCD's blocks share their dy columns in L2)
  const int nwg = a.tiles_o * a.tiles_c;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int to = wg / a.tiles_c, tc = wg - to * a.tiles_c;
  const int o0 = to * BO, c0 = tc * BC;

  // bands holding a real row, in row order, with their rows below the length (the launcher
  // admits lens only with nb_all <= MAXB).  In LDS: a global load of lens in the main loop
  // would make the compiler wait vmcnt(0) there, draining the LDS-DMA ring every band.
  const int nbu = (int)(a.T / BR);
  const int nb_all = (int)(a.M / BR);
  const bool use_list = a.lens != nullptr;
  int nb = nb_all;
  if (use_list) {
    int total = 0;
    for (int k0 = 0; k0 < nb_all; k0 += NT) {
      const int k = k0 + tid;
      bool v = false;
      int rem = 0;
      if (k < nb_all) {
        const int b = k / nbu;
        const int64_t r = a.lens[b] - (int64_t)(k - b * nbu) * BR;
        v = r > 0;
        rem = r < BR ? (int)r : BR;
      }
      const uint64_t mask = __ballot(v);
      if (lane == 0) wcnt[wave] = __popcll(mask);
      __syncthreads();
      int before = total;
      for (int w = 0; w < wave; ++w) before += wcnt[w];
      const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
      if (v) {
        blist[before + below] = (short)k;
        brem[before + below] = (short)rem;
      }
      for (int w = 0; w < W; ++w) total += wcnt[w];
      __syncthreads();
    }
    nb = total;
  }
  const int nbw = nb > wave ? (nb - wave + W - 1) / W : 0;  // this wave: bands wave + W i

  // the 32-B halves of position P swap at (P >> 2) & 1 (16-B chunk index ^ 2)
  auto swz = [](int P) { return ((P >> 2) & 1) << 1; };
  // LDS-DMA through buffer descriptors: dy from row 0, x from row -pad; the band's first row
  // rides in the scalar offset
  const auto dy_rs = buf_rsrc(a.dy, a.M * a.ldy * 2);
  const auto x_rs = buf_rsrc(a.x - (int64_t)a.pad * a.ldx, (a.M + a.pad) * a.ldx * 2);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)smem;
  unsigned char* ring = smem + wave * ST * STAGE_B;

  auto issue = [&](int i, int slot) {
    const int kk = wave + W * i;
    const int k = __builtin_amdgcn_readfirstlane(use_list ? (int)blist[kk] : kk);
    const int rem = __builtin_amdgcn_readfirstlane(use_list ? (int)brem[kk] : BR);
    const int b = k / nbu, t0 = (k - b * nbu) * BR;
    const int64_t r0 = (int64_t)b * a.T + t0;
    unsigned char* St = ring + slot * STAGE_B;
    // per-lane offsets recomputed here (an opaque lane id keeps them out of the registers
    // held across the loop)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int lpos = ln >> 2, lch = ln & 3;
#pragma unroll
    for (int qi = 0; qi < NQD; ++qi) {
      const int P = qi * 16 + lpos;
      const int h = (P & 31) * S + (P >> 5);
      const int col = o0 + ((lch ^ swz(P)) << 3);
      const bool ok = h < rem && col < a.Cout;
      glds16_buf(dy_rs, St + qi * 16 * PB, ok ? (uint32_t)((h * a.ldy + col) * 2) : kOOB,
                 (uint32_t)(r0 * a.ldy * 2));
    }
#pragma unroll
    for (int qi = 0; qi < NQX; ++qi) {
      const int P = qi * 16 + lpos;
      const int h = (P % RS) * S + P / RS;
      const int col = c0 + ((lch ^ swz(P)) << 3);
      const int t = t0 - a.pad + h;
      const bool ok = P < S * RS && h < HR && t >= 0 && t < (int)a.T && col < a.Cin;
      glds16_buf(x_rs, St + (DPOS + qi * 16) * PB, ok ? (uint32_t)((h * a.ldx + col) * 2) : kOOB,
                 (uint32_t)(r0 * a.ldx * 2));
    }
  };

  f32x4 acc[TAPS][2][2], accb[2];
#pragma unroll
  for (int j = 0; j < TAPS; ++j)
#pragma unroll
    for (int io = 0; io < 2; ++io)
#pragma unroll
      for (int ic = 0; ic < 2; ++ic) acc[j][io][ic] = f32x4{0.f, 0.f, 0.f, 0.f};
  accb[0] = accb[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.db != nullptr && tc == 0;  // block-uniform
  bf16x8w ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;

  // per-lane fragment bases: the fragment of 32 positions from pb (rows pb + 4g + q and + 16),
  // 16 columns at col0, reads base(pb mod 8, col0) + (pb - pb mod 8) PB (+ 16 PB): the swizzle
  // of position pb + L depends on pb only through pb mod 8
  const int L = 4 * g + q;
  auto fbase = [&](int r, int col0, int img) -> uint32_t {
    const int lc = (col0 >> 3) + (p >> 1);
    return lds0 + (uint32_t)(wave * ST * STAGE_B + img + (r + L) * PB + ((lc ^ swz(r + L)) << 4) +
                             ((p & 1) << 3));
  };
  uint32_t bA0 = fbase(0, 0, 0), bA1 = fbase(0, 16, 0);
  uint32_t bF[8][2];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int ic = 0; ic < 2; ++ic) bF[r][ic] = fbase(r, ic * 16, DPOS * PB);

  auto compute = [&](auto slot_c) {
    constexpr int SO = decltype(slot_c)::value * STAGE_B;
    bf16x8w A[S][2], F[LOOK + 1][2];
    ww_static_for<S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      A[s][0] = ww_cat(ww_tr<SO + s * 32 * PB>(bA0), ww_tr<SO + (s * 32 + 16) * PB>(bA0));
      A[s][1] = ww_cat(ww_tr<SO + s * 32 * PB>(bA1), ww_tr<SO + (s * 32 + 16) * PB>(bA1));
    });
    auto rdF = [&](auto fc, bf16x8w (&dst)[2]) {
      constexpr int f = decltype(fc)::value;
      constexpr int pb = (f % S) * RS + f / S, r = pb & 7, off = SO + (pb - r) * PB;
      dst[0] = ww_cat(ww_tr<off>(bF[r][0]), ww_tr<off + 16 * PB>(bF[r][0]));
      dst[1] = ww_cat(ww_tr<off>(bF[r][1]), ww_tr<off + 16 * PB>(bF[r][1]));
    };
    ww_static_for<LOOK>([&](auto fc) { rdF(fc, F[decltype(fc)::value]); });
    ww_static_for<NF>([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      if constexpr (f + LOOK < NF) rdF(std::integral_constant<int, f + LOOK>{}, F[(f + LOOK) % (LOOK + 1)]);
      constexpr int younger = (NF - 1 - f < LOOK ? NF - 1 - f : LOOK) * 4;
      wb_lgkm<younger>();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = f - s;
        if (j < 0 || j >= TAPS) continue;
#pragma unroll
        for (int io = 0; io < 2; ++io)
#pragma unroll
          for (int ic = 0; ic < 2; ++ic)
            acc[j][io][ic] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[s][io], F[f % (LOOK + 1)][ic],
                                                                     acc[j][io][ic], 0, 0, 0);
        if (j == 0 && do_bias) {
#pragma unroll
          for (int io = 0; io < 2; ++io)
            accb[io] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[s][io], ones, accb[io], 0, 0, 0);
        }
      }
    });
  };

  // per-wave 2-slot ring, no barrier: wait for this wave's band i (counted vmcnt), refill the
  // other slot with band i + 1, compute band i; the fragment bases step to the other slot
  // after each band (one add per base)
  if (nbw > 0) issue(0, 0);
  int dslot = STAGE_B;
  for (int i = 0; i < nbw; ++i) {
    wb_vm<NQ>(0);
    if (i + 1 < nbw) issue(i + 1, (i + 1) & 1);
    compute(std::integral_constant<int, 0>{});
    bA0 += dslot;
    bA1 += dslot;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      bF[r][0] += dslot;
      bF[r][1] += dslot;
    }
    dslot = -dslot;
  }

  // fixed-order cross-wave sum, a tree through LDS: waves [h, 2h) write their partials, waves
  // [0, h) add them (h = W/2, ..., 2), so wave 0 holds (p0 + p4) + (p2 + p6) and wave 1 the
  // odd pairs (W = 8); both write their sums in the dw layout ([o][c][j], row stride QLD) and
  // every thread adds the two into dw / db
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* Q = reinterpret_cast<float*>(smem);
  f32x4* QB = reinterpret_cast<f32x4*>(Q + (W / 2) * BO * QLD);  // [W / 2][2 io][64 lanes]
#pragma unroll
  for (int h = W / 2; h >= 2; h /= 2) {
    if (wave >= h && wave < 2 * h) {
      f32x4* dst = reinterpret_cast<f32x4*>(Q + (wave - h) * BO * QLD);
#pragma unroll
      for (int j = 0; j < TAPS; ++j)
#pragma unroll
        for (int io = 0; io < 2; ++io)
#pragma unroll
          for (int ic = 0; ic < 2; ++ic) dst[((j * 2 + io) * 2 + ic) * 64 + lane] = acc[j][io][ic];
      if (do_bias) {
        QB[((wave - h) * 2 + 0) * 64 + lane] = accb[0];
        QB[((wave - h) * 2 + 1) * 64 + lane] = accb[1];
      }
    }
    __syncthreads();
    if (wave < h) {
      const f32x4* src = reinterpret_cast<const f32x4*>(Q + wave * BO * QLD);
#pragma unroll
      for (int j = 0; j < TAPS; ++j)
#pragma unroll
        for (int io = 0; io < 2; ++io)
#pragma unroll
          for (int ic = 0; ic < 2; ++ic) acc[j][io][ic] += src[((j * 2 + io) * 2 + ic) * 64 + lane];
      if (do_bias) {
        accb[0] += QB[(wave * 2 + 0) * 64 + lane];
        accb[1] += QB[(wave * 2 + 1) * 64 + lane];
      }
    }
    __syncthreads();
  }
  if (wave < 2) {
    float* dst = Q + wave * BO * QLD;
#pragma unroll
    for (int j = 0; j < TAPS; ++j)
#pragma unroll
      for (int io = 0; io < 2; ++io)
#pragma unroll
        for (int ic = 0; ic < 2; ++ic)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            dst[(io * 16 + 4 * g + r) * QLD + (ic * 16 + r16) * TAPS + j] = acc[j][io][ic][r];
    if (do_bias && r16 == 0) {
#pragma unroll
      for (int io = 0; io < 2; ++io)
#pragma unroll
        for (int r = 0; r < 4; ++r) QB[(wave * 2 + io) * 64 + 4 * g + r][0] = accb[io][r];
    }
  }
  __syncthreads();
  {
    constexpr int V = BC * TAPS / 4;  // f32x4 per output row of the tile
    const int64_t Kp = (int64_t)a.Cin * TAPS;
    const int ncol = (a.Cin - c0 < BC ? a.Cin - c0 : BC) * TAPS;  // valid floats per row
    for (int e = tid; e < BO * V; e += NT) {
      const int o = e / V, v4 = e - o * V;
      if (o0 + o >= a.Cout || 4 * v4 >= ncol) continue;
      const f32x4 s = ld4(Q + o * QLD + 4 * v4) + ld4(Q + BO * QLD + o * QLD + 4 * v4);
      float* d = a.dw + (int64_t)(o0 + o) * Kp + (int64_t)c0 * TAPS + 4 * v4;
      st4(d, ld4(d) + s);
    }
    if (do_bias && tid < BO && o0 + tid < a.Cout) {
      const int io = tid >> 4, gg = (tid & 15) >> 2, r = tid & 3;
      const float b = QB[(0 * 2 + io) * 64 + 4 * gg + r][0] + QB[(1 * 2 + io) * 64 + 4 * gg + r][0];
      a.db[o0 + tid] += b;
    }
  }
}

// ---------------------------------------------------------------- wide-tile weight gradient
// conv_wgrad_wide: the same product on 64 (o) x 64 (c) x taps output tiles, the rows split Z
// ways (Z ~ 256 / tiles) into fp32 slabs summed in split order by one reduce launch.
//
// Why: the band kernel's 32 x 32 tile re-streams every dy column block 8 times and every x column
// block 32 times (684 MB through L2 -> LDS per decoder launch against 63 MB of operands), and
// every one of its waves stages its own operands, so each SIMD's one wave pays 9 LDS-DMA
// instructions and 48 transposed reads per 72 MFMAs with nothing to hide their latency.  A
// 64 x 64 tile halves the staged bytes per MAC (dy 64 + x 72 positions of 128 B per 64-row band
// for 64 x 64 x taps outputs), and the block's eight waves SHARE each staged band: wave (wo, wc)
// owns o 32 wo .. + 31 x c 16 wc .. + 15 x all taps (18 accumulator fragments, ~120 VGPRs: two
// waves per SIMD), the 17 LDS-DMA pieces of a band are spread over the waves, and one barrier
// per band guards a ST-slot ring (17 KB per slot).  The tap-register reduction order of the
// band kernel is kept: step s (s < 2) of a band reduces its rows s + 2 m, tap j of step s needs
// halo fragment F[s + j], and each F[f] is read from LDS once for every (s, j) with s + j = f.
// Per wave and band: 4 dy fragments + 10 x fragments (28 transposed reads) for 36 MFMAs.
//
// Rows: bands of 64 rows inside one utterance (T % 64 == 0); bands made only of rows past an
// utterance's length (lens given) are not visited; split z takes the list's bands
// [z nb / Z, (z + 1) nb / Z) in row order.  Within a block the sum runs over bands in order and
// over the two steps of a band in order; the slabs are summed in split order: bitwise
// reproducible for a given lens.  The bias gradient rides on the dy fragments of the waves with
// wc == 0 in the blocks of the first c tile (MFMA against a ones fragment).  Z == 1 adds the
// tile straight into dw / db.
constexpr int WIDE_MAXB = 2048;  // bands (of 64 rows) listed in LDS when lens are given
struct WgradWide {
  const u16* dy;
  int64_t ldy;
  const u16* x;
  int64_t ldx;
  float* dw;
  float* db;
  float* slab;   // [Z][Cout][Cin taps] (Z > 1)
  float* bslab;  // [Z][Cout] (Z > 1, db given)
  int64_t M, T;
  int Cin, Cout, pad;
  int tiles_o, tiles_c, Z;
  const int64_t* lens;
};


template <int TAPS, int ST>
__global__ __launch_bounds__(512, 4) void conv_wgrad_wide(WgradWide a) {
  constexpr int BO = 64, BC = 64, S = 2, BR = 64, NT = 512;
  constexpr int HR = BR + TAPS - 1, RS = (HR + 1) / 2, NF = S + TAPS - 1;
  constexpr int PB = 128;                                // bytes per image position (64 bf16)
  constexpr int DPOS = BR, XPOS = (2 * RS + 7) / 8 * 8;  // image positions
  constexpr int NPD = DPOS / 8, NPX = XPOS / 8, NP = NPD + NPX;  // 1-KB LDS-DMA pieces per band
  static_assert(NP > 8 && NP <= 24, "piece bookkeeping: 2 or 3 pieces per wave");
  constexpr int STAGE_B = (DPOS + XPOS) * PB;
  constexpr int RING_B = ST * STAGE_B;
  static_assert(RING_B < 65536, "fragment offsets fit the ds immediate");
  constexpr int QLD = BC * TAPS + 4;  // fp32 row stride of a 16-row epilogue slice
  constexpr int EPI_B = 16 * QLD * 4 > 64 * 68 * 4 ? 16 * QLD * 4 : 64 * 68 * 4;
  constexpr int SMEM_B = RING_B > EPI_B ? RING_B : EPI_B;
  constexpr int MAXB = WIDE_MAXB;
  constexpr int LOOK = 1;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM_B + 4 * MAXB + 64];
  short* blist = reinterpret_cast<short*>(smem + SMEM_B);          // band index
  short* brem = reinterpret_cast<short*>(smem + SMEM_B + 2 * MAXB);  // its rows below the length
  int* wcnt = reinterpret_cast<int*>(smem + SMEM_B + 4 * MAXB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wave >> 2, wc = wave & 3;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r16 = lane & 15;

  // block -> (split, o tile, c tile): XCD-contiguous runs, c fastest, then o, then split (an
  // XCD's blocks share the rows of one split)
  // (the bias gradient: Z * ceil(Cout / 64) further blocks after the tiles, see below)
  const int nmain = a.tiles_o * a.tiles_c * a.Z;
  const int nwg = nmain + (a.db != nullptr ? a.Z * a.tiles_o : 0);
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const bool bias_blk = wg >= nmain;  // block-uniform
  const int wb = wg - nmain;
  const int tc = bias_blk ? 0 : wg % a.tiles_c, t2 = bias_blk ? 0 : wg / a.tiles_c;
  const int to = bias_blk ? wb % a.tiles_o : t2 % a.tiles_o;
  const int z = bias_blk ? wb / a.tiles_o : t2 / a.tiles_o;
  const int o0 = to * BO, c0 = tc * BC;

  // bands holding a real row, in row order, with the count of their rows below the length
  // (the launcher admits lens only with nb_all <= MAXB).  Kept in LDS: a global load of lens in
  // the main loop would make the compiler wait vmcnt(0), draining the LDS-DMA ring every band.
  const int nbu = (int)(a.T / BR);
  const int nb_all = (int)(a.M / BR);
  const bool use_list = a.lens != nullptr;
  int nb = nb_all;
  if (use_list) {
    int total = 0;
    for (int k0 = 0; k0 < nb_all; k0 += NT) {
      const int k = k0 + tid;
      bool v = false;
      int rem = 0;
      if (k < nb_all) {
        const int b = k / nbu;
        const int64_t r = a.lens[b] - (int64_t)(k - b * nbu) * BR;
        v = r > 0;
        rem = r < BR ? (int)r : BR;
      }
      const uint64_t mask = __ballot(v);
      if (lane == 0) wcnt[wave] = __popcll(mask);
      __syncthreads();
      int before = total;
      for (int w = 0; w < wave; ++w) before += wcnt[w];
      const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
      if (v) {
        blist[before + below] = (short)k;
        brem[before + below] = (short)rem;
      }
      for (int w = 0; w < 8; ++w) total += wcnt[w];
      __syncthreads();
    }
    nb = total;
  }
  const int kb0 = (int)((int64_t)z * nb / a.Z), kb1 = (int)((int64_t)(z + 1) * nb / a.Z);
  const int nbs = kb1 - kb0;

  if (bias_blk) {
    // db[o0 .. o0 + 63] over this split's bands: thread (row t / 8, 8 columns) loads one 16-B
    // row piece per band (rows past the length skipped), then the 64 row partials of each
    // column are summed in row order through LDS -- kept out of the tile blocks, whose MFMA
    // bias accumulators would cost the registers that keep them at two waves per SIMD
    const int rr = tid >> 3, cc = o0 + (tid & 7) * 8;
    float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < nbs; ++i) {
      const int kk = kb0 + i;
      const int k = use_list ? (int)blist[kk] : kk;
      const int rem = use_list ? (int)brem[kk] : BR;
      const int b = k / nbu, t0 = (k - b * nbu) * BR;
      if (rr < rem && cc < a.Cout) {
        const uint4 v = *reinterpret_cast<const uint4*>(a.dy + ((int64_t)b * a.T + t0 + rr) * a.ldy + cc);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sum[2 * e] += __uint_as_float(w4[e] << 16);
          sum[2 * e + 1] += __uint_as_float(w4[e] & 0xffff0000u);
        }
      }
    }
    float* R = reinterpret_cast<float*>(smem);  // [64 rows][64 + 4 columns]
#pragma unroll
    for (int e = 0; e < 8; ++e) R[rr * 68 + (tid & 7) * 8 + e] = sum[e];
    __syncthreads();
    if (tid < BO && o0 + tid < a.Cout) {
      float acc = 0.f;
      for (int r = 0; r < 64; ++r) acc += R[r * 68 + tid];
      if (a.Z == 1) a.db[o0 + tid] += acc;
      else a.bslab[(int64_t)z * a.Cout + o0 + tid] = acc;
    }
    return;
  }

  // position P's 16-B chunks are XOR-swizzled by ((P >> 1) & 3) << 1: any 8 consecutive
  // positions read as 16-column transposed fragments hit 64 distinct banks per half-wave
  auto swz = [](int P) { return ((P >> 1) & 3) << 1; };
  // LDS-DMA through buffer descriptors: dy from row 0, x from row -pad (the halo's first row);
  // a band's rows ride in the scalar offset, each piece's lanes have a fixed voffset; rows
  // outside the band's valid range select an out-of-range voffset (zeros)
  const auto dy_rs = buf_rsrc(a.dy, a.M * a.ldy * 2);
  const auto x_rs = buf_rsrc(a.x - (int64_t)a.pad * a.ldx, (a.M + a.pad) * a.ldx * 2);
  const int npw = wave + 16 < NP ? 3 : 2;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)smem;

  auto issue = [&](int i, int slot) {
    const int kk = kb0 + i;
    const int k = __builtin_amdgcn_readfirstlane(use_list ? (int)blist[kk] : kk);
    const int rem = __builtin_amdgcn_readfirstlane(use_list ? (int)brem[kk] : BR);
    const int b = k / nbu, t0 = (k - b * nbu) * BR;
    const int64_t r0 = (int64_t)b * a.T + t0;
    unsigned char* St = smem + slot * STAGE_B;
    // the pieces' per-lane rows / offsets are recomputed here (a few VALU) rather than held
    // across the loop: an opaque copy of the lane id keeps the compiler from hoisting them
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int lpos = ln >> 3, lch = ln & 7;
#pragma unroll
    for (int kp = 0; kp < 3; ++kp) {
      if (kp == 2 && npw < 3) break;
      const int pi = wave + 8 * kp;
      if (pi < NPD) {
        const int P = pi * 8 + lpos;
        const int h = (P & 31) * 2 + (P >> 5);
        const int col = o0 + ((lch ^ swz(P)) << 3);
        const bool ok = col < a.Cout && h < rem;
        glds16_buf(dy_rs, St + pi * 8 * PB, ok ? (uint32_t)((h * a.ldy + col) * 2) : kOOB,
                   (uint32_t)(r0 * a.ldy * 2));
      } else {
        const int P = (pi - NPD) * 8 + lpos;
        const int h = (P % RS) * 2 + P / RS;
        const int col = c0 + ((lch ^ swz(P)) << 3);
        const int t = t0 - a.pad + h;
        const bool ok = pi < NP && P < 2 * RS && h < HR && col < a.Cin && t >= 0 && t < (int)a.T;
        glds16_buf(x_rs, St + pi * 8 * PB, ok ? (uint32_t)((h * a.ldx + col) * 2) : kOOB,
                   (uint32_t)(r0 * a.ldx * 2));
      }
    }
  };
  // wait until this wave's pieces of all but the `ahead` youngest issued bands have landed
  auto vm = [&](int ahead) {
    const int n = ahead * npw;
    switch (n) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    }
  };

  f32x4 acc[2][TAPS];
#pragma unroll
  for (int io = 0; io < 2; ++io)
#pragma unroll
    for (int j = 0; j < TAPS; ++j) acc[io][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment bases: a fragment of 32 positions from pb (rows pb + 4g + q and + 16) and
  // 16 columns at col0 reads base(pb mod 8, col0) + (pb - pb mod 8) * PB (+ 16 PB): the swizzle
  // of position pb + L depends on pb only through pb mod 8
  const int L = 4 * g + q;
  auto fbase = [&](int r, int col0, int img) -> uint32_t {
    const int lc = (col0 >> 3) + (p >> 1);
    return lds0 + (uint32_t)(img + (r + L) * PB + ((lc ^ swz(r + L)) << 4) + ((p & 1) << 3));
  };
  const uint32_t bA0 = fbase(0, wo * 32, 0), bA1 = fbase(0, wo * 32 + 16, 0);
  uint32_t bF[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) bF[r] = fbase(r, wc * 16, DPOS * PB);

  auto compute = [&](auto slot_c) {
    constexpr int SO = decltype(slot_c)::value * STAGE_B;
    auto cat = [](s16x4w lo, s16x4w hi) {
      return __builtin_bit_cast(bf16x8w, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    bf16x8w A[S][2], F[LOOK + 1];
    ww_static_for<S>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      A[s][0] = cat(ww_tr<SO + s * 32 * PB>(bA0), ww_tr<SO + (s * 32 + 16) * PB>(bA0));
      A[s][1] = cat(ww_tr<SO + s * 32 * PB>(bA1), ww_tr<SO + (s * 32 + 16) * PB>(bA1));
    });
    auto rdF = [&](auto fc) -> bf16x8w {
      constexpr int f = decltype(fc)::value;
      constexpr int pb = (f % S) * RS + f / S, r = pb & 7, off = SO + (pb - r) * PB;
      return cat(ww_tr<off>(bF[r]), ww_tr<off + 16 * PB>(bF[r]));
    };
    ww_static_for<LOOK>([&](auto fc) { F[decltype(fc)::value] = rdF(fc); });
    ww_static_for<NF>([&](auto fc) {
      constexpr int f = decltype(fc)::value;
      if constexpr (f + LOOK < NF) F[(f + LOOK) % (LOOK + 1)] = rdF(std::integral_constant<int, f + LOOK>{});
      constexpr int younger = (NF - 1 - f < LOOK ? NF - 1 - f : LOOK) * 2;
      wb_lgkm<younger>();
      const bf16x8w Ff = F[f % (LOOK + 1)];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = f - s;
        if (j < 0 || j >= TAPS) continue;
#pragma unroll
        for (int io = 0; io < 2; ++io)
          acc[io][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[s][io], Ff, acc[io][j], 0, 0, 0);
      }
    });
  };

  // ring: ST - 1 bands issued ahead; per band this wave's pieces waited for (counted vmcnt), one
  // raw barrier (every wave's pieces landed AND every wave finished the band whose slot the
  // refill overwrites: its reads were waited for inside compute), refill, MFMAs.  The loop is
  // unrolled by the ring depth so that each band's slot -- and with it every fragment address
  // -- is a compile-time offset.
  static_assert(ST == 3, "the unrolled ring below");
  for (int i = 0; i < ST - 1 && i < nbs; ++i) issue(i, i);
  auto band = [&](auto slot_c, int i) {
    constexpr int SL = decltype(slot_c)::value;
    const int ahead = nbs - 1 - i < ST - 2 ? nbs - 1 - i : ST - 2;
    vm(ahead);
    __builtin_amdgcn_s_barrier();
    if (i + ST - 1 < nbs) issue(i + ST - 1, (SL + ST - 1) % ST);
    compute(slot_c);
  };
  int i = 0;
  for (; i + 3 <= nbs; i += 3) {
    band(std::integral_constant<int, 0>{}, i);
    band(std::integral_constant<int, 1>{}, i + 1);
    band(std::integral_constant<int, 2>{}, i + 2);
  }
  if (i < nbs) band(std::integral_constant<int, 0>{}, i);
  if (i + 1 < nbs) band(std::integral_constant<int, 1>{}, i + 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // epilogue: four 16-row slices of the tile through LDS in the dw layout ([o][c][j]), stored
  // as f32x4 rows (Z == 1: added into dw; else written to this split's slab)
  float* Q = reinterpret_cast<float*>(smem);
  const int64_t Kp = (int64_t)a.Cin * TAPS;
  const int ncol = (a.Cin - c0 < BC ? a.Cin - c0 : BC) * TAPS;  // valid floats per row
  float* dst_base = a.Z == 1 ? a.dw : a.slab + (int64_t)z * a.Cout * Kp;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (wo == (k >> 1)) {
      const int io = k & 1;
#pragma unroll
      for (int j = 0; j < TAPS; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) Q[(4 * g + r) * QLD + (wc * 16 + r16) * TAPS + j] = acc[io][j][r];
    }
    __syncthreads();
    constexpr int V = BC * TAPS / 4;
    for (int e = tid; e < 16 * V; e += NT) {
      const int row = e / V, v4 = e - row * V;
      const int o = o0 + 16 * k + row;
      if (o >= a.Cout || 4 * v4 >= ncol) continue;
      const f32x4 v = ld4(Q + row * QLD + 4 * v4);
      float* d = dst_base + (int64_t)o * Kp + (int64_t)c0 * TAPS + 4 * v4;
      if (a.Z == 1) st4(d, ld4(d) + v);
      else st4(d, v);
    }
    __syncthreads();
  }
}

// kNotEligible: the caller uses the split-K kernels
int conv_wgrad_band_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                           float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out,
                           int taps, int pad, const int64_t* lens, hipStream_t st) {
  const int S = 2, BR = 32 * S;
  if (!(taps == 3 || taps == 5 || taps == 9)) return kNotEligible;
  if (pad < 0 || pad > taps - 1) return kNotEligible;
  if (c_in % 8 || c_out % 8 || ldx % 8 || ldy % 8 || ((uintptr_t)dy & 15) || ((uintptr_t)x & 15))
    return kNotEligible;
  if (seq_len % BR || rows % seq_len || rows / BR > (1 << 15)) return kNotEligible;
  if (lens && rows / BR > 1024) return kNotEligible;  // the kernel's LDS band list
  if (c_in < 32 || c_out < 32) return kNotEligible;
  // taps 3 / 5 with 64-multiple channels (PostNet 512, variance predictors) stay on the split-K
  // halo kernel: step 6.91 vs 6.98 ms with the band kernel there (profiles/r4_ab_experiments.txt)
  if (g_tune[FS2_TUNE_WGRAD_BAND] != 4 && taps != 9 && c_in % 64 == 0 && c_out % 64 == 0 &&
      seq_len % 64 == 0)
    return kNotEligible;
  const int to = (int)((c_out + 31) / 32), tc = (int)((c_in + 31) / 32);
  // grids under half the CUs keep the split-K kernels (the variance predictors' 256 x 256 k=3
  // convs at T = 128: 64 tiles), unless those would be the tap-major kernel (C % 64 != 0: the
  // PostNet's 80-channel convs, 48 tiles -- 26 vs 47 us alone, on 48 CUs)
  const bool halo_ok = c_in % 64 == 0 && c_out % 64 == 0 && seq_len % 64 == 0;
  const int min_tiles = g_tune[FS2_TUNE_WGRAD_BAND] == 3 ? 128 : halo_ok ? 128 : 32;
  if (to * tc < min_tiles) return kNotEligible;
  // f32x4 read-modify-writes of dw: rows of c_in * taps floats, tile columns 32 * taps
  if (((uintptr_t)dw & 15) || (c_in * taps) % 4) return kNotEligible;
  WgradBand a{(const u16*)dy, ldy, (const u16*)x, ldx, dw, db, rows, seq_len, (int)c_in,
              (int)c_out, pad, to, tc, lens};
  const unsigned grid = (unsigned)(to * tc);
  // (4-slot rings and 8-wave blocks measured slower in the step and were removed in round 5:
  // profiles/r4_ab_experiments.txt)
  if (taps == 9) conv_wgrad_band<9, 2, 2, 4><<<grid, 256, 0, st>>>(a);
  else if (taps == 5) conv_wgrad_band<5, 2, 2, 4><<<grid, 256, 0, st>>>(a);
  else conv_wgrad_band<3, 2, 2, 4><<<grid, 256, 0, st>>>(a);
  return launch_status("fs2_conv_wgrad(bf16, band)");
}


// ---------------------------------------------------------------- grouped k = 1 weight gradient
// wgrad_k1_multi: the k = 1 weight gradients of one FFT block -- QKV (768 x 256 + bias), fc
// (256 x 256) and w_2 (256 x 1024) at the decoder shapes, transformer/SubLayers.py:39-55,88 --
// in ONE launch.  Their products are tall reductions (24,576 rows, 0.2 MFLOP per output), so
// they run split-K: a 128 (o) x 128 (c) output tile over a range of rows per block, fp32
// partial tiles into split slabs, summed in split order by ONE reduce launch.  Grouping the
// three GEMMs puts 32 output tiles into the grid instead of 4-16, so the same 256 blocks need 8
// row splits instead of 21-64: a third of the slab bytes, long row loops (48 k-tiles) that
// amortise the prologue / epilogue, and 2 launches per block instead of 6.
// Block: 8 waves; wave w owns the 64 x 64 quadrant w & 3 over rows 32 (w >> 2) .. + 31 of each
// 64-row k-tile (the two row halves of a quadrant are summed through LDS at the end).  The
// k-tiles (dy [64 rows][128 o] and x [64 rows][128 c], 256-B rows, LDS-DMA through buffer
// descriptors) run through a 4-slot ring with three tiles in flight (counted vmcnt, one raw
// barrier per tile).  Transposed fragments (ds_read_b64_tr_b16) with the chunk swizzle
// (R & 7) << 1: a 32-lane read hits 16 distinct bank slots.  The bias gradient rides on the dy
// fragments of the blocks of the first c tile (an MFMA against a ones fragment).
struct K1Job {
  const u16* dy;
  int64_t ldy;
  const u16* x;
  int64_t ldx;
  float* dw;
  float* db;
  float* slab;   // [splits][Cout][Cin]
  float* bslab;  // [splits][Cout] (db != NULL)
  int64_t rps;   // rows per split (multiple of 64)
  int Cin, Cout, tiles_o, tiles_c, splits, begin;  // begin: the job's first block
};
constexpr int K1_MAXJ = 4;
struct K1Multi {
  K1Job job[K1_MAXJ];
  int n, nblocks;
  int64_t M, T;
  const int64_t* lens;
};

namespace {
FS2_DEV bool wb_rows_all_padding(const int64_t* lens, int64_t T, int64_t r0, int64_t r1) {
  int64_t s = r0 / T;
  if (r0 - s * T < lens[s]) return false;
  for (++s; s * T < r1; ++s)
    if (lens[s] > 0) return false;
  return true;
}
}  // namespace

template <int STAGES>
__global__ __launch_bounds__(512, 1) void wgrad_k1_multi(K1Multi m) {
  constexpr int BO = 128, BC = 128, BK = 64, NT = 512;
  constexpr int IMG = BK * 128;     // one operand image: [64 rows][128] bf16 (256-B rows)
  constexpr int STAGE_E = 2 * IMG;  // dy image then x image (32 KB)
  constexpr int EPI_LD = 64 + 4;    // fp32 epilogue rows of a 64 x 64 quadrant
  constexpr int EPI_B = (4 * 64 * EPI_LD + 4 * 64) * 4;
  constexpr int SMEM_B = STAGES * STAGE_E * 2 > EPI_B ? STAGES * STAGE_E * 2 : EPI_B;
  constexpr int MAXKT = 1024;
  __shared__ __attribute__((aligned(1024))) u16 smem[SMEM_B / 2 + MAXKT + 64];
  short* ktl = reinterpret_cast<short*>(smem + SMEM_B / 2);
  int* wcnt = reinterpret_cast<int*>(smem + SMEM_B / 2 + MAXKT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int quad = wave & 3, half = wave >> 2;
  const int qo = (quad >> 1) * 64, qc = (quad & 1) * 64;
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r16 = lane & 15;

  // XCD-contiguous block runs; a job's blocks are split-major, tiles fastest (an XCD's blocks
  // share the rows of dy and x)
  const int nwg = m.nblocks;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  int jb = 0;
#pragma unroll
  for (int j = 1; j < K1_MAXJ; ++j)
    if (j < m.n && wg >= m.job[j].begin) jb = j;
  const K1Job J = m.job[jb];
  const int local = wg - J.begin, tiles = J.tiles_o * J.tiles_c;
  const int z = local / tiles, tile = local - z * tiles;
  const int to = tile / J.tiles_c, tc = tile - to * J.tiles_c;
  const int o0 = to * BO, c0 = tc * BC;
  const int64_t r_begin = (int64_t)z * J.rps;
  int64_t r_end = r_begin + J.rps;
  if (r_end > m.M) r_end = m.M;
  const int nk_all = r_end > r_begin ? (int)((r_end - r_begin + BK - 1) / BK) : 0;
  // ordered list of the split's k-tiles holding a real row
  const bool use_list = m.lens != nullptr && nk_all <= MAXKT;
  int nk = nk_all;
  if (use_list) {
    int total = 0;
    for (int cc0 = 0; cc0 < nk_all; cc0 += NT) {
      const int kt = cc0 + tid;
      bool v = false;
      if (kt < nk_all) {
        const int64_t k0 = r_begin + (int64_t)kt * BK;
        v = !wb_rows_all_padding(m.lens, m.T, k0, k0 + BK < r_end ? k0 + BK : r_end);
      }
      const uint64_t mask = __ballot(v);
      if (lane == 0) wcnt[wave] = __popcll(mask);
      __syncthreads();
      int before = total;
      for (int w = 0; w < wave; ++w) before += wcnt[w];
      const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
      if (v) ktl[before + below] = (short)kt;
      for (int w = 0; w < 8; ++w) total += wcnt[w];
      __syncthreads();
    }
    nk = total;
  }

  // staging: a wave-instruction fills 4 image rows x 256 B; image row R = (2 wave + i) * 4 +
  // lane / 16 (i < 2), physical 16-B chunk lane & 15 holding logical chunk (lane & 15) ^ swz(R).
  // Buffer descriptors over the split's rows (the k-tile advance rides in the scalar offset);
  // chunks past the channel count and rows past the split's end select an out-of-range voffset.
  auto swz = [](int R) { return (R & 7) << 1; };
  const auto dy_rs = buf_rsrc(J.dy + r_begin * J.ldy, (r_end - r_begin) * J.ldy * 2);
  const auto x_rs = buf_rsrc(J.x + r_begin * J.ldx, (r_end - r_begin) * J.ldx * 2);
  int Rl[2];
  uint32_t a_vo[2], b_vo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int R = (wave * 2 + i) * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ swz(R);
    Rl[i] = R;
    a_vo[i] = o0 + lc * 8 < J.Cout ? (uint32_t)((R * J.ldy + o0 + lc * 8) * 2) : kOOB;
    b_vo[i] = c0 + lc * 8 < J.Cin ? (uint32_t)((R * J.ldx + c0 + lc * 8) * 2) : kOOB;
  }
  const int rows = (int)(r_end - r_begin);
  auto issue = [&](int kt, int stage) {
    u16* As = smem + stage * STAGE_E;
    u16* Bs = As + IMG;
    const int tl = __builtin_amdgcn_readfirstlane(use_list ? (int)ktl[kt] : kt);
    const int lim = rows - tl * BK;  // rows of this k-tile inside the split
    const uint32_t sa = (uint32_t)(tl * BK * J.ldy * 2), sb = (uint32_t)(tl * BK * J.ldx * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = Rl[i] < lim;
      glds16_buf(dy_rs, As + (wave * 2 + i) * 4 * 128, ok ? a_vo[i] : kOOB, sa);
      glds16_buf(x_rs, Bs + (wave * 2 + i) * 4 * 128, ok ? b_vo[i] : kOOB, sb);
    }
  };

  f32x4 acc[4][4], accb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool do_bias = J.db != nullptr && tc == 0 && (quad & 1) == 0;  // wave-uniform
  bf16x8w ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (__bf16)1.0f;
  const int rbase = half * 32 + 4 * g + q, sw = swz(rbase);
  auto tr = [&](const u16* img, int col0, int hi) -> s16x4w {
    const int lc = (col0 >> 3) + (p >> 1);
    return wb_tr16(img + (rbase + 16 * hi) * 128 + ((lc ^ sw) << 3) + ((p & 1) << 2));
  };
  auto cat = [](s16x4w lo, s16x4w hi) {
    return __builtin_bit_cast(bf16x8w, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto compute = [&](int stage) {
    const u16* As = smem + stage * STAGE_E;
    const u16* Bs = As + IMG;
    s16x4w ra[4][2], rb[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i][0] = tr(As, qo + i * 16, 0);
      ra[i][1] = tr(As, qo + i * 16, 1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      rb[j][0] = tr(Bs, qc + j * 16, 0);
      rb[j][1] = tr(Bs, qc + j * 16, 1);
    }
    bf16x8w fa[4];
    // c fragment j's MFMAs wait only for the reads up to it (4-bit counter: the 16th read
    // issues once the first has retired, so 6 - 2 j younger reads remain in flight)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j == 0) wb_lgkm<6>();
      else if (j == 1) wb_lgkm<4>();
      else if (j == 2) wb_lgkm<2>();
      else wb_lgkm<0>();
      if (j == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = cat(ra[i][0], ra[i][1]);
      }
      const bf16x8w fb = cat(rb[j][0], rb[j][1]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
    }
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb[i], 0, 0, 0);
    }
  };

  // ring: STAGES - 1 tiles issued ahead; per tile a counted vmcnt (this tile landed, the later
  // ones stay in flight), one raw barrier (every wave's pieces landed AND every wave finished the
  // previous tile, whose slot the refill overwrites), refill, MFMAs
  for (int t = 0; t < STAGES - 1 && t < nk; ++t) issue(t, t);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt < STAGES - 2 ? nk - 1 - kt : STAGES - 2;
    if (ahead >= 2 && STAGES >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    compute(kt % STAGES);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // the two row halves of each quadrant through LDS: half 1 writes, half 0 adds and stores
  float* Cs = reinterpret_cast<float*>(smem);
  float* Bp = Cs + 4 * 64 * EPI_LD;
  if (half == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(quad * 64 + i * 16 + 4 * g + r) * EPI_LD + j * 16 + r16] = acc[i][j][r];
    if (do_bias && r16 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) Bp[quad * 64 + i * 16 + 4 * g + r] = accb[i][r];
    }
  }
  __syncthreads();
  if (half == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(quad * 64 + i * 16 + 4 * g + r) * EPI_LD + j * 16 + r16] += acc[i][j][r];
    if (do_bias && r16 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) Bp[quad * 64 + i * 16 + 4 * g + r] += accb[i][r];
    }
  }
  __syncthreads();
  {
    // 128 x 128 outputs, 32 per thread: row o = tid / 4, 32 consecutive c; quadrant rows
    const int o = tid >> 2, cc = (tid & 3) * 32;
    const int qd = (o >> 6) * 2 + (cc >> 6), ro = o & 63, co = cc & 63;
    float* slab = J.slab + (int64_t)z * J.Cout * J.Cin;
    if (o0 + o < J.Cout) {
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(Cs + (qd * 64 + ro) * EPI_LD + co + 4 * v);
        if (c0 + cc + 4 * v < J.Cin)
          *reinterpret_cast<f32x4*>(slab + (int64_t)(o0 + o) * J.Cin + c0 + cc + 4 * v) = t;
      }
    }
    if (J.db != nullptr && tc == 0 && tid < BO && o0 + tid < J.Cout)
      J.bslab[(int64_t)z * J.Cout + o0 + tid] = Bp[((tid >> 6) * 2) * 64 + (tid & 63)];
  }
}

// dw_j += sum_z slab_j[z] (f32x4 units), db_j += sum_z bslab_j[z]: the splits in order (fixed:
// bitwise reproducible), eight split loads in flight per thread
struct K1Red {
  const float* slab[K1_MAXJ];
  const float* bslab[K1_MAXJ];
  float* dw[K1_MAXJ];
  float* db[K1_MAXJ];
  int64_t u_begin[K1_MAXJ + 1];  // f32x4 units of the weight gradients, per job
  int64_t b_begin[K1_MAXJ + 1];  // bias outputs, per job (after every weight unit)
  int splits[K1_MAXJ];
  int n;
};
__global__ __launch_bounds__(256) void wgrad_k1_multi_reduce(K1Red r) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < r.u_begin[r.n]) {
    int j = 0;
#pragma unroll
    for (int k = 1; k < K1_MAXJ; ++k)
      if (k < r.n && e >= r.u_begin[k]) j = k;
    const int64_t i4 = (e - r.u_begin[j]) * 4, total = (r.u_begin[j + 1] - r.u_begin[j]) * 4;
    const float* s = r.slab[j] + i4;
    const int S = r.splits[j];
    f32x4 acc = ld4(s);
    int zz = 1;
    for (; zz + 7 < S; zz += 8) {
      f32x4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ld4(s + (int64_t)(zz + k) * total);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; zz < S; ++zz) acc += ld4(s + (int64_t)zz * total);
    float* d = r.dw[j] + i4;
    st4(d, ld4(d) + acc);
    return;
  }
  const int64_t eb = e - r.u_begin[r.n];
  if (eb >= r.b_begin[r.n]) return;
  int j = 0;
#pragma unroll
  for (int k = 1; k < K1_MAXJ; ++k)
    if (k < r.n && eb >= r.b_begin[k]) j = k;
  const int64_t o = eb - r.b_begin[j], cout = r.b_begin[j + 1] - r.b_begin[j];
  float acc = 0.f;
  for (int zz = 0; zz < r.splits[j]; ++zz) acc += r.bslab[j][(int64_t)zz * cout + o];
  r.db[j][o] += acc;
}

// jobs: host int64 rows {dy, ldy, x, ldx, dw, db, c_in, c_out}; splits chosen so that the grid
// is about 256 blocks of 128 x 128 tiles
static int k1_multi_splits(int64_t tiles_total, int64_t rows) {
  int64_t s = (256 + tiles_total / 2) / tiles_total;
  if (s > rows / 512) s = rows / 512;  // >= 8 k-tiles per split (small products: fewer slabs)
  return (int)(s < 1 ? 1 : s);
}

int64_t wgrad_k1_multi_ws_floats(const int64_t* jobs, int n, int64_t rows) {
  int64_t tiles = 0;
  for (int j = 0; j < n; ++j) {
    const int64_t cin = jobs[8 * j + 6], cout = jobs[8 * j + 7];
    tiles += ((cout + 127) / 128) * ((cin + 127) / 128);
  }
  const int S = k1_multi_splits(tiles > 0 ? tiles : 1, rows);
  int64_t f = 0;
  for (int j = 0; j < n; ++j) {
    const int64_t cin = jobs[8 * j + 6], cout = jobs[8 * j + 7];
    f += S * cout * cin + (jobs[8 * j + 5] ? S * cout : 0);
    f = (f + 3) / 4 * 4;
  }
  return f;
}

int wgrad_k1_multi_launch(const int64_t* jobs, int n, int64_t rows, int64_t seq_len,
                          const int64_t* lens, float* ws, hipStream_t st) {
  FS2_CHECK_ARG(n >= 1 && n <= K1_MAXJ, "fs2_conv_wgrad_k1_multi: 1..%d jobs", K1_MAXJ);
  int64_t tiles = 0;
  for (int j = 0; j < n; ++j) {
    const int64_t* r = jobs + 8 * j;
    FS2_CHECK_ARG(r[6] % 8 == 0 && r[7] % 8 == 0 && r[1] % 8 == 0 && r[3] % 8 == 0 &&
                      (r[0] & 15) == 0 && (r[2] & 15) == 0 && (r[4] & 15) == 0,
                  "fs2_conv_wgrad_k1_multi: channel counts / strides must be multiples of 8, "
                  "operands 16-B aligned");
    tiles += ((r[7] + 127) / 128) * ((r[6] + 127) / 128);
  }
  const int S = k1_multi_splits(tiles, rows);
  int64_t rps = (rows + S - 1) / S;
  rps = (rps + 63) / 64 * 64;
  for (int j = 0; j < n; ++j) {
    const int64_t ld = jobs[8 * j + 1] > jobs[8 * j + 3] ? jobs[8 * j + 1] : jobs[8 * j + 3];
    FS2_CHECK_ARG((rps + 64) * ld * 2 < ((int64_t)1 << 31),
                  "fs2_conv_wgrad_k1_multi: a row split exceeds 32-bit buffer offsets");
  }
  K1Multi m{};
  K1Red red{};
  m.n = red.n = n;
  m.M = rows;
  m.T = seq_len;
  m.lens = lens;
  int begin = 0;
  int64_t f = 0, ub = 0, bb = 0;
  for (int j = 0; j < n; ++j) {
    const int64_t* r = jobs + 8 * j;
    K1Job& J = m.job[j];
    J.dy = (const u16*)r[0];
    J.ldy = r[1];
    J.x = (const u16*)r[2];
    J.ldx = r[3];
    J.dw = (float*)r[4];
    J.db = (float*)r[5];
    J.Cin = (int)r[6];
    J.Cout = (int)r[7];
    J.tiles_o = (J.Cout + 127) / 128;
    J.tiles_c = (J.Cin + 127) / 128;
    J.splits = S;
    J.rps = rps;
    J.begin = begin;
    begin += J.tiles_o * J.tiles_c * S;
    J.slab = ws + f;
    f += (int64_t)S * J.Cout * J.Cin;
    J.bslab = J.db ? ws + f : nullptr;
    if (J.db) f += (int64_t)S * J.Cout;
    f = (f + 3) / 4 * 4;
    red.slab[j] = J.slab;
    red.bslab[j] = J.bslab;
    red.dw[j] = J.dw;
    red.db[j] = J.db;
    red.splits[j] = S;
    red.u_begin[j] = ub;
    ub += (int64_t)J.Cout * J.Cin / 4;
    red.b_begin[j] = bb;
    bb += J.db ? J.Cout : 0;
  }
  red.u_begin[n] = ub;
  red.b_begin[n] = bb;
  m.nblocks = begin;
  // LDS ring depth (FS2_TUNE_WGRAD_K1M_STAGES, A/B): 0 = 4 slots (128 KB, three k-tiles in flight)
  const int stg = g_tune[FS2_TUNE_WGRAD_K1M_STAGES];
  if (stg == 2) wgrad_k1_multi<2><<<(unsigned)begin, 512, 0, st>>>(m);
  else if (stg == 3) wgrad_k1_multi<3><<<(unsigned)begin, 512, 0, st>>>(m);
  else wgrad_k1_multi<4><<<(unsigned)begin, 512, 0, st>>>(m);
  wgrad_k1_multi_reduce<<<(unsigned)((ub + bb + 255) / 256), 256, 0, st>>>(red);
  return launch_status("fs2_conv_wgrad_k1_multi");
}

// ---------------------------------------------------------------- wide-tile launcher
// split count: about 256 blocks, >= 4 bands per split (FS2_TUNE_WGRAD_WIDE > 1 forces it);
// 0 = not eligible
int conv_wgrad_wide_splits(int64_t rows, int64_t c_in, int64_t c_out, int taps) {
  const int v = g_tune[FS2_TUNE_WGRAD_WIDE];
  if (v < 0) return 0;
  if (!(taps == 3 || taps == 5 || taps == 9)) return 0;
  // default: the channel counts that are not 64-multiples (the PostNet's 80-channel convs:
  // 97.5 -> 36 us alone against the band kernel).  On the 64-multiple shapes it was neutral to
  // slower alone and 0.54 ms/step slower in the step (its 163-VGPR waves, two per SIMD, leave
  // no room for the concurrent data gradient's 244-VGPR waves; profiles/r5_wide_ab.txt)
  if (v == 0 && c_in % 64 == 0 && c_out % 64 == 0) return 0;
  if (rows % 64 || rows / 64 > (1 << 15) || rows < 256) return 0;
  if (c_in % 8 || c_out % 8 || (c_in * taps) % 4) return 0;
  const int64_t tiles = ((c_out + 63) / 64) * ((c_in + 63) / 64);
  const int64_t nb = rows / 64;
  int64_t z = g_tune[FS2_TUNE_WGRAD_WIDE] > 1 ? g_tune[FS2_TUNE_WGRAD_WIDE] : (256 + tiles / 2) / tiles;
  if (z > nb / 4) z = nb / 4;
  if (z > 64) z = 64;
  return (int)(z < 1 ? 1 : z);
}

// slab workspace (floats) the wide kernel needs at this shape (0 when it needs none)
int64_t conv_wgrad_wide_ws_floats(int64_t rows, int64_t c_in, int64_t c_out, int taps) {
  const int z = conv_wgrad_wide_splits(rows, c_in, c_out, taps);
  if (z <= 1) return 0;
  return (int64_t)z * c_out * (c_in * taps + 1);
}

// kNotEligible: the caller uses the other kernels
int conv_wgrad_wide_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                           float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out,
                           int taps, int pad, const int64_t* lens, float* ws, hipStream_t st) {
  const int Z = conv_wgrad_wide_splits(rows, c_in, c_out, taps);
  if (Z < 1 || seq_len <= 0 || seq_len % 64 || rows % seq_len) return kNotEligible;
  if (lens && rows / 64 > WIDE_MAXB) return kNotEligible;
  if (pad < 0 || pad > taps - 1) return kNotEligible;
  if (ldx % 8 || ldy % 8 || ((uintptr_t)dy & 15) || ((uintptr_t)x & 15) || ((uintptr_t)dw & 15))
    return kNotEligible;
  if (Z > 1 && (ws == nullptr || ((uintptr_t)ws & 15))) return kNotEligible;
  const int to = (int)((c_out + 63) / 64), tc = (int)((c_in + 63) / 64);
  const int64_t Kp = c_in * taps;
  float* bslab = (Z > 1 && db) ? ws + (int64_t)Z * c_out * Kp : nullptr;
  WgradWide a{(const u16*)dy, ldy, (const u16*)x, ldx, dw, db, Z > 1 ? ws : nullptr, bslab,
              rows, seq_len, (int)c_in, (int)c_out, pad, to, tc, Z, lens};
  const unsigned grid = (unsigned)(to * tc * Z + (db ? Z * to : 0));
  if (taps == 9) conv_wgrad_wide<9, 3><<<grid, 512, 0, st>>>(a);
  else if (taps == 5) conv_wgrad_wide<5, 3><<<grid, 512, 0, st>>>(a);
  else conv_wgrad_wide<3, 3><<<grid, 512, 0, st>>>(a);
  if (Z > 1) {
    K1Red red{};
    red.n = 1;
    red.slab[0] = ws;
    red.bslab[0] = bslab;
    red.dw[0] = dw;
    red.db[0] = db;
    red.splits[0] = Z;
    red.u_begin[0] = 0;
    red.u_begin[1] = c_out * Kp / 4;
    red.b_begin[0] = 0;
    red.b_begin[1] = db ? c_out : 0;
    const int64_t n = red.u_begin[1] + red.b_begin[1];
    wgrad_k1_multi_reduce<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(red);
  }
  return launch_status("fs2_conv_wgrad(bf16, wide)");
}

}  // namespace fs2
