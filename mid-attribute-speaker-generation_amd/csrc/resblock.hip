// Fused HiFi-GAN ResBlock1 for the narrow vocoder stages (hifigan/models.py:21-53 with the
// upsample loop of 161-166): one launch runs a whole residual block -- three
// (leaky-ReLU, dilated conv, leaky-ReLU, conv, residual add) pairs -- on a row tile that stays
// in LDS, and folds the stage's running average over the kernel sizes (xs) into its store.
//
// Per-conv launches (fs2_conv_gemm_ex) move every intermediate through HBM: at 32 / 64
// channels a conv has K = 32..704 and is bound by those round trips, not by the MFMA (the
// 32-channel stage ran its 18 convs at ~3 TB/s effective).  Here a block owns R output rows
// plus the block's receptive radius (<= RB_RAD rows each side), loads x once, runs the six
// convs out of LDS (each conv's output region shrinks by its padding) and writes xs (or the
// bf16 leaky-ReLU copy the next upsample reads) once.
//
// LDS (one block per CU): CUR fp32 [WR][C] (the residual stream), two bf16 MFMA operand
// images [WR][64] (CURL = leaky_relu(CUR), T = the first conv's output) with 128-B rows and
// the 16-B chunk swizzle c ^ (row & 7) -- conflict-free fragment reads at every row offset,
// as in the halo conv kernel.  MFMA v_mfma_f32_16x16x32_bf16: A = 16 operand rows x 32
// channels from LDS, B = 32 channels x 16 output channels straight from the prepped weight
// (c_out, taps * c_in) in L2.  Rounding points are the per-conv path's (bf16 operands, fp32
// residual stream and bias / residual adds in the same order); only the MFMA summation order
// differs.  Rows outside the tile's utterance are zero in every conv input (each Conv1d
// zero-pads at the utterance edges), so a tile must lie inside one utterance (T % R == 0).
#include "common.hpp"

namespace fs2 {

namespace {

typedef __bf16 bf16x8r __attribute__((ext_vector_type(8)));
typedef unsigned short u16;

constexpr int RB_WAVES = 8;
constexpr int RB_RAD = 64;  // max receptive radius per side (V1 k=11 chain: 3*5 + 5*(1+3+5) = 60)
constexpr int RB_LD = 64;   // bf16 operand row: 64 elements = 128 B

FS2_DEV u16 to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<u16*>(&b);
}

FS2_DEV float lrelu(float v, float a) { return v >= 0.f ? v : a * v; }

// element (row b, channel c) of a swizzled bf16 operand image
FS2_DEV int op_index(int b, int c) { return b * RB_LD + ((((c >> 3) ^ (b & 7))) << 3) + (c & 7); }

struct ResBlockArgs {
  const float* x;       // (rows, C) fp32 stage input
  const u16* w1[3];     // prepped bf16 (C, k * C): k = j * C + c
  const u16* w2[3];
  const float* b1[3];
  const float* b2[3];
  int dil[3];
  int k;
  float* xs;            // (rows, C) fp32 running sum over the stage's resblocks
  int acc;              // 1: xs = (xs + out) * scale ; 0: xs = out * scale
  float scale;
  int store_xs;
  u16* hc;              // optional (rows, C) bf16 leaky_relu(xs, alpha2)
  float alpha2;
  int64_t rows, T;
  const int64_t* lens;  // optional: tiles of padding rows only store nothing
};

// One conv of the chain: output rows rel in [-E, R + E) (rounded up to 16-row fragments),
// input image `in` (operand rows b = rel + RB_RAD + j*dil - pad), epi(rel, o0, acc[4]) per
// 4 consecutive output channels o0..o0+3 of one row.  Orientation D = W X^T: a wave owns one
// 16-output-channel slice (its weights for every k-step live in registers, loaded once per
// conv -- at most 11 taps x 2 chunks x 4 VGPRs) and walks its share of the 16-row fragments
// RB_FG at a time, the activations read from LDS.  KT (taps) is a template parameter, so the
// k loop is straight-line code the compiler can schedule reads ahead in.
constexpr int RB_FG = 4;  // row fragments per pass (independent accumulators)

// the wave's weight slice for one conv: every k-step's A fragment, loaded once
template <int C, int KT>
FS2_DEV void rb_load_w(const u16* __restrict__ w, int wave, int lane, bf16x8r (&wr)[KT * (C / 32)]) {
  constexpr int NB = C / 16, CH = C / 32;
  const int n = wave % NB;
  const u16* wl = w + (int64_t)(n * 16 + (lane & 15)) * (KT * C) + (lane >> 4) * 8;
#pragma unroll
  for (int st = 0; st < KT * CH; ++st)
    wr[st] = *reinterpret_cast<const bf16x8r*>(wl + (st / CH) * C + (st % CH) * 32);
}

template <int C, int R, int KT, typename Epi>
FS2_DEV void rb_conv(const u16* in, bf16x8r (&wr)[KT * (C / 32)], const u16* w_next, int dil,
                     int pad, int E, int wave, int lane, Epi epi) {
  constexpr int NB = C / 16;            // output-channel slices
  constexpr int WPS = RB_WAVES / NB;    // waves per slice
  constexpr int CH = C / 32;            // 32-channel chunks per tap
  constexpr int STEPS = KT * CH;        // k-steps
  constexpr int NFMAX = (R + 2 * RB_RAD + 15) / 16;
  constexpr int FW = ((NFMAX + WPS - 1) / WPS + RB_FG - 1) / RB_FG * RB_FG;  // frags per wave
  const int NF = (R + 2 * E + 15) / 16;
  const int col = lane & 15, kq = lane >> 4;
  const int part = wave / NB;
  f32x4 acc[FW];
#pragma unroll
  for (int g0 = 0; g0 < FW; g0 += RB_FG) {
    if (part + g0 * WPS < NF) {  // wave-uniform
      int base[RB_FG];
#pragma unroll
      for (int g = 0; g < RB_FG; ++g) {
        acc[g0 + g] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int f = part + (g0 + g) * WPS;
        base[g] = RB_RAD - E - pad + 16 * (f < NF ? f : part) + col;  // past NF: not stored
      }
#pragma unroll
      for (int st = 0; st < STEPS; ++st) {
        const int j = st / CH, ch = (st % CH) * 32 + kq * 8;
#pragma unroll
        for (int g = 0; g < RB_FG; ++g) {
          const bf16x8r x = *reinterpret_cast<const bf16x8r*>(in + op_index(base[g] + j * dil, ch));
          acc[g0 + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[st], x, acc[g0 + g], 0, 0, 0);
        }
      }
    }
  }
  // the next conv's weights fly during this conv's epilogue and the barrier after it
  if (w_next) rb_load_w<C, KT>(w_next, wave, lane, wr);
  // D: column = row (lane & 15), rows = output channels 4 * (lane >> 4) + i: each lane
  // holds 4 consecutive channels of one row -> 16-B / 8-B LDS accesses in the epilogue
#pragma unroll
  for (int g = 0; g < FW; ++g) {
    const int f = part + g * WPS;
    if (f < NF) epi(-E + 16 * f + col, (wave % NB) * 16 + 4 * kq, acc[g]);
  }
}

template <int C, int R, int KT>
__global__ __launch_bounds__(RB_WAVES * 64, 1) void resblock1_fused(ResBlockArgs a) {
  constexpr int WR = R + 2 * RB_RAD + 16;
  constexpr int LDC = C + 4;  // fp32 row stride: +16 B per row spreads a fragment's rows over the banks
  // static LDS: with the same size as dynamic LDS (hipFuncSetAttribute opt-in) an EMPTY launch
  // of this kernel measured 0.5-2.3 ms; declared statically it dispatches in ~5 us
  __shared__ __attribute__((aligned(16))) unsigned char rb_smem[WR * LDC * 4 + 2 * WR * RB_LD * 2];
  float* cur = reinterpret_cast<float*>(rb_smem);              // [WR][LDC]
  u16* curl = reinterpret_cast<u16*>(cur + WR * LDC);          // [WR][64] swizzled
  u16* tb = curl + WR * RB_LD;                                 // [WR][64] swizzled
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // persistent over the row tiles (one block per CU holds all of its LDS): padding tiles cost
  // one test here instead of a block dispatch each
  const int64_t ntiles = a.rows / R;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int64_t m0 = tile * R;
  if (a.lens) {  // the tile lies in one utterance: all padding iff its first row is
    const int64_t u = m0 / a.T;
    if (m0 - u * a.T >= a.lens[u]) continue;
  }
  const int64_t u0 = (m0 / a.T) * a.T, u1 = u0 + a.T < a.rows ? u0 + a.T : a.rows;
  bf16x8r wr[KT * (C / 32)];
  rb_load_w<C, KT>(a.w1[0], wave, lane, wr);  // in flight under the tile load
  auto pack4 = [](float x0, float x1, float x2, float x3) {
    uint2 p;
    p.x = (uint32_t)to_bf16(x0) | ((uint32_t)to_bf16(x1) << 16);
    p.y = (uint32_t)to_bf16(x2) | ((uint32_t)to_bf16(x3) << 16);
    return p;
  };
  // ---- load x rows [m0 - RB_RAD, m0 + R + RB_RAD + 16): CUR and CURL = lrelu(x, 0.1)
  // every global load of the tile is issued before the first LDS store (a rolled loop would
  // wait one HBM round trip per iteration)
  constexpr int V4 = C / 4, NT = RB_WAVES * 64;
  constexpr int LIT = (WR * V4 + NT - 1) / NT;
  float4 xv[LIT];
#pragma unroll
  for (int it = 0; it < LIT; ++it) {
    const int e = tid + it * NT;
    const int b = e / V4, c4 = (e - b * V4) * 4;
    const int64_t g = m0 - RB_RAD + b;
    xv[it] = (e < WR * V4 && g >= u0 && g < u1) ? *reinterpret_cast<const float4*>(a.x + g * C + c4)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int it = 0; it < LIT; ++it) {
    const int e = tid + it * NT;
    if (e < WR * V4) {
      const int b = e / V4, c4 = (e - b * V4) * 4;
      const float4 v = xv[it];
      *reinterpret_cast<float4*>(cur + b * LDC + c4) = v;
      *reinterpret_cast<uint2*>(curl + op_index(b, c4)) =
          pack4(lrelu(v.x, 0.1f), lrelu(v.y, 0.1f), lrelu(v.z, 0.1f), lrelu(v.w, 0.1f));
    }
  }
  __syncthreads();
  int rad = 0;
  for (int m = 0; m < 3; ++m) rad += (a.k - 1) / 2 * a.dil[m] + (a.k - 1) / 2;
  int used = 0;
  for (int m = 0; m < 3; ++m) {
    const int p1 = (a.k - 1) / 2 * a.dil[m];
    used += p1;
    const float* b1 = a.b1[m];
    rb_conv<C, R, KT>(curl, wr, a.w2[m], a.dil[m], p1, rad - used, wave, lane,
                  [&](int rel, int o, f32x4 v) {
                    const int64_t g = m0 + rel;
                    const bool in = g >= u0 && g < u1;
                    const float4 bb = *reinterpret_cast<const float4*>(b1 + o);
                    *reinterpret_cast<uint2*>(tb + op_index(rel + RB_RAD, o)) =
                        in ? pack4(lrelu(v[0] + bb.x, 0.1f), lrelu(v[1] + bb.y, 0.1f),
                                   lrelu(v[2] + bb.z, 0.1f), lrelu(v[3] + bb.w, 0.1f))
                           : make_uint2(0u, 0u);
                  });
    __syncthreads();
    const int p2 = (a.k - 1) / 2;
    used += p2;
    const float* b2 = a.b2[m];
    const bool next = m < 2;
    rb_conv<C, R, KT>(tb, wr, next ? a.w1[m + 1] : nullptr, 1, p2, rad - used, wave, lane,
                  [&](int rel, int o, f32x4 v) {
                    const int64_t g = m0 + rel;
                    const int b = rel + RB_RAD;
                    float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (g >= u0 && g < u1) {
                      const float4 bb = *reinterpret_cast<const float4*>(b2 + o);
                      const float4 r = *reinterpret_cast<const float4*>(cur + b * LDC + o);
                      y = make_float4((v[0] + bb.x) + r.x, (v[1] + bb.y) + r.y,
                                      (v[2] + bb.z) + r.z, (v[3] + bb.w) + r.w);
                    }
                    *reinterpret_cast<float4*>(cur + b * LDC + o) = y;
                    if (next)
                      *reinterpret_cast<uint2*>(curl + op_index(b, o)) =
                          pack4(lrelu(y.x, 0.1f), lrelu(y.y, 0.1f), lrelu(y.z, 0.1f),
                                lrelu(y.w, 0.1f));
                  });
    __syncthreads();
  }
  // ---- store rows [m0, m0 + R): the stage's running sum and / or its leaky-ReLU'd copy
  // (the xs reads of the running sum are all issued first, as in the loader)
  constexpr int SIT = R * V4 / NT;
  static_assert(R * V4 % NT == 0, "store loop");
  float4 ov[SIT];
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    const int e = tid + it * NT, r = e / V4, c4 = (e - r * V4) * 4;
    const int64_t g = m0 + r;
    ov[it] = (a.acc && g < a.rows) ? *reinterpret_cast<const float4*>(a.xs + g * C + c4)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    const int e = tid + it * NT, r = e / V4, c4 = (e - r * V4) * 4;
    const int64_t g = m0 + r;
    if (g >= a.rows) continue;
    float4 v = *reinterpret_cast<const float4*>(cur + (r + RB_RAD) * LDC + c4);
    const float4 o = ov[it];
    v = make_float4((v.x + o.x) * a.scale, (v.y + o.y) * a.scale, (v.z + o.z) * a.scale,
                    (v.w + o.w) * a.scale);
    if (a.store_xs) *reinterpret_cast<float4*>(a.xs + g * C + c4) = v;
    if (a.hc) {
      uint2 p;
      p.x = (uint32_t)to_bf16(lrelu(v.x, a.alpha2)) | ((uint32_t)to_bf16(lrelu(v.y, a.alpha2)) << 16);
      p.y = (uint32_t)to_bf16(lrelu(v.z, a.alpha2)) | ((uint32_t)to_bf16(lrelu(v.w, a.alpha2)) << 16);
      *reinterpret_cast<uint2*>(a.hc + g * C + c4) = p;
    }
  }
  __syncthreads();  // the next tile's loader overwrites CUR
  }
}

template <int C, int R, int KT>
int launch_rb(const ResBlockArgs& a, hipStream_t st) {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
      n_cu = 256;
  }
  const int64_t ntiles = a.rows / R;
  const unsigned grid = (unsigned)(ntiles < n_cu ? ntiles : n_cu);
  resblock1_fused<C, R, KT><<<grid, RB_WAVES * 64, 0, st>>>(a);
  return launch_status("fs2_resblock1_fused");
}

}  // namespace

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_resblock1_supported(int64_t channels, int64_t seq_len, int kernel_size, const int* dil) {
  if (channels != 32 && channels != 64) return 0;
  const int R = channels == 32 ? 256 : 128;
  if (seq_len % R != 0 || kernel_size < 3 || kernel_size > 11 || kernel_size % 2 == 0) return 0;
  int rad = 0;
  for (int m = 0; m < 3; ++m) {
    if (dil[m] < 1) return 0;
    rad += (kernel_size - 1) / 2 * dil[m] + (kernel_size - 1) / 2;
  }
  return rad <= RB_RAD;
}

int fs2_resblock1_fused(const void* x, int64_t rows, int64_t seq_len, int64_t channels,
                        int kernel_size, const int* dil, const void* const* w1,
                        const void* const* w2, const float* const* b1, const float* const* b2,
                        float* xs, int acc, float scale, int store_xs, void* hc, float alpha2,
                        const int64_t* lens, void* stream) {
  FS2_CHECK_ARG(x && w1 && w2 && b1 && b2 && dil && xs && rows >= 0,
                "fs2_resblock1_fused: missing operand");
  FS2_CHECK_ARG(fs2_resblock1_supported(channels, seq_len, kernel_size, dil),
                "fs2_resblock1_fused: channels %lld / seq_len %lld / kernel %d not supported",
                (long long)channels, (long long)seq_len, kernel_size);
  FS2_CHECK_ARG(rows % seq_len == 0, "fs2_resblock1_fused: rows must be whole utterances");
  FS2_CHECK_ARG(store_xs || hc, "fs2_resblock1_fused: no output");
  if (rows == 0) return FS2_OK;
  ResBlockArgs a{};
  a.x = (const float*)x;
  for (int m = 0; m < 3; ++m) {
    FS2_CHECK_ARG(w1[m] && w2[m] && b1[m] && b2[m], "fs2_resblock1_fused: missing conv %d", m);
    a.w1[m] = (const u16*)w1[m];
    a.w2[m] = (const u16*)w2[m];
    a.b1[m] = b1[m];
    a.b2[m] = b2[m];
    a.dil[m] = dil[m];
  }
  a.k = kernel_size;
  a.xs = xs;
  a.acc = acc;
  a.scale = scale;
  a.store_xs = store_xs;
  a.hc = (u16*)hc;
  a.alpha2 = alpha2;
  a.rows = rows;
  a.T = seq_len;
  a.lens = lens;
  hipStream_t st = as_stream(stream);
#define FS2_RB(KT_)                                                                   \
  case KT_:                                                                           \
    return channels == 32 ? launch_rb<32, 256, KT_>(a, st) : launch_rb<64, 128, KT_>(a, st);
  switch (kernel_size) {
    FS2_RB(3)
    FS2_RB(5)
    FS2_RB(7)
    FS2_RB(9)
    FS2_RB(11)
  }
#undef FS2_RB
  set_error("fs2_resblock1_fused: kernel size %d", kernel_size);
  return FS2_ERR_ARG;
}

}  // extern "C"
