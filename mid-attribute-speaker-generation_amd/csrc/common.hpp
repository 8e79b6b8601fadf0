// Shared device helpers for the gfx950 kernels of libfs2hip.so.
//
// Wave64 everywhere: lane = threadIdx.x & 63; cross-lane reductions use permlane swaps for
// the 16- / 32-lane exchanges and __shfl_xor below.  Dropout masks come from a counter-based Philox4x32-10 stream keyed by
// (seed, site offset, element index), so backward recomputes the forward mask instead of
// storing it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fs2hip.h"

#define FS2_DEV __device__ __forceinline__


typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace fs2 {

extern int g_tune[FS2_TUNE_COUNT];  // fs2_set_tuning knobs (abi.hip)

// ------------------------------------------------------------------ error reporting
void set_error(const char* fmt, ...);
int launch_status(const char* what);

// Stale-read poisoning (debug, off by default; fs2_debug_poison / FS2_POISON, abi.hip): the
// byte every caller workspace and the library's own reused scratch is filled with before each
// use, or -1.  A kernel that reads scratch it has not written then reads the poison, so two
// runs with different bytes differ instead of depending on what ran before in the process.
int poison_byte();
void poison(void* p, int64_t bytes, hipStream_t st);
// ... and the LDS of every CU filled with it on `st` (no-op when poisoning is off)
void lds_poison(hipStream_t st);
// debug: append a copy of [p, p + bytes) to the snapshot buffer on `st` (fs2_debug_snap)
void snap(const void* p, int64_t bytes, hipStream_t st);

#define FS2_CHECK_ARG(cond, ...)                     \
  do {                                               \
    if (!(cond)) {                                   \
      fs2::set_error(__VA_ARGS__);                   \
      return FS2_ERR_ARG;                            \
    }                                                \
  } while (0)

// in-order column reduction of partial rows (defined in gemm.hip):
//   out[c] (+)= sum_p part[p * cols + c]
int colsum_final_launch(const float* part, int64_t nparts, int64_t cols, float* out, int acc,
                        hipStream_t st);
struct ColsumJob {
  const float* part;
  int64_t nparts, cols;
  float* out;
};
struct ColsumJobs {
  ColsumJob job[6];
  int n, acc;
  void add(const float* part, int64_t nparts, int64_t cols, float* out) {
    job[n++] = ColsumJob{part, nparts, cols, out};
  }
};
int colsum_final_multi_launch(const ColsumJobs& jobs, hipStream_t st);
int colsum_launch(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out, int acc,
                  float* ws, hipStream_t st);

// vocoder extension of the conv epilogue (fs2_conv_gemm_ex): tap dilation, leaky-ReLU slope,
// ACC_Y scale, second output y2 (compute dtype, ld = c_out) with its own slope
struct VocEpi {
  int dil = 1;
  float alpha = 0.f, scale = 1.f;
  void* y2 = nullptr;
  float alpha2 = 0.f;
};

// bf16 launchers (gemm_bf16.hip)
int conv_gemm_bf16_launch(const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                          int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                          int pad, const int64_t* lens, const float* bias, int flags,
                          const void* aux, int64_t ld_aux, const VocEpi& ve, hipStream_t st);
int conv_gemm_ln_glds_launch(const void* x, int64_t ldx, const void* wk, int64_t rows,
                             int64_t seq_len, int64_t c_in, int taps, int pad, const int64_t* lens,
                             const float* bias, const float* res, const float* gamma,
                             const float* beta, float* out, void* out_t, float* xhat, float* rstd,
                             float p_in, const uint64_t* seed, uint64_t site_in, hipStream_t st);
int conv_gemm_lnbwd_glds_launch(const void* x, int64_t ldx, const void* wk, int64_t rows,
                                int64_t seq_len, int64_t c_in, int taps, int pad,
                                const int64_t* lens, const float* aux, const float* xhat,
                                const float* rstd, const float* gamma, float p_in,
                                const uint64_t* seed, uint64_t site_in, float* dres, int dres_add,
                                void* dy_t, float* ws, hipStream_t st);
int conv_gemm_glds_launch(const void* x, int64_t ldx, const void* wk, void* y, int64_t ldy,
                          int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                          int pad, const int64_t* lens, const float* bias, int flags,
                          const void* aux, int64_t ld_aux, const VocEpi& ve, hipStream_t st);
int conv_wgrad_glds_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                           float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out,
                           int taps, int pad, const int64_t* lens, int splits, int tile, float* ws,
                           hipStream_t st);
// returned by a launcher whose kernel does not apply to the shape (the caller tries the next
// one); distinct from every FS2_ERR_* status, so an argument error is never taken for it
constexpr int kNotEligible = 1;
int conv_wgrad_band_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                           float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out,
                           int taps, int pad, const int64_t* lens, hipStream_t st);
int conv_wgrad_wide_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* dw,
                           float* db, int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out,
                           int taps, int pad, const int64_t* lens, float* ws, hipStream_t st);
int64_t conv_wgrad_wide_ws_floats(int64_t rows, int64_t c_in, int64_t c_out, int taps);
int64_t wgrad_k1_multi_ws_floats(const int64_t* jobs, int n, int64_t rows);
int wgrad_k1_multi_launch(const int64_t* jobs, int n, int64_t rows, int64_t seq_len,
                          const int64_t* lens, float* ws, hipStream_t st);
int conv_wgrad_bf16_launch(const void* dy, int64_t ldy, const void* x, int64_t ldx, float* slab,
                           int64_t rows, int64_t seq_len, int64_t c_in, int64_t c_out, int taps,
                           int pad, int splits, hipStream_t st);
int weight_prep_bf16_launch(const float* w, int64_t c_out, int64_t c_in, int taps, void* wf,
                            void* wb, hipStream_t st);
int attn_fwd_bf16_launch(const void* qkv, void* o, float* lse, const int64_t* lens, int64_t batch,
                         int64_t seq_len, int heads, float scale, hipStream_t st);
int attn_bwd_bf16_launch(const void* qkv, const void* o, const void* d_o, const float* lse,
                         void* d_qkv, const int64_t* lens, int64_t batch, int64_t seq_len,
                         int heads, float scale, float* ws, hipStream_t st);
int colsum_bf16_launch(const void* x, int64_t ldx, int64_t rows, int64_t cols, float* out, int acc,
                       float* ws, hipStream_t st);

// ------------------------------------------------------------------ wave reductions
// Exchanges across 16- and 32-lane distances go through v_permlane16_swap / v_permlane32_swap
// (VALU, no LDS round trip as ds_bpermute): with both operands = v the pair {r[0], r[1]} holds
// this lane's value and its partner's (lane ^ 16, lane ^ 32), so the sums / maxima are the
// __shfl_xor ones bitwise (a + b == b + a).
FS2_DEV float x16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
FS2_DEV float x32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
FS2_DEV float x16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
FS2_DEV float x32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
FS2_DEV float wave_sum(float v) {
  v = x32_sum(v);
  v = x16_sum(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
FS2_DEV float wave_max(float v) {
  v = x32_max(v);
  v = x16_max(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce across the 4 lane-groups of 16 (lanes l, l^16, l^32, l^48)
FS2_DEV float group4_sum(float v) { return x32_sum(x16_sum(v)); }
FS2_DEV float group4_max(float v) { return x32_max(x16_max(v)); }

// ------------------------------------------------------------------ LDS-DMA through buffers
// buffer_load_dwordx4 ... lds: the wave's 64 x 16 B land contiguously at lds_wave_base; the
// per-lane byte offset rides in voffset, the wave-uniform rest in soffset; offsets past the
// descriptor's record count read as zeros.
FS2_DEV void glds16_buf(__amdgpu_buffer_rsrc_t r, void* lds_wave_base, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff, 0, 0);
}
// the dword form: lane i's 4 B land at lds_wave_base + 4 i
FS2_DEV void glds4_buf(__amdgpu_buffer_rsrc_t r, void* lds_wave_base, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      r, (__attribute__((address_space(3))) void*)lds_wave_base, 4, voff, soff, 0, 0);
}
// a block-uniform buffer descriptor over [p, p + bytes)
FS2_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                           (int)(bytes < 0x7fffffff ? bytes : 0x7fffffff), 0x00020000);
}
constexpr uint32_t kOOB = 0x80000000u;  // a voffset past every record count: reads zeros

// Wait until at most `ahead` tiles of PER LDS-DMA instructions each are still in flight.
template <int PER>
FS2_DEV void vm_wait_tiles(int ahead) {
  switch (ahead) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory"); break;
  }
}

// ------------------------------------------------------------------ Philox4x32-10
struct u32x4 {
  uint32_t x, y, z, w;
};
FS2_DEV u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product (lo and hi words together) instead of mul_lo + mul_hi
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
FS2_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// Dropout keep-scales.  One Philox-4x32-10 call serves 8 consecutive elements of a site
// (counter = e >> 3): word w gives the 16-bit draws of elements 2w (low half) and 2w+1 (high
// half); an element is dropped when its draw is below round(p * 65536), i.e. with
// probability p to within 2^-17, and kept elements are scaled by 1/(1-p).  Kernels that own
// 8 consecutive elements per lane call dropout8 (one Philox per lane); dropout4 / dropout1
// give the same masks for narrower ownership.
FS2_DEV uint32_t drop_thr16(float p) {
  const float t = p * 65536.f + 0.5f;
  return t >= 65536.f ? 65536u : (uint32_t)t;
}
FS2_DEV void dropout8(uint64_t seed, uint64_t site, uint64_t e0, float p, f32x4& lo, f32x4& hi) {
  if (p <= 0.f) {
    lo = hi = f32x4{1.f, 1.f, 1.f, 1.f};
    return;
  }
  const uint64_t c = e0 >> 3;
  const u32x4 r = philox((uint32_t)c, (uint32_t)(c >> 32), (uint32_t)site, (uint32_t)(site >> 32), seed);
  const uint32_t th = drop_thr16(p);
  const float s = 1.f / (1.f - p);
  lo = f32x4{(r.x & 0xffffu) >= th ? s : 0.f, (r.x >> 16) >= th ? s : 0.f,
             (r.y & 0xffffu) >= th ? s : 0.f, (r.y >> 16) >= th ? s : 0.f};
  hi = f32x4{(r.z & 0xffffu) >= th ? s : 0.f, (r.z >> 16) >= th ? s : 0.f,
             (r.w & 0xffffu) >= th ? s : 0.f, (r.w >> 16) >= th ? s : 0.f};
}
// 4 consecutive elements e0..e0+3 (e0 % 4 == 0): one half of the 8-element group
FS2_DEV f32x4 dropout4(uint64_t seed, uint64_t site, uint64_t e0, float p) {
  if (p <= 0.f) return f32x4{1.f, 1.f, 1.f, 1.f};
  f32x4 lo, hi;
  dropout8(seed, site, e0 & ~7ull, p, lo, hi);
  return (e0 & 4) ? hi : lo;
}
FS2_DEV float dropout1(uint64_t seed, uint64_t site, uint64_t e, float p) {
  if (p <= 0.f) return 1.f;
  f32x4 k = dropout4(seed, site, e & ~3ull, p);
  int j = (int)(e & 3);
  return j == 0 ? k.x : j == 1 ? k.y : j == 2 ? k.z : k.w;
}

// ------------------------------------------------------------------ vector memory
FS2_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
FS2_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

FS2_DEV int div_up(int a, int b) { return (a + b - 1) / b; }

// bf16 compute copies (round to nearest even; gfx950 v_cvt_pk_bf16_f32)
FS2_DEV unsigned short to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<unsigned short*>(&b);
}
FS2_DEV void st4_bf16(void* p, f32x4 v) {
  uint2 w;
  w.x = (uint32_t)to_bf16(v.x) | ((uint32_t)to_bf16(v.y) << 16);
  w.y = (uint32_t)to_bf16(v.z) | ((uint32_t)to_bf16(v.w) << 16);
  *reinterpret_cast<uint2*>(p) = w;
}

FS2_DEV void st8_bf16(void* p, f32x4 a, f32x4 b) {
  uint4 w;
  w.x = (uint32_t)to_bf16(a.x) | ((uint32_t)to_bf16(a.y) << 16);
  w.y = (uint32_t)to_bf16(a.z) | ((uint32_t)to_bf16(a.w) << 16);
  w.z = (uint32_t)to_bf16(b.x) | ((uint32_t)to_bf16(b.y) << 16);
  w.w = (uint32_t)to_bf16(b.z) | ((uint32_t)to_bf16(b.w) << 16);
  *reinterpret_cast<uint4*>(p) = w;
}
// sum over the 32 lanes of a half-wave (every lane gets the half's sum)
FS2_DEV float half_sum(float v) {
  v = x16_sum(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace fs2

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
