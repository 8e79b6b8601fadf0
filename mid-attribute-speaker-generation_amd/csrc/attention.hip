// Fused key-padding-masked attention for the FFT blocks (d_head = 128), gfx950 MFMA.
//
// Replaces transformer/SubLayers.py:39-52 + Modules.py:14-25 (bmm, /temperature,
// masked_fill(-inf), softmax, bmm) without materialising the (h*B, T, T) score tensor.
// Work unit: one (utterance, head) x 64 queries (forward, dQ) or x 64 keys (dK/dV);
// 4 waves x 16 rows each.  K/V (or Q/dO) tiles of 64 rows are staged in LDS.
//
// The scores are computed *transposed* (S^T = K Q^T): with the MFMA C-layout
// (row = 4*(lane>>4) + reg, col = lane & 15) each lane then owns one query column, so the
// online-softmax statistics are per-lane scalars (two cross-group shuffles per row
// reduction), P^T is already the B operand of O^T += V^T P^T, and O^T's columns are
// queries again: the rescale by exp(m_old - m_new) is a per-lane multiply.  The backward
// uses the same trick (dQ kernel: S^T / dP^T; dK/dV kernel: S / dP with the key on the
// lane).  Padded query tiles are skipped (their outputs are zero-filled; the FFT block
// masks those rows anyway, Layers.py:25); key tiles past the utterance length are never
// loaded.  fp32 path: v_mfma_f32_16x16x4_f32 (exact f32).
#include <math.h>

#include "common.hpp"

namespace fs2 {

constexpr int DH = 128;
constexpr int LDH = DH + 4;  // padded LDS row (floats)
constexpr int QB = 64;       // rows per block (4 waves x 16)

#define MFMA4(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// Cooperative load of a 64 x 128 tile (rows r0.., column offset col0 of row stride ld)
FS2_DEV void load_tile(float* dst, const float* base, int64_t ld, int r0, int nrows, int tid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = tid + i * 256, row = c >> 5, col = (c & 31) * 4;
    const int r = r0 + row;
    f32x4 v = r < nrows ? ld4(base + (int64_t)r * ld + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    st4(&dst[row * LDH + col], v);
  }
}

// per-lane fragment of a 16-row operand: row `r`, d = 32c + 8g + jj for c < 4, jj < 8
FS2_DEV void load_frag(float (&f)[4][8], const float* rowp, int g) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    f32x4 a = ld4(rowp + 32 * c + 8 * g), b = ld4(rowp + 32 * c + 8 * g + 4);
    f[c][0] = a.x; f[c][1] = a.y; f[c][2] = a.z; f[c][3] = a.w;
    f[c][4] = b.x; f[c][5] = b.y; f[c][6] = b.z; f[c][7] = b.w;
  }
}

// acc += (LDS rows row0 + r16) . frag  over d = 128  -> 16x16 tile, rows from LDS
FS2_DEV f32x4 dot_tile(const float* S, int row0, const float (&f)[4][8], int g, int r16) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* p = S + (row0 + r16) * LDH + 8 * g;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    f32x4 a = ld4(p + 32 * c), b = ld4(p + 32 * c + 4);
    acc = MFMA4(a.x, f[c][0], acc); acc = MFMA4(a.y, f[c][1], acc);
    acc = MFMA4(a.z, f[c][2], acc); acc = MFMA4(a.w, f[c][3], acc);
    acc = MFMA4(b.x, f[c][4], acc); acc = MFMA4(b.y, f[c][5], acc);
    acc = MFMA4(b.z, f[c][6], acc); acc = MFMA4(b.w, f[c][7], acc);
  }
  return acc;
}

// acc[ds] (+)= sum over 16 LDS rows (row0 + 4g + r, r < 4 per call step) of
//              LDS[row][16 ds + r16] * w[r]   -> 8 x (16 d x 16 cols)
FS2_DEV void accum_t(f32x4 (&acc)[8], const float* S, int row0, const f32x4& w, int g, int r16) {
#pragma unroll
  for (int ds = 0; ds < 8; ++ds) {
    const float* p = S + (row0 + 4 * g) * LDH + 16 * ds + r16;
    acc[ds] = MFMA4(p[0], w.x, acc[ds]);
    acc[ds] = MFMA4(p[LDH], w.y, acc[ds]);
    acc[ds] = MFMA4(p[2 * LDH], w.z, acc[ds]);
    acc[ds] = MFMA4(p[3 * LDH], w.w, acc[ds]);
  }
}

__global__ __launch_bounds__(256) void attn_fwd_f32(const float* __restrict__ qkv, float* __restrict__ o,
                                                    float* __restrict__ lse,
                                                    const int64_t* __restrict__ lens, int T, int H,
                                                    float scale) {
  __shared__ __attribute__((aligned(16))) float Ks[QB * LDH];
  __shared__ __attribute__((aligned(16))) float Vs[QB * LDH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blockIdx.x * QB;
  const float* base = qkv + (int64_t)b * T * ld;
  float* obase = o + (int64_t)b * T * ldo + h * DH;

  if (q0 >= L) {  // fully padded query tile: outputs are masked downstream; write zeros
    for (int e = tid; e < QB * DH / 4; e += 256) {
      const int row = e / (DH / 4), col = (e % (DH / 4)) * 4, q = q0 + row;
      if (q < T) st4(obase + (int64_t)q * ldo + col, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    if (tid < QB && q0 + tid < T) lse[(int64_t)bh * T + q0 + tid] = 0.f;
    return;
  }

  const int q = q0 + wave * 16 + r16;
  float qf[4][8];
  load_frag(qf, base + (int64_t)min(q, T - 1) * ld + h * DH, g);

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 oacc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (L + QB - 1) / QB;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    load_tile(Ks, base + (int64_t)H * DH + h * DH, ld, kt * QB, T, tid);
    load_tile(Vs, base + 2LL * H * DH + h * DH, ld, kt * QB, T, tid);
    __syncthreads();

    f32x4 s[4];
    float mt = -INFINITY;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = dot_tile(Ks, 16 * st, qf, g, r16);  // S^T[key = 16 st + 4g + r][q = r16]
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
        const float p = __expf(s[st][r] - m_new);
        s[st][r] = p;
        ps += p;
      }
    ps = group4_sum(ps);
    l_run = l_run * alpha + ps;
    m_run = m_new;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) oacc[ds] *= alpha;
    // O^T[d][q] += sum_key V[key][d] P^T[key][q]
#pragma unroll
    for (int st = 0; st < 4; ++st) accum_t(oacc, Vs, 16 * st, s[st], g, r16);
  }

  if (q < T) {
    const float inv = 1.f / l_run;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) st4(obase + (int64_t)q * ldo + 16 * ds + 4 * g, oacc[ds] * inv);
    if (g == 0) lse[(int64_t)bh * T + q] = m_run + __logf(l_run);
  }
}

// delta[bh, q] = sum_d dO[q, h, d] * O[q, h, d]
__global__ void attn_bwd_delta(const float* __restrict__ o, const float* __restrict__ d_o,
                               float* __restrict__ delta, int64_t rows, int T, int H) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= rows * H) return;
  const int64_t r = w / H;
  const int h = (int)(w - r * H);
  const float* po = o + r * H * DH + h * DH + 2 * lane;
  const float* pd = d_o + r * H * DH + h * DH + 2 * lane;
  float s = wave_sum(po[0] * pd[0] + po[1] * pd[1]);
  if (lane == 0) {
    const int64_t b = r / T, q = r - b * T;
    delta[(b * H + h) * T + q] = s;
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dq_f32(const float* __restrict__ qkv,
                                                       const float* __restrict__ d_o,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ delta,
                                                       float* __restrict__ d_qkv,
                                                       const int64_t* __restrict__ lens, int T,
                                                       int H, float scale) {
  __shared__ __attribute__((aligned(16))) float Ks[QB * LDH];
  __shared__ __attribute__((aligned(16))) float Vs[QB * LDH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int q0 = blockIdx.x * QB;
  const float* base = qkv + (int64_t)b * T * ld;
  float* dbase = d_qkv + (int64_t)b * T * ld + h * DH;

  if (q0 >= L) {
    for (int e = tid; e < QB * DH / 4; e += 256) {
      const int row = e / (DH / 4), col = (e % (DH / 4)) * 4, q = q0 + row;
      if (q < T) st4(dbase + (int64_t)q * ld + col, f32x4{0.f, 0.f, 0.f, 0.f});
    }
    return;
  }
  const int q = q0 + wave * 16 + r16;
  const int qc = min(q, T - 1);
  float qf[4][8], df[4][8];
  load_frag(qf, base + (int64_t)qc * ld + h * DH, g);
  load_frag(df, d_o + ((int64_t)b * T + qc) * ldo + h * DH, g);
  const float my_lse = lse[(int64_t)bh * T + qc];
  const float my_delta = delta[(int64_t)bh * T + qc];
  const bool qvalid = q < L;

  f32x4 dq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (L + QB - 1) / QB;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    load_tile(Ks, base + (int64_t)H * DH + h * DH, ld, kt * QB, T, tid);
    load_tile(Vs, base + 2LL * H * DH + h * DH, ld, kt * QB, T, tid);
    __syncthreads();
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      f32x4 s = dot_tile(Ks, 16 * st, qf, g, r16);   // S^T[key][q]
      f32x4 dp = dot_tile(Vs, 16 * st, df, g, r16);  // dP^T[key][q]
      f32x4 dsv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * QB + 16 * st + 4 * g + r;
        const float p = (key < L && qvalid) ? __expf(s[r] * scale - my_lse) : 0.f;
        dsv[r] = p * (dp[r] - my_delta);
      }
      // dQ^T[d][q] += sum_key K[key][d] dS^T[key][q]
      accum_t(dq, Ks, 16 * st, dsv, g, r16);
    }
  }
  if (q < T) {
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) st4(dbase + (int64_t)q * ld + 16 * ds + 4 * g, dq[ds] * scale);
  }
}

__global__ __launch_bounds__(256) void attn_bwd_dkdv_f32(const float* __restrict__ qkv,
                                                         const float* __restrict__ d_o,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta,
                                                         float* __restrict__ d_qkv,
                                                         const int64_t* __restrict__ lens, int T,
                                                         int H, float scale) {
  __shared__ __attribute__((aligned(16))) float Qs[QB * LDH];
  __shared__ __attribute__((aligned(16))) float Ds[QB * LDH];
  __shared__ float lse_s[QB], del_s[QB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, r16 = lane & 15;
  const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
  const int L = (int)min(lens[b], (int64_t)T);
  const int64_t ld = 3LL * H * DH, ldo = (int64_t)H * DH;
  const int k0 = blockIdx.x * QB;
  const float* base = qkv + (int64_t)b * T * ld;
  float* dk_base = d_qkv + (int64_t)b * T * ld + (int64_t)H * DH + h * DH;
  float* dv_base = d_qkv + (int64_t)b * T * ld + 2LL * H * DH + h * DH;

  if (k0 >= L) {
    for (int e = tid; e < QB * DH / 4; e += 256) {
      const int row = e / (DH / 4), col = (e % (DH / 4)) * 4, k = k0 + row;
      if (k < T) {
        st4(dk_base + (int64_t)k * ld + col, f32x4{0.f, 0.f, 0.f, 0.f});
        st4(dv_base + (int64_t)k * ld + col, f32x4{0.f, 0.f, 0.f, 0.f});
      }
    }
    return;
  }
  const int key = k0 + wave * 16 + r16;
  const int kc = min(key, T - 1);
  float kf[4][8], vf[4][8];
  load_frag(kf, base + (int64_t)kc * ld + (int64_t)H * DH + h * DH, g);
  load_frag(vf, base + (int64_t)kc * ld + 2LL * H * DH + h * DH, g);
  const bool kvalid = key < L;

  f32x4 dk[8], dv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nqt = (L + QB - 1) / QB;
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();
    load_tile(Qs, base + h * DH, ld, qt * QB, T, tid);
    load_tile(Ds, d_o + (int64_t)b * T * ldo + h * DH, ldo, qt * QB, T, tid);
    if (tid < QB) {
      const int qq = qt * QB + tid;
      lse_s[tid] = qq < T ? lse[(int64_t)bh * T + qq] : 0.f;
      del_s[tid] = qq < T ? delta[(int64_t)bh * T + qq] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      f32x4 s = dot_tile(Qs, 16 * qs, kf, g, r16);   // S[q = 16 qs + 4g + r][key = r16]
      f32x4 dp = dot_tile(Ds, 16 * qs, vf, g, r16);  // dP[q][key]
      f32x4 p, dsv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * qs + 4 * g + r, qq = qt * QB + ql;
        p[r] = (qq < L && kvalid) ? __expf(s[r] * scale - lse_s[ql]) : 0.f;
        dsv[r] = p[r] * (dp[r] - del_s[ql]);
      }
      accum_t(dv, Ds, 16 * qs, p, g, r16);    // dV^T[d][key] += dO^T[d][q] P[q][key]
      accum_t(dk, Qs, 16 * qs, dsv, g, r16);  // dK^T[d][key] += Q^T[d][q] dS[q][key]
    }
  }
  if (key < T) {
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) {
      st4(dk_base + (int64_t)key * ld + 16 * ds + 4 * g, dk[ds] * scale);
      st4(dv_base + (int64_t)key * ld + 16 * ds + 4 * g, dv[ds]);
    }
  }
}

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_attn_fwd(int dtype, const void* qkv, void* o, float* lse, const int64_t* lens,
                 int64_t batch, int64_t seq_len, int heads, int d_head, float scale, void* stream) {
  FS2_CHECK_ARG(d_head == DH, "fs2_attn_fwd: only d_head = 128 is supported (got %d)", d_head);
  FS2_CHECK_ARG(batch >= 0 && seq_len > 0 && heads > 0, "fs2_attn_fwd: bad shape");
  if (batch == 0) return FS2_OK;
  if (dtype == FS2_BF16)
    return attn_fwd_bf16_launch(qkv, o, lse, lens, batch, seq_len, heads, scale, as_stream(stream));
  if (dtype != FS2_F32) {
    set_error("fs2_attn_fwd: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  dim3 grid((unsigned)((seq_len + QB - 1) / QB), (unsigned)(batch * heads));
  attn_fwd_f32<<<grid, 256, 0, as_stream(stream)>>>((const float*)qkv, (float*)o, lse, lens,
                                                     (int)seq_len, heads, scale);
  return launch_status("fs2_attn_fwd");
}

int64_t fs2_attn_bwd_ws_bytes(int64_t batch, int64_t seq_len, int heads) {
  return batch * seq_len * heads * 4;
}

int fs2_attn_bwd(int dtype, const void* qkv, const void* o, const void* d_o, const float* lse,
                 void* d_qkv, const int64_t* lens, int64_t batch, int64_t seq_len, int heads,
                 int d_head, float scale, float* ws, int64_t ws_bytes, void* stream) {
  FS2_CHECK_ARG(d_head == DH, "fs2_attn_bwd: only d_head = 128 is supported (got %d)", d_head);
  FS2_CHECK_ARG(ws_bytes >= fs2_attn_bwd_ws_bytes(batch, seq_len, heads),
                "fs2_attn_bwd: workspace too small");
  if (batch == 0) return FS2_OK;
  poison(ws, ws_bytes, as_stream(stream));
  if (dtype == FS2_BF16)
    return attn_bwd_bf16_launch(qkv, o, d_o, lse, d_qkv, lens, batch, seq_len, heads, scale, ws,
                                as_stream(stream));
  if (dtype != FS2_F32) {
    set_error("fs2_attn_bwd: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  hipStream_t st = as_stream(stream);
  const int64_t rows = batch * seq_len;
  const int64_t waves = rows * heads;
  attn_bwd_delta<<<(unsigned)((waves * 64 + 255) / 256), 256, 0, st>>>(
      (const float*)o, (const float*)d_o, ws, rows, (int)seq_len, heads);
  dim3 grid((unsigned)((seq_len + QB - 1) / QB), (unsigned)(batch * heads));
  attn_bwd_dq_f32<<<grid, 256, 0, st>>>((const float*)qkv, (const float*)d_o, lse, ws,
                                        (float*)d_qkv, lens, (int)seq_len, heads, scale);
  attn_bwd_dkdv_f32<<<grid, 256, 0, st>>>((const float*)qkv, (const float*)d_o, lse, ws,
                                          (float*)d_qkv, lens, (int)seq_len, heads, scale);
  return launch_status("fs2_attn_bwd");
}

}  // extern "C"
