// Index-driven kernels of the step: embeddings, bucketized variance embeddings and the
// LengthRegulator.  All are HBM-bound row gathers/scatters: one wave per 256-wide row,
// 4 channels per lane (16-B accesses).
//
// LengthRegulator (model/modules.py:161-194 + utils/tools.py:363-381) without the
// reference's per-phoneme `.item()` loop: a per-utterance inclusive scan of
// max(trunc(d), 0) gives cum[b, i]; output frame t copies phoneme row
// i = #{cum[b, :] <= t} (upper-bound search), frames past the total are zero, the output
// is cropped/padded to out_len while mel_len keeps the uncropped total.  Its backward is a
// contiguous in-order segmented sum per phoneme (no atomics, bitwise reproducible).
#include "common.hpp"

namespace fs2 {

__global__ void encoder_embed(const int64_t* texts, const int64_t* accents, const float* wtab,
                              const float* atab, const float* pos, int64_t rows, int64_t T, int d,
                              float* out, unsigned short* out_t) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int64_t t = r % T;
  const int64_t ti = texts[r], ai = accents[r];
  for (int c = 4 * lane; c < d; c += 256) {
    f32x4 v = ld4(wtab + ti * d + c) + ld4(atab + ai * d + c) + ld4(pos + t * d + c);
    st4(out + r * d + c, v);
    if (out_t) st4_bf16(out_t + r * d + c, v);
  }
}

// Deterministic scatter-add of rows by id (embedding backward), skew-proof.
// Pass 1: block (id, chunk) lists, in row order, the rows of its 1024-row chunk that carry
// `id` (wave ballots + prefix popcounts), then sums them (4 row lanes x 4 channels per
// thread, loads unrolled) into ws[chunk][id].  Pass 2 adds the chunk partials to the table
// row in chunk order.  No atomics; a table row hit by every row costs n/1024 blocks.
constexpr int IA_CHUNK = 1024;

template <typename I>
__global__ __launch_bounds__(256) void index_add_partial(const float* __restrict__ dout,
                                                         const I* __restrict__ ids, int64_t n,
                                                         int d, int n_table, float* ws) {
  __shared__ int list[IA_CHUNK];
  __shared__ int wcnt[4][4];
  __shared__ f32x4 red[4][64];
  const int id = blockIdx.x, chunk = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)chunk * IA_CHUNK;
  bool match[4];
  uint64_t mask[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t r = r0 + wave * 256 + k * 64 + lane;
    match[k] = r < n && (int64_t)ids[r] == id;
    mask[k] = __ballot(match[k]);
    if (lane == 0) wcnt[wave][k] = __popcll(mask[k]);
  }
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wave; ++w)
    for (int k = 0; k < 4; ++k) base += wcnt[w][k];
  int count = 0;
  for (int w = 0; w < 4; ++w)
    for (int k = 0; k < 4; ++k) count += wcnt[w][k];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask[k] >> 32),
                                                __builtin_amdgcn_mbcnt_lo((uint32_t)mask[k], 0));
    if (match[k]) list[base + below] = wave * 256 + k * 64 + lane;
    base += __popcll(mask[k]);
  }
  __syncthreads();
  const int tx = lane, ty = wave;
  for (int c0 = 0; c0 < d; c0 += 256) {
    const int c = c0 + 4 * tx;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (c < d) {
#pragma unroll 8
      for (int i = ty; i < count; i += 4) acc += ld4(dout + (r0 + list[i]) * d + c);
    }
    red[ty][tx] = acc;
    __syncthreads();
    if (ty == 0 && c < d)
      st4(ws + ((int64_t)chunk * n_table + id) * d + c,
          ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void index_add_final(const float* __restrict__ ws, int nchunks,
                                                       int n_table, int d, int64_t pad_idx,
                                                       float* dtab) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // float4 index into the table
  const int64_t total4 = (int64_t)n_table * d / 4;
  if (q >= total4) return;
  const int64_t row = q * 4 / d;
  if (row == pad_idx) return;
  f32x4 s = ld4(ws + q * 4);
  for (int ch = 1; ch < nchunks; ++ch) s += ld4(ws + ((int64_t)ch * n_table * d) + q * 4);
  st4(dtab + q * 4, ld4(dtab + q * 4) + s);
}

template <typename I>
static int index_add_launch(const float* dout, const I* ids, int64_t n, int d, int64_t pad_idx,
                            float* dtab, int64_t n_table, float* ws, hipStream_t st) {
  const int64_t nchunks = (n + IA_CHUNK - 1) / IA_CHUNK;
  dim3 grid((unsigned)n_table, (unsigned)nchunks);
  index_add_partial<I><<<grid, 256, 0, st>>>(dout, ids, n, d, (int)n_table, ws);
  const int64_t total4 = n_table * d / 4;
  index_add_final<<<(unsigned)((total4 + 255) / 256), 256, 0, st>>>(ws, (int)nchunks, (int)n_table,
                                                                    d, pad_idx, dtab);
  return launch_status("index_add");
}

__global__ void rowvec_add(const float* x, const int64_t* ids, const float* tab, int64_t rows,
                           int64_t T, int d, float* out, unsigned short* out_t) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int64_t id = ids[r / T];
  for (int c = 4 * lane; c < d; c += 256) {
    const f32x4 v = ld4(x + r * d + c) + ld4(tab + id * d + c);
    st4(out + r * d + c, v);
    if (out_t) st4_bf16(out_t + r * d + c, v);
  }
}

// dtab[ids[b]] += sum_t dout[b, t].  One block per utterance; the block of the FIRST
// utterance carrying an id sums every utterance with that id (in utterance order, frames in
// 4 row lanes combined in lane order), so repeated speakers need no atomics.
__global__ __launch_bounds__(256) void rowvec_add_bwd(const float* __restrict__ dout,
                                                      const int64_t* __restrict__ ids, int64_t batch,
                                                      int64_t T, int d, float* dtab) {
  __shared__ f32x4 red[4][64];
  __shared__ unsigned char hit[256];
  const int64_t b = blockIdx.x, id = ids[b];
  // the id comparisons are made 256 at a time by the whole block (one serial global load per
  // earlier utterance made the last blocks of a 48-utterance batch the launch's 21-us tail)
  for (int64_t j0 = 0; j0 < b; j0 += 256) {
    const int64_t j = j0 + threadIdx.x;
    if (__syncthreads_or(j < b && ids[j] == id)) return;  // an earlier utterance owns this id
  }
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int c0 = 0; c0 < d; c0 += 256) {
    const int c = c0 + 4 * tx;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int64_t q0 = b; q0 < batch; q0 += 256) {  // same rows, same order as one by one
      __syncthreads();
      hit[threadIdx.x] = q0 + threadIdx.x < batch && ids[q0 + threadIdx.x] == id;
      __syncthreads();
      const int64_t nq = batch - q0 < 256 ? batch - q0 : 256;
      if (c < d)
        for (int64_t u = 0; u < nq; ++u) {
          if (!hit[u]) continue;
          const int64_t bb = q0 + u;
          for (int64_t t = ty; t < T; t += 4) acc += ld4(dout + (bb * T + t) * d + c);
        }
    }
    red[ty][tx] = acc;
    __syncthreads();
    if (ty == 0 && c < d)
      st4(dtab + id * d + c, ld4(dtab + id * d + c) + (((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]));
    __syncthreads();
  }
}

// torch.bucketize(v, bins, right=False) = number of bins strictly below v
template <typename V>
FS2_DEV int lower_bound(const float* bins, int n, V v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((V)bins[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

template <typename V>
__global__ void bucket_embed(const float* x, const V* vals, const float* bins, int nb,
                             const float* tab, int64_t rows, int d, float* out, int32_t* idx,
                             unsigned short* out_t) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int k = lower_bound<V>(bins, nb, vals[r]);
  if (lane == 0 && idx) idx[r] = k;
  for (int c = 4 * lane; c < d; c += 256) {
    const f32x4 v = ld4(x + r * d + c) + ld4(tab + (int64_t)k * d + c);
    st4(out + r * d + c, v);
    if (out_t) st4_bf16(out_t + r * d + c, v);
  }
}

template <typename V>
__global__ void bucketize_k(const V* vals, const float* bins, int nb, int64_t n, int32_t* idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) idx[i] = lower_bound<V>(bins, nb, vals[i]);
}

// ------------------------------------------------------------------ LengthRegulator
template <typename D>
FS2_DEV int64_t rep_of(D v);
template <>
FS2_DEV int64_t rep_of<int64_t>(int64_t v) { return v > 0 ? v : 0; }
template <>
FS2_DEV int64_t rep_of<float>(float v) {
  const float t = truncf(v);  // python int() truncates toward zero (modules.py:187)
  return t > 0.f ? (int64_t)t : 0;
}

// one block per utterance: cum = inclusive scan of max(trunc(d), 0)
template <typename D>
__global__ void lr_index(const D* dur, int64_t Ts, int32_t* cum, int64_t* mel_len) {
  __shared__ int64_t part[256];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t per = (Ts + 255) / 256;
  const int64_t i0 = tid * per, i1 = i0 + per < Ts ? i0 + per : Ts;
  int64_t s = 0;
  for (int64_t i = i0; i < i1; ++i) s += rep_of<D>(dur[b * Ts + i]);
  part[tid] = s;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {  // Hillis-Steele inclusive scan of 256 partials
    int64_t v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int64_t run = tid > 0 ? part[tid - 1] : 0;
  for (int64_t i = i0; i < i1; ++i) {
    run += rep_of<D>(dur[b * Ts + i]);
    cum[b * Ts + i] = (int32_t)run;
  }
  if (tid == 255) mel_len[b] = part[255];
}

FS2_DEV int upper_bound_i32(const int32_t* a, int n, int64_t t) {  // first i with a[i] > t
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] <= t) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void lr_source(const int32_t* cum, int64_t B, int64_t Ts, int64_t Tout, int32_t* src) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * Tout) return;
  const int64_t b = e / Tout, t = e - b * Tout;
  const int i = upper_bound_i32(cum + b * Ts, (int)Ts, t);
  src[e] = i < Ts ? i : -1;
}

__global__ void lr_expand(const float* x, const int32_t* cum, int64_t B, int64_t Ts, int64_t Tout,
                          int d, const float* pos, float* out, unsigned short* out_t) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= B * Tout) return;
  const int64_t b = r / Tout, t = r - b * Tout;
  const int i = upper_bound_i32(cum + b * Ts, (int)Ts, t);
  for (int c = 4 * lane; c < d; c += 256) {
    f32x4 v = i < Ts ? ld4(x + (b * Ts + i) * d + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (pos) v += ld4(pos + t * d + c);
    st4(out + r * d + c, v);
    if (out_t) st4_bf16(out_t + r * d + c, v);
  }
}

__global__ void lr_expand_bwd(const float* dout, const int32_t* cum, int64_t B, int64_t Ts,
                              int64_t Tout, int d, float* dx) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= B * Ts) return;
  const int64_t b = r / Ts, i = r - b * Ts;
  int64_t t0 = i > 0 ? cum[r - 1] : 0, t1 = cum[r];
  if (t1 > Tout) t1 = Tout;
  for (int c = 4 * lane; c < d; c += 256) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int64_t t = t0; t < t1; ++t) s += ld4(dout + (b * Tout + t) * d + c);
    st4(dx + r * d + c, s);
  }
}

__global__ void embedding_fwd(const int64_t* ids, const float* tab, int64_t n, int d, float* out) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const int64_t id = ids[r];
  for (int c = lane; c < d; c += 64) out[r * d + c] = tab[id * d + c];
}

// mask[b, t] = t >= lens[b]   (utils/tools.py:155-163, true = padding)
__global__ void length_mask(const int64_t* lens, int64_t B, int64_t T, uint8_t* mask) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * T) return;
  const int64_t b = e / T;
  mask[e] = (e - b * T) >= lens[b] ? 1 : 0;
}

static unsigned rows_grid(int64_t rows) { return (unsigned)((rows * 64 + 255) / 256); }

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_encoder_embed_fwd(const int64_t* texts, const int64_t* accents, const float* word_emb,
                          const float* accent_emb, const float* posenc, int64_t batch,
                          int64_t seq_len, int d, float* out, void* out_t, void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_encoder_embed_fwd: d must be a multiple of 4");
  const int64_t rows = batch * seq_len;
  if (rows == 0) return FS2_OK;
  encoder_embed<<<rows_grid(rows), 256, 0, as_stream(stream)>>>(texts, accents, word_emb,
                                                                accent_emb, posenc, rows, seq_len,
                                                                d, out, (unsigned short*)out_t);
  return launch_status("fs2_encoder_embed_fwd");
}

int fs2_embedding_fwd(const int64_t* ids, const float* table, int64_t n, int d, float* out,
                      void* stream) {
  if (n == 0) return FS2_OK;
  embedding_fwd<<<rows_grid(n), 256, 0, as_stream(stream)>>>(ids, table, n, d, out);
  return launch_status("fs2_embedding_fwd");
}

int fs2_length_mask(const int64_t* lens, int64_t batch, int64_t max_len, uint8_t* mask,
                    void* stream) {
  const int64_t n = batch * max_len;
  if (n == 0) return FS2_OK;
  length_mask<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(lens, batch, max_len, mask);
  return launch_status("fs2_length_mask");
}

int64_t fs2_embedding_bwd_ws_bytes(int64_t n, int d, int64_t n_table) {
  return ((n + IA_CHUNK - 1) / IA_CHUNK) * n_table * d * 4;
}

int fs2_embedding_bwd(const float* dout, const int64_t* ids, int64_t n, int d, int padding_idx,
                      float* dtable, int64_t n_table, float* ws, int64_t ws_bytes, void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_embedding_bwd: d must be a multiple of 4");
  FS2_CHECK_ARG(ws_bytes >= fs2_embedding_bwd_ws_bytes(n, d, n_table),
                "fs2_embedding_bwd: workspace too small");
  if (n == 0 || n_table == 0) return FS2_OK;
  poison(ws, ws_bytes, as_stream(stream));
  return index_add_launch<int64_t>(dout, ids, n, d, padding_idx, dtable, n_table, ws,
                                   as_stream(stream));
}

int fs2_rowvec_add_fwd(const float* x, const int64_t* ids, const float* table, int64_t batch,
                       int64_t seq_len, int d, float* out, void* out_t, void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_rowvec_add_fwd: d must be a multiple of 4");
  const int64_t rows = batch * seq_len;
  if (rows == 0) return FS2_OK;
  rowvec_add<<<rows_grid(rows), 256, 0, as_stream(stream)>>>(x, ids, table, rows, seq_len, d, out,
                                                             (unsigned short*)out_t);
  return launch_status("fs2_rowvec_add_fwd");
}

int fs2_rowvec_add_bwd(const float* dout, const int64_t* ids, int64_t batch, int64_t seq_len,
                       int d, float* dtable, void* stream) {
  if (batch == 0) return FS2_OK;
  FS2_CHECK_ARG(d % 4 == 0, "fs2_rowvec_add_bwd: d must be a multiple of 4");
  rowvec_add_bwd<<<(unsigned)batch, 256, 0, as_stream(stream)>>>(dout, ids, batch, seq_len, d, dtable);
  return launch_status("fs2_rowvec_add_bwd");
}

int fs2_bucket_embed_fwd(const float* x, const void* values, int values_dtype, const float* bins,
                         int n_bins, const float* table, int64_t rows, int d, float* out,
                         void* out_t, int32_t* idx, void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_bucket_embed_fwd: d must be a multiple of 4");
  if (rows == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  if (values_dtype == FS2_F32)
    bucket_embed<float><<<rows_grid(rows), 256, 0, st>>>(x, (const float*)values, bins, n_bins,
                                                         table, rows, d, out, idx, (unsigned short*)out_t);
  else if (values_dtype == 2)
    bucket_embed<double><<<rows_grid(rows), 256, 0, st>>>(x, (const double*)values, bins, n_bins,
                                                          table, rows, d, out, idx, (unsigned short*)out_t);
  else {
    set_error("fs2_bucket_embed_fwd: values dtype %d", values_dtype);
    return FS2_ERR_DTYPE;
  }
  return launch_status("fs2_bucket_embed_fwd");
}

int fs2_bucket_embed_bwd(const float* dout, const int32_t* idx, int64_t rows, int d,
                         float* dtable, int64_t n_table, float* ws, int64_t ws_bytes, void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_bucket_embed_bwd: d must be a multiple of 4");
  FS2_CHECK_ARG(ws_bytes >= fs2_embedding_bwd_ws_bytes(rows, d, n_table),
                "fs2_bucket_embed_bwd: workspace too small");
  if (rows == 0 || n_table == 0) return FS2_OK;
  poison(ws, ws_bytes, as_stream(stream));
  return index_add_launch<int32_t>(dout, idx, rows, d, -1, dtable, n_table, ws, as_stream(stream));
}

int fs2_bucketize(const void* values, int values_dtype, const float* bins, int n_bins, int64_t n,
                  int32_t* idx, void* stream) {
  if (n == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)((n + 255) / 256);
  if (values_dtype == FS2_F32)
    bucketize_k<float><<<grid, 256, 0, st>>>((const float*)values, bins, n_bins, n, idx);
  else if (values_dtype == 2)
    bucketize_k<double><<<grid, 256, 0, st>>>((const double*)values, bins, n_bins, n, idx);
  else {
    set_error("fs2_bucketize: values dtype %d", values_dtype);
    return FS2_ERR_DTYPE;
  }
  return launch_status("fs2_bucketize");
}

int fs2_lr_index(const void* durations, int dur_dtype, int64_t batch, int64_t src_len,
                 int32_t* cum, int64_t* mel_len, void* stream) {
  FS2_CHECK_ARG(src_len > 0, "fs2_lr_index: empty phoneme axis");
  if (batch == 0) return FS2_OK;
  hipStream_t st = as_stream(stream);
  if (dur_dtype == 0)
    lr_index<int64_t><<<(unsigned)batch, 256, 0, st>>>((const int64_t*)durations, src_len, cum, mel_len);
  else if (dur_dtype == 1)
    lr_index<float><<<(unsigned)batch, 256, 0, st>>>((const float*)durations, src_len, cum, mel_len);
  else {
    set_error("fs2_lr_index: duration dtype %d", dur_dtype);
    return FS2_ERR_DTYPE;
  }
  return launch_status("fs2_lr_index");
}

// torch.clamp(torch.round(torch.exp(log_d) - 1) * d_control, min=0): round half to even
// (rintf under the default rounding mode); a NaN stays NaN as in torch.clamp
__global__ void duration_round(const float* log_d, int64_t n, float d_control, float* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = rintf(expf(log_d[i]) - 1.f) * d_control;
    out[i] = v < 0.f ? 0.f : v;
  }
}

int fs2_duration_round(const float* log_d, int64_t n, float d_control, float* out, void* stream) {
  if (n == 0) return FS2_OK;
  FS2_CHECK_ARG(n > 0 && log_d && out, "fs2_duration_round: bad arguments");
  duration_round<<<(unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096), 256, 0,
                   as_stream(stream)>>>(log_d, n, d_control, out);
  return launch_status("fs2_duration_round");
}

int fs2_lr_source(const int32_t* cum, int64_t batch, int64_t src_len, int64_t out_len,
                  int32_t* src, void* stream) {
  const int64_t n = batch * out_len;
  if (n == 0) return FS2_OK;
  lr_source<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(cum, batch, src_len,
                                                                        out_len, src);
  return launch_status("fs2_lr_source");
}

int fs2_lr_expand_fwd(const float* x, const int32_t* cum, int64_t batch, int64_t src_len,
                      int64_t out_len, int d, const float* posenc, float* out, void* out_t,
                      void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_lr_expand_fwd: d must be a multiple of 4");
  const int64_t rows = batch * out_len;
  if (rows == 0) return FS2_OK;
  lr_expand<<<rows_grid(rows), 256, 0, as_stream(stream)>>>(x, cum, batch, src_len, out_len, d,
                                                            posenc, out, (unsigned short*)out_t);
  return launch_status("fs2_lr_expand_fwd");
}

int fs2_lr_expand_bwd(const float* dout, const int32_t* cum, int64_t batch, int64_t src_len,
                      int64_t out_len, int d, float* dx, void* stream) {
  FS2_CHECK_ARG(d % 4 == 0, "fs2_lr_expand_bwd: d must be a multiple of 4");
  const int64_t rows = batch * src_len;
  if (rows == 0) return FS2_OK;
  lr_expand_bwd<<<rows_grid(rows), 256, 0, as_stream(stream)>>>(dout, cum, batch, src_len,
                                                                out_len, d, dx);
  return launch_status("fs2_lr_expand_bwd");
}

}  // extern "C"
