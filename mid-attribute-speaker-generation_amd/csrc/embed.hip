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

__global__ void embedding_bwd(const float* dout, const int64_t* ids, int64_t n, int d, int pad_idx,
                              float* dtab) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const int64_t id = ids[r];
  if (id == pad_idx) return;
  for (int c = lane; c < d; c += 64) atomicAdd(dtab + id * d + c, dout[r * d + c]);
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

// dtab[ids[b]] += sum_t dout[b, t]   (one block per utterance, thread per channel)
__global__ void rowvec_add_bwd(const float* dout, const int64_t* ids, int64_t T, int d, float* dtab) {
  const int64_t b = blockIdx.x;
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    float s = 0.f;
    for (int64_t t = 0; t < T; ++t) s += dout[(b * T + t) * d + c];
    atomicAdd(dtab + ids[b] * d + c, s);
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

__global__ void bucket_embed_bwd(const float* dout, const int32_t* idx, int64_t rows, int d, float* dtab) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int64_t k = idx[r];
  for (int c = lane; c < d; c += 64) atomicAdd(dtab + k * d + c, dout[r * d + c]);
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

int fs2_embedding_bwd(const float* dout, const int64_t* ids, int64_t n, int d, int padding_idx,
                      float* dtable, void* stream) {
  if (n == 0) return FS2_OK;
  embedding_bwd<<<rows_grid(n), 256, 0, as_stream(stream)>>>(dout, ids, n, d, padding_idx, dtable);
  return launch_status("fs2_embedding_bwd");
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
  rowvec_add_bwd<<<(unsigned)batch, 256, 0, as_stream(stream)>>>(dout, ids, seq_len, d, dtable);
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
                         float* dtable, void* stream) {
  if (rows == 0) return FS2_OK;
  bucket_embed_bwd<<<rows_grid(rows), 256, 0, as_stream(stream)>>>(dout, idx, rows, d, dtable);
  return launch_status("fs2_bucket_embed_bwd");
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
