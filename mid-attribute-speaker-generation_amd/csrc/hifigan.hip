// HiFi-GAN generator pieces that are not a plain implicit-GEMM conv (hifigan/models.py).
//
// The generator's convolutions all run through fs2_conv_gemm_ex (dilated taps, leaky-ReLU
// epilogues, the running multi-receptive-field sum, and a second leaky-ReLU'd compute copy
// of each output for the next conv).  Two pieces live here:
//
// * fs2_convT_weight_prep: ConvTranspose1d(k = 2s, stride s, pad s/2) is a 3-tap conv over
//   the input frames q-1, q, q+1 whose s*c_out output columns are the s output phases of
//   frame q -- the GEMM's row-major (frames, s*c_out) output IS the upsampled
//   (frames*s, c_out) activation, so no scatter and no zero-stuffing exist.  This re-lays
//   the (c_in, c_out, 2s) weight into that (s*c_out, c_in, 3) conv weight (1 of the 3 taps
//   of every phase is zero: 1.5x the minimal MACs, all on MFMA).
// * fs2_vocoder_post: conv_post (c_in -> 1, k = 7) + tanh (+ int16 PCM, utils/model.py:84-88)
//   -- an N = 1 "GEMM" belongs on the vector units: each 256-row block stages its rows and
//   the 3-row halo in LDS (fp32), every thread reduces 7 x c_in products for one sample.
#include <math.h>

#include "common.hpp"

namespace fs2 {

__global__ void convT_prep_kernel(const float* w, const float* bias, int c_in, int c_out, int s,
                                  float* wc, float* bias_c) {
  // one thread per (phase column p = ph*c_out + o, c, jj)
  const int64_t n = (int64_t)s * c_out * c_in * 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int jj = (int)(i % 3);
    const int c = (int)((i / 3) % c_in);
    const int p = (int)(i / (3 * (int64_t)c_in));
    const int ph = p / c_out, o = p - ph * c_out;
    const int tap = s * (1 - jj) + ph + s / 2;  // kernel tap feeding output phase ph from frame q+jj-1
    wc[i] = (tap >= 0 && tap < 2 * s) ? w[((int64_t)c * c_out + o) * (2 * s) + tap] : 0.f;
    if (bias_c && c == 0 && jj == 0) bias_c[p] = bias[o];
  }
}

template <typename T>
FS2_DEV float ldf(const T* p);
template <>
FS2_DEV float ldf<float>(const float* p) { return *p; }
template <>
FS2_DEV float ldf<unsigned short>(const unsigned short* p) {
  return __uint_as_float(((uint32_t)*p) << 16);
}

constexpr int POST_ROWS = 256, POST_TAPS = 7, POST_PAD = 3;

template <typename T>
__global__ __launch_bounds__(256) void vocoder_post_kernel(const T* x, int64_t rows, int64_t T_,
                                                           int c_in, const int64_t* lens,
                                                           const float* w,
                                                           const float* bias, float max_wav,
                                                           float* wav, int16_t* pcm) {
  extern __shared__ float sm[];  // [(POST_ROWS + 6) * c_in] rows, then [7 * c_in] weights
  float* xs = sm;
  float* ws = sm + (POST_ROWS + POST_TAPS - 1) * c_in;
  const int64_t r0 = (int64_t)blockIdx.x * POST_ROWS;
  if (lens) {  // a block of rows past their utterances' valid lengths writes zeros only
    const int64_t r1 = r0 + POST_ROWS < rows ? r0 + POST_ROWS : rows;
    bool all_pad = true;
    for (int64_t b = r0 / T_; b <= (r1 - 1) / T_; ++b) {
      const int64_t lo = b * T_ > r0 ? b * T_ : r0;
      if (lo - b * T_ < lens[b]) {
        all_pad = false;
        break;
      }
    }
    if (all_pad) {
      const int64_t r = r0 + threadIdx.x;
      if (r < rows) {
        wav[r] = 0.f;
        if (pcm) pcm[r] = 0;
      }
      return;
    }
  }
  const int HR = POST_ROWS + POST_TAPS - 1;
  for (int i = threadIdx.x; i < POST_TAPS * c_in; i += blockDim.x) {
    const int j = i / c_in, c = i - j * c_in;
    ws[i] = w[c * POST_TAPS + j];  // reference layout (1, c_in, 7)
  }
  // halo row h holds global row r0 - 3 + h (zero outside its utterance / the matrix); rows of
  // one block may span two utterances, so the check is per (row, output utterance) below
  for (int i = threadIdx.x; i < HR * c_in; i += blockDim.x) {
    const int h = i / c_in, c = i - h * c_in;
    const int64_t r = r0 - POST_PAD + h;
    xs[i] = (r >= 0 && r < rows) ? ldf<T>(x + r * c_in + c) : 0.f;
  }
  __syncthreads();
  const int64_t r = r0 + threadIdx.x;
  if (r >= rows) return;
  const int64_t t = r % T_;  // frame within the utterance
  if (lens && t >= lens[r / T_]) {
    wav[r] = 0.f;
    if (pcm) pcm[r] = 0;
    return;
  }
  float acc = bias[0];
  for (int j = 0; j < POST_TAPS; ++j) {
    const int64_t tt = t + j - POST_PAD;
    if (tt < 0 || tt >= T_) continue;  // zero padding at the utterance edges
    const float* xr = xs + (threadIdx.x + j) * c_in;
    const float* wr = ws + j * c_in;
    for (int c = 0; c < c_in; ++c) acc += wr[c] * xr[c];
  }
  const float v = tanhf(acc);
  wav[r] = v;
  // truncate toward zero to int32, keep the low 16 bits: numpy's float32 -> int16 astype on
  // x86 (so a saturated tanh of exactly 1.0 wraps to -32768 there as here)
  if (pcm) pcm[r] = (int16_t)(uint16_t)(uint32_t)(int32_t)(v * max_wav);
}

}  // namespace fs2

using namespace fs2;

extern "C" {

int fs2_convT_weight_prep(const float* w, const float* bias, int64_t c_in, int64_t c_out,
                          int stride, float* wc, float* bias_c, void* stream) {
  FS2_CHECK_ARG(w && wc && c_in > 0 && c_out > 0 && stride >= 2 && stride % 2 == 0,
                "fs2_convT_weight_prep: needs k = 2*stride, even stride (got stride %d)", stride);
  FS2_CHECK_ARG(!bias_c || bias, "fs2_convT_weight_prep: bias_c without bias");
  const int64_t n = (int64_t)stride * c_out * c_in * 3;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  convT_prep_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(w, bias, (int)c_in, (int)c_out,
                                                                      stride, wc, bias_c);
  return launch_status("fs2_convT_weight_prep");
}

int fs2_vocoder_post(int dtype, const void* x, int64_t rows, int64_t seq_len, int64_t c_in,
                     const int64_t* lens, const float* w, const float* bias, float max_wav_value,
                     float* wav, int16_t* pcm, void* stream) {
  FS2_CHECK_ARG(x && w && bias && wav && rows >= 0 && seq_len > 0 && c_in > 0 && c_in <= 64,
                "fs2_vocoder_post: bad arguments (c_in %lld <= 64)", (long long)c_in);
  if (rows == 0) return FS2_OK;
  const unsigned grid = (unsigned)((rows + POST_ROWS - 1) / POST_ROWS);
  const size_t smem = ((POST_ROWS + POST_TAPS - 1) + POST_TAPS) * c_in * sizeof(float);
  hipStream_t st = as_stream(stream);
  if (dtype == FS2_BF16)
    vocoder_post_kernel<unsigned short><<<grid, 256, smem, st>>>(
        (const unsigned short*)x, rows, seq_len, (int)c_in, lens, w, bias, max_wav_value, wav,
        pcm);
  else if (dtype == FS2_F32)
    vocoder_post_kernel<float><<<grid, 256, smem, st>>>((const float*)x, rows, seq_len, (int)c_in,
                                                        lens, w, bias, max_wav_value, wav, pcm);
  else {
    set_error("fs2_vocoder_post: dtype %d not built", dtype);
    return FS2_ERR_DTYPE;
  }
  return launch_status("fs2_vocoder_post");
}

}  // extern "C"
