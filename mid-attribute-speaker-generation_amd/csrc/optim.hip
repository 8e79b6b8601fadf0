// clip_grad_norm_ + Adam over one flat fp32 parameter buffer (train.py:202,
// model/optimizer.py:10-51, torch.optim.Adam semantics with weight_decay = 0).
//
// Gradient norm: per-block sums of squares (16-B loads, grid-stride), then one block adds
// the partials in a fixed order and writes [norm, clip coefficient] to device memory.
// Adam reads the coefficient from device memory, so clip + step need no host sync and the
// gradient buffer is read exactly once by the update (the clipped gradient is never
// written back).
#include <math.h>

#include "common.hpp"

namespace fs2 {

constexpr int GN_BLOCKS = 1024;

__global__ void sumsq_partial(const float* g, int64_t n, float* part) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 v = ld4(g + 4 * i);
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += blockDim.x) s += g[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// one block of GN_BLOCKS threads: fixed-shape tree over the partials in double
__global__ __launch_bounds__(1024) void norm_final(const float* part, int np, float max_norm,
                                                   float* norm_coef) {
  __shared__ double red[1024];
  double v = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) v += part[i];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int off = blockDim.x / 2; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double s = red[0];
  const float norm = (float)sqrt(s);
  norm_coef[0] = norm;
  const float coef = max_norm / (norm + 1e-6f);
  norm_coef[1] = coef < 1.f ? coef : 1.f;
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, const float* __restrict__ norm_coef,
                            float lr, float b1, float b2, float eps, float bc1, float bc2s,
                            const float* __restrict__ hyper) {
  if (hyper) {  // device-side schedule (fs2_sched_step): [lr, 1 - b1^t, sqrt(1 - b2^t)]
    lr = hyper[0];
    bc1 = hyper[1];
    bc2s = hyper[2];
  }
  const float coef = norm_coef ? norm_coef[1] : 1.f;
  const float step = lr / bc1;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 gv = ld4(g + 4 * i) * coef;
    f32x4 mv = ld4(m + 4 * i), vv = ld4(v + 4 * i), pv = ld4(p + 4 * i);
    mv = b1 * mv + (1.f - b1) * gv;
    vv = b2 * vv + (1.f - b2) * gv * gv;
    f32x4 den;
    den.x = sqrtf(vv.x) / bc2s + eps;
    den.y = sqrtf(vv.y) / bc2s + eps;
    den.z = sqrtf(vv.z) / bc2s + eps;
    den.w = sqrtf(vv.w) / bc2s + eps;
    pv -= step * mv / den;
    st4(m + 4 * i, mv);
    st4(v + 4 * i, vv);
    st4(p + 4 * i, pv);
  }
  if (blockIdx.x == 0)
    for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += blockDim.x) {
      const float gv = g[i] * coef;
      m[i] = b1 * m[i] + (1.f - b1) * gv;
      v[i] = b2 * v[i] + (1.f - b2) * gv * gv;
      p[i] -= step * m[i] / (sqrtf(v[i]) / bc2s + eps);
    }
}

// ScheduledOptim.step_and_update_lr on the device (model/optimizer.py:33-51): one step of
// the counters [lr step, Adam t] and the hyper-parameters [lr, 1 - b1^t, sqrt(1 - b2^t)],
// in double like the host's numpy arithmetic, so a captured graph replays the schedule.
__global__ void sched_step_kernel(int64_t* steps, float* hyper, double init_lr, int64_t warmup,
                                  int64_t a0, int64_t a1, int64_t a2, int n_anneal, double rate,
                                  double b1, double b2, int advance_lr) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t s = advance_lr ? ++steps[0] : steps[0];
  const int64_t t = ++steps[1];
  double sc = fmin(pow((double)s, -0.5), pow((double)warmup, -1.5) * (double)s);
  const int64_t an[3] = {a0, a1, a2};
  for (int i = 0; i < n_anneal && i < 3; ++i)
    if (s > an[i]) sc *= rate;
  hyper[0] = (float)(init_lr * sc);
  hyper[1] = (float)(1.0 - pow(b1, (double)t));
  hyper[2] = (float)sqrt(1.0 - pow(b2, (double)t));
}

// Per-step dropout seed: state = [base, counter, current]; current = splitmix64 of
// (base, ++counter).
__global__ void seed_next_kernel(uint64_t* st) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint64_t c = ++st[1];
  uint64_t z = st[0] + 0x9E3779B97F4A7C15ull * c;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  st[2] = z ^ (z >> 31);
}

__global__ void add_i64(int64_t* x, int64_t n, int64_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += v;
}

}  // namespace fs2

using namespace fs2;

extern "C" {

int64_t fs2_grad_norm_ws_bytes(int64_t n) {
  (void)n;
  return GN_BLOCKS * 4;
}

int fs2_grad_norm(const float* g, int64_t n, float max_norm, float* norm_coef, float* ws,
                  int64_t ws_bytes, void* stream) {
  FS2_CHECK_ARG(ws_bytes >= fs2_grad_norm_ws_bytes(n), "fs2_grad_norm: workspace too small");
  FS2_CHECK_ARG(((uintptr_t)g & 15) == 0, "fs2_grad_norm: gradient buffer must be 16-B aligned");
  hipStream_t st = as_stream(stream);
  poison(ws, ws_bytes, st);
  sumsq_partial<<<GN_BLOCKS, 256, 0, st>>>(g, n, ws);
  norm_final<<<1, 1024, 0, st>>>(ws, GN_BLOCKS, max_norm, norm_coef);
  return launch_status("fs2_grad_norm");
}

int fs2_adam_step(float* p, const float* g, float* m, float* v, int64_t n, const float* norm_coef,
                  float lr, float beta1, float beta2, float eps, float bias_corr1,
                  float bias_corr2_sqrt, const float* hyper, void* stream) {
  FS2_CHECK_ARG((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0,
                "fs2_adam_step: buffers must be 16-B aligned");
  if (n == 0) return FS2_OK;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  adam_kernel<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(p, g, m, v, n, norm_coef, lr, beta1,
                                                               beta2, eps, bias_corr1,
                                                               bias_corr2_sqrt, hyper);
  return launch_status("fs2_adam_step");
}

int fs2_sched_step(int64_t* steps, float* hyper, double init_lr, int64_t n_warmup,
                   const int64_t* anneal_steps_host, int n_anneal, double anneal_rate, double beta1,
                   double beta2, int advance_lr, void* stream) {
  FS2_CHECK_ARG(n_anneal >= 0 && n_anneal <= 3, "fs2_sched_step: at most 3 anneal steps");
  int64_t an[3] = {0, 0, 0};
  for (int i = 0; i < n_anneal; ++i) an[i] = anneal_steps_host[i];
  sched_step_kernel<<<1, 64, 0, as_stream(stream)>>>(steps, hyper, init_lr, n_warmup, an[0], an[1],
                                                     an[2], n_anneal, anneal_rate, beta1, beta2,
                                                     advance_lr);
  return launch_status("fs2_sched_step");
}

int fs2_seed_next(uint64_t* state, void* stream) {
  seed_next_kernel<<<1, 64, 0, as_stream(stream)>>>(state);
  return launch_status("fs2_seed_next");
}

int fs2_add_i64(int64_t* x, int64_t n, int64_t value, void* stream) {
  if (n == 0) return FS2_OK;
  add_i64<<<(unsigned)((n + 255) / 256), 256, 0, as_stream(stream)>>>(x, n, value);
  return launch_status("fs2_add_i64");
}

}  // extern "C"
