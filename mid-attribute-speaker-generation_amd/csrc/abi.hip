// Error reporting and small utility entry points of the C-ABI.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "common.hpp"

namespace fs2 {

int g_tune[FS2_TUNE_COUNT] = {};

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return FS2_ERR_LAUNCH;
  }
  return FS2_OK;
}

__global__ void fill_kernel(float* x, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = v;
}
__global__ void scale_kernel(float* x, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= v;
}

__global__ void add_kernel(float* out, const float* a, const float* b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a[i] + b[i];
}

__global__ void fill_from_kernel(float* x, int64_t n, const float* src, float scale,
                                 const float* den) {
  const float v = src[0] * scale / (den ? den[0] : 1.f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] = v;
}

static int g_poison = -2;  // -2: FS2_POISON not read yet

int poison_byte() {
  if (g_poison == -2) {
    const char* e = getenv("FS2_POISON");
    g_poison = (e && *e) ? (atoi(e) & 0xff) : -1;
  }
  return g_poison;
}

void poison(void* p, int64_t bytes, hipStream_t st) {
  const int b = poison_byte();
  if (b >= 0 && p && bytes > 0) (void)hipMemsetAsync(p, b, (size_t)bytes, st);
}

static unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace fs2

using namespace fs2;

extern "C" {

const char* fs2_last_error(void) { return g_err; }

int fs2_abi_version(void) { return 1; }

int fs2_set_tuning(int knob, int value) {
  FS2_CHECK_ARG(knob >= 0 && knob < FS2_TUNE_COUNT, "fs2_set_tuning: unknown knob %d", knob);
  g_tune[knob] = value;
  return FS2_OK;
}

// Cross-stream ordering without host objects: a ring of timing-free events; a wait binds to
// the record made just before it, so re-recording a ring slot later is harmless.
int fs2_stream_wait(void* waiter, void* signaler) {
  static hipEvent_t ring[64];
  static int next = 0;
  static bool init = false;
  if (!init) {
    for (auto& e : ring)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        set_error("fs2_stream_wait: hipEventCreate failed");
        return FS2_ERR_LAUNCH;
      }
    init = true;
  }
  hipEvent_t ev = ring[next];
  next = (next + 1) & 63;
  if (hipEventRecord(ev, as_stream(signaler)) != hipSuccess ||
      hipStreamWaitEvent(as_stream(waiter), ev, 0) != hipSuccess) {
    set_error("fs2_stream_wait: event record/wait failed");
    return FS2_ERR_LAUNCH;
  }
  return FS2_OK;
}

int fs2_debug_poison(int byte) {
  g_poison = byte < 0 ? -1 : (byte & 0xff);
  return FS2_OK;
}

// torch.cuda.memory.CUDAPluggableAllocator pair: no caching, every block filled with the poison
// byte (0xff when poisoning is off) at allocation; a free waits for the device to drain first
void* fs2_debug_alloc(int64_t size, int device, void* stream) {
  (void)device;
  (void)stream;
  void* p = nullptr;
  if (hipMalloc(&p, size > 0 ? (size_t)size : 1) != hipSuccess) return nullptr;
  const int b = poison_byte();
  if (size > 0 && hipMemset(p, b >= 0 ? b : 0xff, (size_t)size) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  return p;
}

void fs2_debug_free(void* p, int64_t size, int device, void* stream) {
  (void)size;
  (void)device;
  (void)stream;
  (void)hipDeviceSynchronize();
  (void)hipFree(p);
}

int fs2_fill(float* x, int64_t n, float value, void* stream) {
  if (n <= 0) return FS2_OK;
  fill_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(x, n, value);
  return launch_status("fs2_fill");
}

int fs2_fill_from(float* x, int64_t n, const float* src, float scale, const float* den,
                  void* stream) {
  if (n <= 0) return FS2_OK;
  fill_from_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(x, n, src, scale, den);
  return launch_status("fs2_fill_from");
}

int fs2_add(float* out, const float* a, const float* b, int64_t n, void* stream) {
  if (n <= 0) return FS2_OK;
  add_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(out, a, b, n);
  return launch_status("fs2_add");
}

int fs2_scale(float* x, int64_t n, float value, void* stream) {
  if (n <= 0) return FS2_OK;
  scale_kernel<<<grid_for(n), 256, 0, as_stream(stream)>>>(x, n, value);
  return launch_status("fs2_scale");
}

}  // extern "C"
