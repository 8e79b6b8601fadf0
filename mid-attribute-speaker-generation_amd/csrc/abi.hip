// Error reporting and small utility entry points of the C-ABI.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <mutex>
#include <vector>

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

// LDS poisoning (with fs2_debug_poison): one 160 KiB block per CU fills its LDS with the poison
// byte, so a kernel that reads LDS it did not write in its own launch reads the byte instead of
// what the CU's previous kernel left there
__global__ __launch_bounds__(256) void lds_fill_kernel(uint32_t word) {
  extern __shared__ uint32_t lds_all[];
  for (int i = threadIdx.x; i < 163840 / 4; i += 256) lds_all[i] = word;
  __syncthreads();
  if (lds_all[(threadIdx.x * 37) % (163840 / 4)] == 0x12345678u && word == 1u) lds_all[0] = 0;
}
void lds_poison(hipStream_t st) {
  const int b = poison_byte();
  if (b < 0) return;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lds_fill_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  const uint32_t w = 0x01010101u * (uint32_t)b;
  lds_fill_kernel<<<512, 256, 163840, st>>>(w);
}

// debug snapshots (fs2_debug_snap): copies of intermediate buffers appended, in stream order,
// to one caller-owned device buffer; nothing is copied while no buffer is set
__global__ void snap_copy_kernel(const unsigned char* src, unsigned char* dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
static unsigned char* g_snap = nullptr;
static int64_t g_snap_cap = 0, g_snap_used = 0;
void snap(const void* p, int64_t bytes, hipStream_t st) {
  if (!g_snap || !p || bytes <= 0) return;
  if (g_snap_used + bytes > g_snap_cap) {
    g_snap_used = g_snap_cap + 1;  // overflow: reported by fs2_debug_snap_used
    return;
  }
  // a kernel, not hipMemcpyAsync: the copy must see memory exactly as the next kernel would
  snap_copy_kernel<<<grid_for((bytes + 3) / 4), 256, 0, st>>>(
      static_cast<const unsigned char*>(p), g_snap + g_snap_used, bytes);
  g_snap_used += bytes;
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

// race mode (fs2_debug_race): mode 0 holds every stream other than `main` back this long after
// each cross-stream wait it receives, so it trails the main stream; mode 1 holds the main stream
// back after each event a non-main stream waits on, so the main stream trails instead.
static int g_race_us = 0;
static int g_race_mode = 0;
static void* g_race_main = nullptr;
static uint64_t g_race_rng = 0;

__global__ void delay_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}

static int race_delay(void* st, int us) {
  static uint64_t per_us = 0;
  if (!per_us) {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || khz <= 0)
      khz = 100000;  // the 100 MHz constant clock
    per_us = (uint64_t)khz / 1000;
  }
  delay_kernel<<<1, 1, 0, as_stream(st)>>>((uint64_t)us * per_us);
  return launch_status("fs2_debug_race delay");
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
  lds_poison(as_stream(waiter));
  if (g_race_us > 0) {
    if (g_race_mode == 0 && waiter != g_race_main) return race_delay(waiter, g_race_us);
    if (g_race_mode == 1 && signaler == g_race_main && waiter != g_race_main)
      return race_delay(signaler, g_race_us);
    if (g_race_mode == 2) {  // seeded random schedule: either side may be held back
      for (void* st : {waiter, signaler}) {
        g_race_rng = g_race_rng * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t r = (uint32_t)(g_race_rng >> 33);
        if (r & 1) {
          const int rc = race_delay(st, (int)((r >> 1) % (uint32_t)g_race_us));
          if (rc) return rc;
        }
      }
    }
  }
  return FS2_OK;
}

// cross-XCD visibility probe (fs2_debug_coherence): every block reads all of x (so every XCD's
// L2 may hold its lines), then ONE block writes x[i] = tag + i, then every block reads x again
// and counts the elements that are not tag + i; three launches on one stream
__global__ void coh_read_kernel(const uint32_t* x, int64_t n, uint32_t tag, uint32_t* bad) {
  uint32_t acc = 0, nbad = 0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t v = x[i];
    acc += v;
    if (tag && v != tag + (uint32_t)i) ++nbad;
  }
  if (tag && nbad) bad[blockIdx.x] += nbad;
  if (acc == 0x9e3779b9u && !tag) bad[gridDim.x] = acc;  // keep the loads
}
__global__ void coh_write_kernel(uint32_t* x, int64_t n, uint32_t tag) {
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) x[i] = tag + (uint32_t)i;
}
int fs2_debug_coherence(void* x, int64_t n, int rounds, int blocks, void* bad, void* stream) {
  hipStream_t st = as_stream(stream);
  for (int r = 1; r <= rounds; ++r) {
    coh_read_kernel<<<blocks, 256, 0, st>>>((const uint32_t*)x, n, 0u, (uint32_t*)bad);
    coh_write_kernel<<<1, 256, 0, st>>>((uint32_t*)x, n, 0x1000000u * (uint32_t)r);
    coh_read_kernel<<<blocks, 256, 0, st>>>((const uint32_t*)x, n, 0x1000000u * (uint32_t)r,
                                            (uint32_t*)bad);
  }
  return launch_status("fs2_debug_coherence");
}

int fs2_debug_snap(void* buf, int64_t cap) {
  g_snap = static_cast<unsigned char*>(buf);
  g_snap_cap = buf ? cap : 0;
  g_snap_used = 0;
  return FS2_OK;
}
int64_t fs2_debug_snap_used(void) { return g_snap_used; }

int fs2_debug_race(int delay_us, void* main_stream, int mode, int seed) {
  FS2_CHECK_ARG(mode >= 0 && mode <= 2,
                "fs2_debug_race: mode 0 (side trails), 1 (main trails) or 2 (seeded random)");
  g_race_us = delay_us > 0 ? delay_us : 0;
  g_race_mode = mode;
  g_race_main = main_stream;
  g_race_rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)seed;
  return FS2_OK;
}

// LDS-DMA of an out-of-range buffer offset: what lands in LDS (one wave; out[i], i < 64 * 4,
// the dwords of 16 B per lane after the LDS was filled with 0xAB bytes)
__global__ void lds_dma_oob_kernel(const float* src, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t img[64 * 4];
  for (int i = threadIdx.x; i < 64 * 4; i += 64) img[i] = 0xABABABABu;
  __syncthreads();
  const auto r = buf_rsrc(src, 64 * 16);
  const uint32_t voff = threadIdx.x < 32 ? threadIdx.x * 16u : kOOB;
  glds16_buf(r, img, voff, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 4; i += 64) out[i] = img[i];
}
int fs2_debug_lds_dma_oob(const float* src, void* out, void* stream) {
  lds_dma_oob_kernel<<<1, 64, 0, as_stream(stream)>>>(src, (uint32_t*)out);
  return launch_status("fs2_debug_lds_dma_oob");
}

int fs2_debug_poison(int byte) {
  g_poison = byte < 0 ? -1 : (byte & 0xff);
  return FS2_OK;
}

// torch.cuda.memory.CUDAPluggableAllocator pair: no caching and no device synchronisation.  A
// block is filled with the poison byte (0xff when poisoning is off) at allocation (complete
// before the call returns) and again on its stream at its free; freed blocks are quarantined (never handed out again) until the
// quarantine passes kQuarantineBytes, then drained after a device synchronisation.  A read of
// a block after its free -- another stream still using it, unordered against the free --
// therefore sees the poison instead of whatever reused the memory.
static std::mutex g_dbg_mu;
static std::vector<void*> g_quarantine;
static size_t g_quarantine_bytes = 0;
static constexpr size_t kQuarantineBytes = size_t(6) << 30;

void* fs2_debug_alloc(int64_t size, int device, void* stream) {
  (void)device;
  void* p = nullptr;
  if (hipMalloc(&p, size > 0 ? (size_t)size : 1) != hipSuccess) {
    std::lock_guard<std::mutex> lock(g_dbg_mu);  // drain the quarantine and try once more
    (void)hipDeviceSynchronize();
    for (void* q : g_quarantine) (void)hipFree(q);
    g_quarantine.clear();
    g_quarantine_bytes = 0;
    if (hipMalloc(&p, size > 0 ? (size_t)size : 1) != hipSuccess) return nullptr;
  }
  // fresh memory: filled on a stream of our own and waited for here, so the fill precedes every
  // later use on any stream without ordering it behind (or draining) the work already queued on
  // the allocating stream -- which the race modes hold back on purpose
  (void)stream;
  static hipStream_t fill_st = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_dbg_mu);  // the allocator is called from several threads
    if (!fill_st && hipStreamCreateWithFlags(&fill_st, hipStreamNonBlocking) != hipSuccess)
      fill_st = nullptr;
  }
  const int b = poison_byte();
  if (size > 0 && (!fill_st || hipMemsetAsync(p, b >= 0 ? b : 0xff, (size_t)size, fill_st) != hipSuccess ||
                   hipStreamSynchronize(fill_st) != hipSuccess)) {
    (void)hipFree(p);
    return nullptr;
  }
  return p;
}

void fs2_debug_free(void* p, int64_t size, int device, void* stream) {
  (void)device;
  const int b = poison_byte();
  if (size > 0) (void)hipMemsetAsync(p, b >= 0 ? b : 0xff, (size_t)size, as_stream(stream));
  std::lock_guard<std::mutex> lock(g_dbg_mu);
  g_quarantine.push_back(p);
  g_quarantine_bytes += size > 0 ? (size_t)size : 1;
  if (g_quarantine_bytes > kQuarantineBytes) {
    (void)hipDeviceSynchronize();
    for (void* q : g_quarantine) (void)hipFree(q);
    g_quarantine.clear();
    g_quarantine_bytes = 0;
  }
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
