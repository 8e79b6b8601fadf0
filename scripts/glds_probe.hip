// L2 -> CU load-path throughput probe (standalone): how many bytes per second the chip moves
// from a buffer into LDS by LDS-DMA (global_load_lds_dwordx4) and into VGPRs by
// global_load_dwordx4, as a function of waves per workgroup, workgroups per CU, tiles in flight
// and the buffer size (L2-resident or not).  Each workgroup streams 16 KiB tiles: tile t of
// workgroup w starts at ((w * 7 + t) * 16 KiB) mod the buffer size.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/glds_probe.hip -o scripts/glds_probe && scripts/glds_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr int TILE = 16384;  // bytes per tile

__device__ inline void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int AHEAD>
__device__ inline void wait_tiles(int per) {
  // at most AHEAD tiles (per instructions each) in flight
  if (AHEAD == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (AHEAD == 1) {
    if (per == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if (per == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (per == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (per == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// LDS-DMA: NW waves, STAGES LDS slots of 16 KiB, STAGES-1 tiles ahead; one raw barrier per tile
template <int NW, int STAGES>
__global__ __launch_bounds__(NW * 64) void probe_glds(const char* buf, size_t nbytes, int tiles,
                                                      float* sink) {
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * TILE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  constexpr int PER = TILE / (NW * 64 * 16);  // glds instructions per wave per tile
  auto issue = [&](int t, int slot) {
    const size_t base = ((size_t)(blockIdx.x * 7 + t) * TILE) % nbytes;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int off = ((wave * PER + i) * 64 + lane) * 16;
      glds16(buf + base + off, lds + slot * TILE + (wave * PER + i) * 1024);
    }
  };
  for (int t = 0; t < STAGES - 1 && t < tiles; ++t) issue(t, t);
  float acc = 0.f;
  for (int t = 0; t < tiles; ++t) {
    wait_tiles<STAGES - 2>(PER);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + STAGES - 1 < tiles) issue(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    acc += reinterpret_cast<const float*>(lds + (t % STAGES) * TILE)[tid];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

// register loads: each wave streams its share of each tile with global_load_dwordx4, DEPTH
// tiles' loads outstanding per lane
template <int NW, int DEPTH>
__global__ __launch_bounds__(NW * 64) void probe_vgpr(const char* buf, size_t nbytes, int tiles,
                                                      float* sink) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  constexpr int PER = TILE / (NW * 64 * 16);
  uint4 r[DEPTH][PER];
  uint32_t acc = 0;
  auto load = [&](int t, uint4 (&dst)[PER]) {
    const size_t base = ((size_t)(blockIdx.x * 7 + t) * TILE) % nbytes;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      dst[i] = *reinterpret_cast<const uint4*>(buf + base + ((wave * PER + i) * 64 + lane) * 16);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, r[d]);
  for (int t = 0; t < tiles; t += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int i = 0; i < PER; ++i) acc ^= r[d][i].x ^ r[d][i].w;
      if (t + DEPTH + d < tiles) load(t + DEPTH + d, r[d]);
    }
  }
  if (acc == 12345u) sink[blockIdx.x] = (float)acc;
}

template <typename F>
static double time_ms(F launch, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const size_t big = (size_t)1 << 30;  // 1 GiB: HBM / Infinity Cache
  char* buf;
  float* sink;
  CHECK(hipMalloc(&buf, big));
  CHECK(hipMemset(buf, 1, big));
  CHECK(hipMalloc(&sink, 1 << 20));
  const int tiles = 256;
  struct Size { size_t n; const char* name; } sizes[] = {{(size_t)2 << 20, "2 MiB (L2)"},
                                                        {(size_t)64 << 20, "64 MiB (MALL)"},
                                                        {big, "1 GiB (HBM)"}};
  for (auto sz : sizes) {
    for (int wgs_per_cu : {1, 2, 4}) {
      const int grid = 256 * wgs_per_cu;
      const double bytes = (double)grid * tiles * TILE;
#define RUN(label, KERN, NW)                                                               \
  {                                                                                        \
    const double ms = time_ms([&] { KERN<<<grid, NW * 64>>>(buf, sz.n, tiles, sink); }, 5); \
    std::printf("%-14s wg/CU %d  %-22s %7.2f TB/s  (%.1f GB/s per CU)\n", sz.name,        \
                wgs_per_cu, label, bytes / ms / 1e9, bytes / ms / 1e6 / 256);              \
  }
      RUN("glds 4w 2 stages", (probe_glds<4, 2>), 4)
      RUN("glds 4w 3 stages", (probe_glds<4, 3>), 4)
      RUN("glds 8w 2 stages", (probe_glds<8, 2>), 8)
      RUN("glds 8w 3 stages", (probe_glds<8, 3>), 8)
      RUN("vgpr 4w depth 1", (probe_vgpr<4, 1>), 4)
      RUN("vgpr 4w depth 2", (probe_vgpr<4, 2>), 4)
      RUN("vgpr 8w depth 2", (probe_vgpr<8, 2>), 8)
#undef RUN
    }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
