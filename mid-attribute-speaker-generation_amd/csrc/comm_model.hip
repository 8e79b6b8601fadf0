// Stand-in for one data-parallel gradient all-reduce, for pricing the N > 1 collective schedule
// on one GPU (profiles/r5_dp_collective_model.txt).  Not on the training path.
//
// An RCCL ring all-reduce of S bytes over n ranks runs a few tens of workgroups (its channels)
// on every rank for about 2 (n - 1) / n * S / busbw seconds, reading and writing its slice of
// the bucket in HBM as the chunks pass through.  This kernel does the same to the GPU it runs
// on: `blocks` workgroups stream `bytes` of read + write-back over the buffer (values
// unchanged: each 16-B vector is read and stored back) paced to last `duration_ns`, so the step
// around it sees a collective's CU occupancy, HBM traffic and duration, without the
// interconnect.  Pacing uses the 100 MHz constant clock (s_memrealtime); every wave exits after
// its share and its time, so the grid always drains.
#include "common.hpp"

namespace fs2 {

__global__ __launch_bounds__(256) void collective_standin(float* buf, int64_t n4, int64_t iters,
                                                          int64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int64_t it = 0; it < iters; ++it) {
    if (n4 > 0) {
      const int64_t e = i % n4;
      f32x4* p = reinterpret_cast<f32x4*>(buf) + e;
      const f32x4 v = *p;
      asm volatile("" ::"v"(v));  // keep the read (the store writes the same bytes back)
      *p = v;
      i += stride;
    }
    // pace: this iteration may not finish before its share of the duration
    const uint64_t due = t0 + (uint64_t)((it + 1) * ticks / iters);
    while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace fs2

using namespace fs2;

extern "C" int fs2_collective_standin(float* buf, int64_t n, int64_t bytes, int blocks,
                                      int64_t duration_ns, void* stream) {
  FS2_CHECK_ARG(n < 4 || (buf != nullptr && ((uintptr_t)buf & 15) == 0),
                "fs2_collective_standin: 16-B aligned buffer");
  FS2_CHECK_ARG(blocks >= 1 && blocks <= 1024 && bytes >= 0 && duration_ns >= 0 &&
                    duration_ns <= 1000000000LL,
                "fs2_collective_standin: 1..1024 blocks, duration <= 1 s");
  // each iteration moves 2 x 16 B per thread (read + write back)
  const int64_t per_iter = (int64_t)blocks * 256 * 32;
  int64_t iters = (bytes + per_iter - 1) / per_iter;
  if (iters < 1) iters = 1;
  const int64_t ticks = duration_ns / 10;  // 100 MHz
  collective_standin<<<blocks, 256, 0, as_stream(stream)>>>(buf, n / 4, iters, ticks);
  return launch_status("fs2_collective_standin");
}
