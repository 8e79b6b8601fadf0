// Probe: launch cost of a persistent-style kernel vs its LDS allocation and code size.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int BYTES>
__global__ __launch_bounds__(512, 1) void k_lds(int* out, int flag) {
  __shared__ unsigned char s[BYTES];
  if (flag) {  // never taken: keeps the allocation
    s[threadIdx.x] = (unsigned char)threadIdx.x;
    __syncthreads();
    out[blockIdx.x] = s[(threadIdx.x + 1) % 512];
  }
}
template <int BYTES>
float time_it(int* d, int grid) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  k_lds<BYTES><<<grid, 512>>>(d, 0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < 20; ++i) k_lds<BYTES><<<grid, 512>>>(d, 0);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 20 * 1000.f;
}
int main() {
  int* d;
  (void)hipMalloc(&d, 1 << 20);
  for (int grid : {256, 2048}) {
    printf("grid %d: 16K %.1f us | 64K %.1f us | 65K %.1f us | 96K %.1f us | 128K %.1f us | 150K %.1f us\n",
           grid, time_it<16384>(d, grid), time_it<65536>(d, grid), time_it<66560>(d, grid),
           time_it<98304>(d, grid), time_it<131072>(d, grid), time_it<153600>(d, grid));
  }
  return 0;
}
