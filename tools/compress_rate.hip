// Microbenchmark: the BLAKE2b compression of blake2b.hip on register-resident data (no memory
// traffic), to separate the VALU-bound ceiling of the current code from the memory pipeline.
// Build: hipcc --offload-arch=gfx950 -O3 -I prysm_amd/csrc tools/compress_rate.hip -o build/compress_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define main blake2b_unused_main
#include "../prysm_amd/csrc/blake2b.hip"
#undef main

__global__ void __launch_bounds__(256) crate(uint64_t* out, int iters, uint64_t seed) {
  uint64_t h[8], m[16];
  pz::init_h(h);
  for (int k = 0; k < 16; ++k) m[k] = seed * (k + 1) + threadIdx.x + blockIdx.x * 977ull;
  for (int i = 0; i < iters; ++i) {
    pz::compress(h, m, 128ull * (i + 1), false);
    m[i & 15] ^= h[0];
  }
  uint64_t x = 0;
  for (int k = 0; k < 8; ++k) x ^= h[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint64_t* out;
  hipMalloc(&out, (size_t)cus * 64 * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int bpc : {4, 8, 16}) {
    const int blocks = cus * bpc, iters = 400;
    hipLaunchKernelGGL(crate, dim3(blocks), dim3(256), 0, 0, out, 20, 1);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(crate, dim3(blocks), dim3(256), 0, 0, out, iters, rep + 2);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double comps = (double)blocks * 256 * iters;
    printf("blocks/CU %2d: %.3f ms  %.2f G compressions/s  (%.2f G 512-B records/s)\n", bpc, best,
           comps / best / 1e6, comps / 4 / best / 1e6);
  }
  return 0;
}
