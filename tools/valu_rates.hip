// Microbenchmark: issue rate of the VALU instructions the BLAKE2b kernel is made of, on
// every CU (gfx950).  Each lane runs 8 independent chains of one instruction in inline asm;
// the rate is reported as lane-instructions per second and per CU-cycle at the measured clock.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o build/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters, uint64_t* clk) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b0 = a0 * 3, b1 = a1 * 3, b2 = a2 * 3, b3 = a3 * 3, b4 = a4 * 3, b5 = a5 * 3, b6 = a6 * 3, b7 = a7 * 3;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (OP == 0) {  // v_xor_b32
        asm volatile("v_xor_b32 %0, %0, %1\n v_xor_b32 %2, %2, %3\n v_xor_b32 %4, %4, %5\n v_xor_b32 %6, %6, %7" : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3));
        asm volatile("v_xor_b32 %0, %0, %1\n v_xor_b32 %2, %2, %3\n v_xor_b32 %4, %4, %5\n v_xor_b32 %6, %6, %7" : "+v"(a4), "+v"(b4), "+v"(a5), "+v"(b5), "+v"(a6), "+v"(b6), "+v"(a7), "+v"(b7));
      } else if (OP == 1) {  // v_alignbit_b32
        asm volatile("v_alignbit_b32 %0, %0, %1, 24\n v_alignbit_b32 %2, %2, %3, 24\n v_alignbit_b32 %4, %4, %5, 24\n v_alignbit_b32 %6, %6, %7, 24" : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1), "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3));
        asm volatile("v_alignbit_b32 %0, %0, %1, 24\n v_alignbit_b32 %2, %2, %3, 24\n v_alignbit_b32 %4, %4, %5, 24\n v_alignbit_b32 %6, %6, %7, 24" : "+v"(a4), "+v"(b4), "+v"(a5), "+v"(b5), "+v"(a6), "+v"(b6), "+v"(a7), "+v"(b7));
      } else if (OP == 2) {  // v_lshl_add_u64 (64-bit add)
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %2, %2, 0, %3" : "+v"(*(uint64_t*)&a0), "+v"(*(uint64_t*)&b0), "+v"(*(uint64_t*)&a2), "+v"(*(uint64_t*)&b2));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %2, %2, 0, %3" : "+v"(*(uint64_t*)&a4), "+v"(*(uint64_t*)&b4), "+v"(*(uint64_t*)&a6), "+v"(*(uint64_t*)&b6));
      } else {  // v_add_co_u32 + v_addc_co_u32 pair (64-bit add the other way), counted as 2
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, %3, vcc" : "+v"(a0), "+v"(b0), "+v"(a1), "+v"(b1) :: "vcc");
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, %3, vcc" : "+v"(a2), "+v"(b2), "+v"(a3), "+v"(b3) :: "vcc");
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, %3, vcc" : "+v"(a4), "+v"(b4), "+v"(a5), "+v"(b5) :: "vcc");
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, %3, vcc" : "+v"(a6), "+v"(b6), "+v"(a7), "+v"(b7) :: "vcc");
      }
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *clk = t1 - t0;
}

int main() {
  int cus = 0;
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  cus = p.multiProcessorCount;
  const int blocks = cus * 8, threads = 256, iters = 2000;
  uint32_t* out; uint64_t* clk;
  CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
  CHK(hipMalloc(&clk, 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const char* names[4] = {"v_xor_b32", "v_alignbit_b32", "v_lshl_add_u64", "v_add_co+v_addc_co"};
  // instructions per lane per inner (r) iteration: 8, 8, 4, 8
  const double per_r[4] = {8, 8, 4, 8};
  for (int op = 0; op < 4; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      CHK(hipEventRecord(e0));
      if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
      if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
      if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
      if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(threads), 0, 0, out, iters, clk);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      uint64_t cyc; CHK(hipMemcpy(&cyc, clk, 8, hipMemcpyDeviceToHost));
      double lane_ops = (double)blocks * threads * iters * 16 * per_r[op];
      double rate = lane_ops / (ms * 1e-3);
      if (rep == 1)
        printf("%-20s %8.3f ms  %7.2f T lane-instr/s  (%.1f lane-instr per CU-cycle at 2.4 GHz)  block0 cycles %llu\n",
               names[op], ms, rate / 1e12, rate / (cus * 2.4e9), (unsigned long long)cyc);
    }
  }
  return 0;
}
