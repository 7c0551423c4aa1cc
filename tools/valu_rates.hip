// Microbenchmark: issue rate of candidate VALU instructions for the BLAKE2b G function on
// every CU (gfx950).  Each lane runs 8 independent register chains of one instruction form
// in inline asm; rates are reported per CU-cycle at 2.4 GHz and relative to v_xor_b32.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o build/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

#define X4(ins) ins "\n" ins "\n" ins "\n" ins
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b0 = a0 * 3, b1 = a1 * 3, b2 = a2 * 3, b3 = a3 * 3, b4 = a4 * 3, b5 = a5 * 3, b6 = a6 * 3, b7 = a7 * 3;
  uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  const uint32_t sel = __builtin_amdgcn_readfirstlane(0x05040706u + (iters >> 30));
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#define EIGHT(fmt) \
  asm volatile(fmt : "+v"(a0) : "v"(b0)); asm volatile(fmt : "+v"(a1) : "v"(b1)); \
  asm volatile(fmt : "+v"(a2) : "v"(b2)); asm volatile(fmt : "+v"(a3) : "v"(b3)); \
  asm volatile(fmt : "+v"(a4) : "v"(b4)); asm volatile(fmt : "+v"(a5) : "v"(b5)); \
  asm volatile(fmt : "+v"(a6) : "v"(b6)); asm volatile(fmt : "+v"(a7) : "v"(b7));
      if (OP == 0) { EIGHT("v_xor_b32 %0, %0, %1") }
      else if (OP == 1) { EIGHT("v_alignbit_b32 %0, %0, %1, 24") }
      else if (OP == 2) {  // selector from an SGPR (VOP3 takes no literal on gfx9)
#define PERM(a, b) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(sel));
        PERM(a0, b0) PERM(a1, b1) PERM(a2, b2) PERM(a3, b3) PERM(a4, b4) PERM(a5, b5) PERM(a6, b6) PERM(a7, b7)
      }
      else if (OP == 3) { EIGHT("v_add_u32 %0, %0, %1") }
      else if (OP == 4) { EIGHT("v_add3_u32 %0, %0, %1, %0") }
      else if (OP == 5) { EIGHT("v_lshl_or_b32 %0, %0, 1, %1") }
      else if (OP == 6) { EIGHT("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96") }
      else if (OP == 7) {  // 64-bit add via v_lshl_add_u64, 4 independent pairs
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a0) : "v"(*(uint64_t*)&b0));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a2) : "v"(*(uint64_t*)&b2));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a4) : "v"(*(uint64_t*)&b4));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a6) : "v"(*(uint64_t*)&b6));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a0) : "v"(*(uint64_t*)&b0));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a2) : "v"(*(uint64_t*)&b2));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a4) : "v"(*(uint64_t*)&b4));
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(*(uint64_t*)&a6) : "v"(*(uint64_t*)&b6));
      } else if (OP == 8) {  // 64-bit add as v_add_co_u32 + v_addc_co_u32 with private SGPR carries
#define ADDCO(lo, hi, blo, bhi, c) asm volatile("v_add_co_u32 %0, %2, %0, %3\n v_addc_co_u32 %1, %2, %1, %4, %2" : "+v"(lo), "+v"(hi), "=&s"(c) : "v"(blo), "v"(bhi));
        ADDCO(a0, a1, b0, b1, c0) ADDCO(a2, a3, b2, b3, c1) ADDCO(a4, a5, b4, b5, c2) ADDCO(a6, a7, b6, b7, c3)
      } else if (OP == 9) {  // 64-bit shift
        asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&a0)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&a2));
        asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&a4)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&a6));
        asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&b0)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&b2));
        asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&b4)); asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(*(uint64_t*)&b6));
      } else if (OP == 10) {  // v_mad_u64_u32 (64-bit result)
#define MAD(lo, hi, b, c) asm volatile("v_mad_u64_u32 %0, %1, %2, 1, %0" : "+v"(*(uint64_t*)&lo), "=&s"(c) : "v"(b));
        MAD(a0, a1, b0, c0) MAD(a2, a3, b2, c1) MAD(a4, a5, b4, c2) MAD(a6, a7, b6, c3)
        MAD(a0, a1, b1, c0) MAD(a2, a3, b3, c1) MAD(a4, a5, b5, c2) MAD(a6, a7, b7, c3)
      } else if (OP == 11) {  // v_add_co_u32 alone (VOP3, private carries)
#define CO(lo, b, c) asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(lo), "=&s"(c) : "v"(b));
        CO(a0, b0, c0) CO(a1, b1, c1) CO(a2, b2, c2) CO(a3, b3, c3) CO(a4, b4, c0) CO(a5, b5, c1) CO(a6, b6, c2) CO(a7, b7, c3)
      } else if (OP == 12) {  // 64-bit add as VOP2 v_add_co_u32_e32 + v_addc_co_u32_e32 through VCC
#define ADDVCC(lo, hi, blo, bhi) asm volatile("v_add_co_u32_e32 %0, vcc, %2, %0\n v_addc_co_u32_e32 %1, vcc, %3, %1, vcc" : "+v"(lo), "+v"(hi) : "v"(blo), "v"(bhi) : "vcc");
        ADDVCC(a0, a1, b0, b1) ADDVCC(a2, a3, b2, b3) ADDVCC(a4, a5, b4, b5) ADDVCC(a6, a7, b6, b7)
      } else if (OP == 13) { EIGHT("v_add_u32_e64 %0, %0, %1") }
      else if (OP == 14) { EIGHT("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1") }
      else if (OP == 15) { EIGHT("v_lshlrev_b32_e32 %0, 1, %0") }
      else if (OP == 16) { EIGHT("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD") }
      else if (OP == 17) { EIGHT("v_xor_b32_e64 %0, %0, %1") }
      else if (OP == 18) {  // dependent chain: one 64-bit VCC add chain per lane-pair (latency)
        ADDVCC(a0, a1, b0, b1) ADDVCC(a0, a1, b2, b3) ADDVCC(a0, a1, b4, b5) ADDVCC(a0, a1, b6, b7)
      } else if (OP == 19) { EIGHT("v_alignbit_b32 %0, %0, %1, %1") }
      else if (OP == 20) { EIGHT("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0") }
      else if (OP == 21) { EIGHT("v_lshl_add_u32 %0, %0, 1, %1") }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b2 ^ b4 ^ b6 ^ (uint32_t)(c0 ^ c1 ^ c2 ^ c3);
}

typedef void (*kfn)(uint32_t*, int);
int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8, threads = 256, iters = 1000;
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  struct { const char* name; kfn f; double per_r; } ops[] = {
      {"v_xor_b32", k<0>, 8}, {"v_alignbit_b32", k<1>, 8}, {"v_perm_b32", k<2>, 8},
      {"v_add_u32", k<3>, 8}, {"v_add3_u32", k<4>, 8}, {"v_lshl_or_b32", k<5>, 8},
      {"v_bitop3_b32", k<6>, 8}, {"v_lshl_add_u64", k<7>, 8}, {"v_add_co+v_addc_co (s carry)", k<8>, 8},
      {"v_lshlrev_b64", k<9>, 8}, {"v_mad_u64_u32", k<10>, 8}, {"v_add_co_u32 (s carry)", k<11>, 8},
      {"v_add_co_e32+v_addc_co_e32 (vcc)", k<12>, 8}, {"v_add_u32_e64", k<13>, 8}, {"v_xor_b32_sdwa", k<14>, 8},
      {"v_lshlrev_b32_e32", k<15>, 8}, {"v_xor_b32_sdwa dword", k<16>, 8}, {"v_xor_b32_e64", k<17>, 8},
      {"vcc add64 dependent chain", k<18>, 8}, {"v_alignbit_b32 (vgpr shift)", k<19>, 8},
      {"v_mov_b32_sdwa", k<20>, 8}, {"v_lshl_add_u32", k<21>, 8}};
  double xor_rate = 0;
  for (auto& o : ops) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(o.f, dim3(blocks), dim3(threads), 0, 0, out, iters);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    double rate = (double)blocks * threads * iters * 16 * o.per_r / (best * 1e-3);
    if (xor_rate == 0) xor_rate = rate;
    printf("%-30s %8.3f ms  %7.2f T lane-instr/s  %6.1f per CU-cycle@2.4GHz  rel. xor %.3f\n", o.name, best,
           rate / 1e12, rate / (cus * 2.4e9), rate / xor_rate);
  }
  return 0;
}
