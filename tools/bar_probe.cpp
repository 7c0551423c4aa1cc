// Which device allocations can the host write directly (PCIe BAR), and what a kernel's read
// latency is for each (tools/ only; a child process per attempt, so a host fault ends only it).
//   hipcc --offload-arch=gfx950 -O2 tools/bar_probe.cpp -o /tmp/bar_probe && /tmp/bar_probe
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void chase(const uint32_t* p, uint32_t n, uint32_t* out, uint64_t* ticks) {
  // one lane follows a dependent chain of n loads: the per-load latency of this memory
  uint32_t i = 0;
  const uint64_t t0 = wall_clock64();
  for (uint32_t k = 0; k < n; ++k) i = __builtin_nontemporal_load(p + i);
  const uint64_t t1 = wall_clock64();
  out[0] = i;
  ticks[0] = t1 - t0;
}

static void probe(const char* name, int kind) {
  pid_t pid = fork();
  if (pid == 0) {
    void* p = nullptr;
    hipError_t e = hipSuccess;
    const size_t bytes = 1 << 20;
    if (kind == 0) e = hipMalloc(&p, bytes);
    if (kind == 1) e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained);
    if (kind == 2) e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
    if (kind == 3) e = hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (kind == 4) e = hipMallocManaged(&p, bytes);
    if (e != hipSuccess) {
      printf("%-28s alloc failed: %s\n", name, hipGetErrorString(e));
      fflush(stdout);
      _exit(1);
    }
    hipPointerAttribute_t at;
    hipPointerGetAttributes(&at, p);
    printf("%-28s ptr %p type %d hostPointer %p devicePointer %p\n", name, p, (int)at.type, at.hostPointer,
           at.devicePointer);
    fflush(stdout);
    // host writes: a chain 0 -> 16 -> 32 ... (64-B steps), wrapping
    const uint32_t n = 4096;
    uint32_t* h = static_cast<uint32_t*>(p);
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; k < n; ++k) h[k * 16] = ((k + 1) % n) * 16;
    __builtin_ia32_sfence();
    auto t1 = std::chrono::steady_clock::now();
    printf("%-28s host wrote %u words: %.2f us\n", name, n, std::chrono::duration<double, std::micro>(t1 - t0).count());
    fflush(stdout);
    uint32_t* d_out;
    uint64_t* d_t;
    hipMalloc(&d_out, 4);
    hipMalloc(&d_t, 8);
    const void* dp = at.devicePointer ? at.devicePointer : p;
    for (int r = 0; r < 3; ++r) {
      hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, static_cast<const uint32_t*>(dp), 256u, d_out, d_t);
      hipDeviceSynchronize();
    }
    uint64_t t;
    hipMemcpy(&t, d_t, 8, hipMemcpyDeviceToHost);
    printf("%-28s kernel dependent load: %.0f ns each (256 loads)\n", name, t * 10.0 / 256);
    fflush(stdout);
    _exit(0);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  if (WIFSIGNALED(st)) printf("%-28s child died with signal %d (host access faulted)\n", name, WTERMSIG(st));
  fflush(stdout);
}

int main() {
  probe("hipMalloc", 0);
  probe("hipExtMalloc(Finegrained)", 1);
  probe("hipExtMalloc(Uncached)", 2);
  probe("hipHostMalloc(mapped,coh)", 3);
  probe("hipMallocManaged", 4);
  return 0;
}
