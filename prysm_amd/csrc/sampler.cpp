// Internal (tools/walk_sampler.py): a wall-clock PC sampler for the calling thread, to find
// where the chain walk's host time goes (there is no perf on the boxes).  A POSIX timer
// delivers SIGPROF to this thread every `interval_us`; the handler stores the interrupted
// instruction pointer and up to kDepth - 1 of its callers (the unwinder steps through the
// signal frame; backtrace() is called once at start so that it is loaded before any signal).
// pz_debug_sample_stop maps each PC to (object file, offset in it) with dladdr, for
// llvm-symbolizer.  Not for product use: one sampler per process; backtrace() in a signal
// handler is not async-signal-safe in general (it is warmed up at start, and glibc's loader
// lock it may take is recursive, so a sample that lands inside the walk's own unwinding --
// a rejected attestation's throw -- re-enters it on the same thread).
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

constexpr int kDepth = 16;
std::vector<uint64_t> g_pcs;  // [sample][kDepth], 0-terminated
std::atomic<uint64_t> g_n{0};
timer_t g_timer;
bool g_on = false;
struct sigaction g_old;

void on_sample(int, siginfo_t*, void* uc) {
  const uint64_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if ((i + 1) * kDepth > g_pcs.size()) return;
  uint64_t* out = &g_pcs[i * kDepth];
  const uint64_t rip = (uint64_t)static_cast<ucontext_t*>(uc)->uc_mcontext.gregs[REG_RIP];
  out[0] = rip;
  void* bt[kDepth + 8];
  const int n = backtrace(bt, kDepth + 8);
  int k = 0;
  while (k < n && (uint64_t)bt[k] != rip) ++k;  // frames above the handler and the trampoline
  for (int d = 1; d < kDepth; ++d) out[d] = (k + d < n) ? (uint64_t)bt[k + d] : 0;
}

}  // namespace

extern "C" int pz_debug_sample_start(int interval_us, uint64_t cap) {
  if (g_on || interval_us <= 0 || !cap) return -1;
  g_pcs.assign(cap * kDepth, 0);
  void* warm[4];
  (void)backtrace(warm, 4);
  g_n.store(0);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_sample;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old)) return -2;
  struct sigevent ev;
  std::memset(&ev, 0, sizeof ev);
  ev.sigev_notify = SIGEV_THREAD_ID;
  ev.sigev_signo = SIGPROF;
  ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
  if (timer_create(CLOCK_MONOTONIC, &ev, &g_timer)) return -3;
  struct itimerspec its;
  its.it_interval.tv_sec = interval_us / 1000000;
  its.it_interval.tv_nsec = (long)(interval_us % 1000000) * 1000;
  its.it_value = its.it_interval;
  if (timer_settime(g_timer, 0, &its, nullptr)) return -4;
  g_on = true;
  return 0;
}

// Stops the sampler.  For sample i and depth d (kDepth entries per sample, frame 0 the
// interrupted PC): offs[i*kDepth+d] = PC - base of its object, obj[...] = index into the
// '\n'-separated object names written to `names` (cap `ncap` bytes), UINT32_MAX past the
// stack's end.  `cap` counts samples.  Returns the number of samples.
extern "C" int pz_debug_sample_depth() { return kDepth; }

extern "C" int64_t pz_debug_sample_stop(uint64_t* offs, uint32_t* obj, uint64_t cap, char* names, uint64_t ncap) {
  if (!g_on) return -1;
  timer_delete(g_timer);
  sigaction(SIGPROF, &g_old, nullptr);
  g_on = false;
  const uint64_t n = std::min<uint64_t>(g_n.load(), std::min<uint64_t>(cap, g_pcs.size() / kDepth));
  std::vector<std::string> objs;
  for (uint64_t i = 0; i < n * kDepth; ++i) {
    if (!g_pcs[i]) {
      offs[i] = 0;
      obj[i] = UINT32_MAX;
      continue;
    }
    Dl_info info;
    std::string name = "?";
    uint64_t base = 0;
    if (dladdr((void*)g_pcs[i], &info) && info.dli_fname) {
      name = info.dli_fname;
      base = (uint64_t)info.dli_fbase;
    }
    uint32_t k = 0;
    while (k < objs.size() && objs[k] != name) ++k;
    if (k == objs.size()) objs.push_back(name);
    offs[i] = g_pcs[i] - base;
    obj[i] = k;
  }
  std::string all;
  for (auto& o : objs) all += o + "\n";
  if (names && ncap) {
    const size_t m = std::min<size_t>(all.size(), ncap - 1);
    std::memcpy(names, all.data(), m);
    names[m] = 0;
  }
  return (int64_t)n;
}
