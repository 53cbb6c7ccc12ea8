#include "sampler.h"

#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <stdexcept>

namespace igp {
namespace sampler {
namespace {

Sample* g_ring = nullptr;
size_t g_cap = 0;
std::atomic<uint64_t> g_n{0};
std::atomic<bool> g_on{false};
struct sigaction g_old {};

void on_prof(int, siginfo_t*, void* ctx) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  const auto* uc = static_cast<const ucontext_t*>(ctx);
  const uint64_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  Sample& s = g_ring[i % g_cap];
  s.pc = uint64_t(uc->uc_mcontext.gregs[REG_RIP]);
  s.tid = int32_t(syscall(SYS_gettid));
}

}  // namespace

void start(int hz, size_t capacity) {
  if (g_on.load()) throw std::runtime_error("sampler: already running");
  if (hz < 1 || hz > 20000 || capacity < 1) throw std::runtime_error("sampler: hz 1..20000, capacity >= 1");
  delete[] g_ring;
  g_ring = new Sample[capacity]();
  g_cap = capacity;
  g_n.store(0);
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old) != 0) throw std::runtime_error("sampler: sigaction");
  g_on.store(true);
  itimerval it{};
  it.it_interval.tv_sec = 0;
  it.it_interval.tv_usec = 1000000 / hz;
  it.it_value = it.it_interval;
  if (setitimer(ITIMER_PROF, &it, nullptr) != 0) {
    g_on.store(false);
    throw std::runtime_error("sampler: setitimer");
  }
}

std::vector<Sample> stop() {
  itimerval it{};
  setitimer(ITIMER_PROF, &it, nullptr);
  g_on.store(false);
  sigaction(SIGPROF, &g_old, nullptr);
  const uint64_t n = g_n.load();
  std::vector<Sample> out;
  if (!g_ring) return out;
  const uint64_t first = n > g_cap ? n - g_cap : 0;
  out.reserve(size_t(n - first));
  for (uint64_t i = first; i < n; ++i) out.push_back(g_ring[i % g_cap]);
  return out;
}

}  // namespace sampler
}  // namespace igp
