// C-ABI plumbing: thread-local last-error string and version query.
#include <atomic>
#include <mutex>
#include <vector>

#include "common.h"

#include "../../include/gr_hstu.h"

namespace gr {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

const char* last_error() { return g_err.c_str(); }

// ---------------------------------------------------------------- live kernel timing
struct TimedPair {
  std::string name;
  hipEvent_t start, stop;
};
static std::mutex g_tm_mu;
static std::vector<TimedPair> g_tm;
static std::atomic<bool> g_tm_on{false};

bool timing_enabled() { return g_tm_on.load(std::memory_order_relaxed); }

void timing_push(const char* name, hipEvent_t start, hipEvent_t stop) {
  std::lock_guard<std::mutex> lk(g_tm_mu);
  g_tm.push_back({name, start, stop});
}

}  // namespace gr

extern "C" {

const char* gr_last_error(void) { return gr::last_error(); }

int gr_version(void) { return GR_HSTU_ABI_VERSION; }

int gr_timing_enable(int on) {
  gr::g_tm_on.store(on != 0);
  return 0;
}

int gr_timing_query(const char* kernel, double* total_ms, int* launches) {
  GR_REQUIRE(kernel && total_ms && launches, "gr_timing_query: null pointer");
  std::lock_guard<std::mutex> lk(gr::g_tm_mu);
  double tot = 0.0;
  int n = 0;
  std::vector<gr::TimedPair> keep;
  for (auto& p : gr::g_tm) {
    if (p.name != kernel) {
      keep.push_back(p);
      continue;
    }
    float ms = 0.f;
    if (hipEventSynchronize(p.stop) == hipSuccess &&
        hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
      tot += ms;
      ++n;
    }
    (void)hipEventDestroy(p.start);
    (void)hipEventDestroy(p.stop);
  }
  gr::g_tm.swap(keep);
  *total_ms = tot;
  *launches = n;
  return 0;
}

int gr_timing_reset(void) {
  std::lock_guard<std::mutex> lk(gr::g_tm_mu);
  for (auto& p : gr::g_tm) {
    (void)hipEventDestroy(p.start);
    (void)hipEventDestroy(p.stop);
  }
  gr::g_tm.clear();
  return 0;
}

}  // extern "C"
