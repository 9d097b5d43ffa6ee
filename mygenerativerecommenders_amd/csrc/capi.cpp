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

// ---------------------------------------------------------------- launch options
static std::atomic<int64_t> g_opt[GR_OPT_COUNT_] = {0, 0, 0, 0, 0, 0, 1, 1, 1, 0, 0, 1, 1, 0, 1, 0, 1, 1};
// Per-thread overrides (gr_set_thread_option): bit i of t_set = option i overridden on this
// thread.  A launch and the workspace query before it read the same thread's values, so
// threads that use different options never see each other's.
static thread_local int64_t t_opt[GR_OPT_COUNT_];
static thread_local uint32_t t_set = 0u;
static_assert(GR_OPT_COUNT_ <= 32, "t_set holds one bit per option");

int64_t option(int which) {
  if ((t_set >> which) & 1u) return t_opt[which];
  return g_opt[which].load(std::memory_order_relaxed);
}

static int check_option(int option, int64_t value) {
  GR_REQUIRE(option > 0 && option < GR_OPT_COUNT_, "gr_set_option: unknown option %d", option);
  GR_REQUIRE(option != GR_OPT_MIPS_FILTER_WGS || (value >= 0 && value <= 16),
             "gr_set_option: filter WGs per CU %lld not in [0, 16]", (long long)value);
  GR_REQUIRE(value >= 0, "gr_set_option: negative value %lld", (long long)value);
  return 0;
}

// ---------------------------------------------------------------- live kernel timing
struct TimedPair {
  std::string name;
  hipEvent_t start, stop;
};
static std::mutex g_tm_mu;
static std::vector<TimedPair> g_tm;
static std::atomic<bool> g_tm_on{false};

bool timing_enabled() { return g_tm_on.load(std::memory_order_relaxed); }

const char*& timing_region() {
  static thread_local const char* name = nullptr;
  return name;
}

void timing_push(const char* name, hipEvent_t start, hipEvent_t stop) {
  std::lock_guard<std::mutex> lk(g_tm_mu);
  g_tm.push_back({name, start, stop});
}

}  // namespace gr

extern "C" {

const char* gr_last_error(void) { return gr::last_error(); }

int gr_version(void) { return GR_HSTU_ABI_VERSION; }

int gr_set_option(int option, int64_t value) {
  if (gr::check_option(option, value)) return 1;
  gr::g_opt[option].store(value, std::memory_order_relaxed);
  return 0;
}

int gr_set_thread_option(int option, int64_t value) {
  if (gr::check_option(option, value)) return 1;
  gr::t_opt[option] = value;
  gr::t_set |= 1u << option;
  return 0;
}

int gr_clear_thread_option(int option) {
  GR_REQUIRE(option >= 0 && option < GR_OPT_COUNT_, "gr_clear_thread_option: unknown option %d", option);
  if (option == 0)
    gr::t_set = 0u;
  else
    gr::t_set &= ~(1u << option);
  return 0;
}

int64_t gr_get_option(int option) {
  if (option <= 0 || option >= GR_OPT_COUNT_) return -1;
  return gr::option(option);
}

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
