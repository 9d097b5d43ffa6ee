// C-ABI plumbing: thread-local last-error string and version query.
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

}  // namespace gr

extern "C" {

const char* gr_last_error(void) { return gr::last_error(); }

int gr_version(void) { return GR_HSTU_ABI_VERSION; }

}  // extern "C"
