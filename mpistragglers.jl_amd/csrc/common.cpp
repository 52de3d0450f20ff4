#include <atomic>

#include "comm.hpp"
#include "common.hpp"

namespace mpa {

static thread_local std::string g_err;
std::atomic<int64_t> g_timer_pending{0};

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
}

const char* last_error() { return g_err.c_str(); }

void fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  throw Failure{code};
}

}  // namespace mpa
