// status.cpp — bprmf_last_error() and the fail() helper every entry point reports through.
// Host-only C++ (no HIP): the ingestion code and its sanitizer build (tests/sanitize) link it alone.
#include "status.h"

#include <stdarg.h>
#include <stdio.h>

#include <string>

#include "../../include/bprmf.h"

static thread_local std::string g_err;

namespace bprmf {
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
}  // namespace bprmf

extern "C" const char* bprmf_last_error(void) { return g_err.c_str(); }
