// status.h — the library's error reporting (host only, no HIP): fail() records a thread-local
// message for bprmf_last_error() (include/bprmf.h) and returns the status code.
#pragma once

namespace bprmf {
int fail(int code, const char* fmt, ...);
}  // namespace bprmf
