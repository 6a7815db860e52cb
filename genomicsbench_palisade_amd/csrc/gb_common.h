// gb_common.h -- shared host-side plumbing for the C ABI (error state, HIP checks).
#pragma once
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <cstdarg>
#include <cstdio>
#include <string>

namespace gb {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
const char *last_error();

// Returns from the enclosing int-returning function with GB_ERR_HIP on failure.
#define GB_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::gb::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                      __LINE__);                                                        \
      return GB_ERR_HIP;                                                                \
    }                                                                                   \
  } while (0)

#define GB_ARG(cond, ...)          \
  do {                             \
    if (!(cond)) {                 \
      ::gb::set_error(__VA_ARGS__); \
      return GB_ERR_ARG;           \
    }                              \
  } while (0)

// roctx range around a host entry point (visible in rocprofv3 --marker-trace; a no-op otherwise)
struct Range {
  explicit Range(const char *name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
  Range(const Range &) = delete;
  Range &operator=(const Range &) = delete;
};

}  // namespace gb
