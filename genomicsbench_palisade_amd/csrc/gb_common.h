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

// Synchronous copy in pieces of at most 1 GiB, for the copies that can pass 4 GiB (index tables,
// SMEM and coordinate read-backs): no single transfer's size field reaches 32 bits.
inline hipError_t memcpy_big(void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
  constexpr size_t kPiece = size_t(1) << 30;
  for (size_t o = 0; o < bytes; o += kPiece) {
    const size_t b = bytes - o < kPiece ? bytes - o : kPiece;
    const hipError_t e = hipMemcpy(static_cast<char *>(dst) + o, static_cast<const char *>(src) + o, b, kind);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// roctx range around a host entry point (visible in rocprofv3 --marker-trace; a no-op otherwise)
struct Range {
  explicit Range(const char *name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
  Range(const Range &) = delete;
  Range &operator=(const Range &) = delete;
};

}  // namespace gb
