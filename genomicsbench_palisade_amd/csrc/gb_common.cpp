// gb_common.cpp -- error state and device selection shared by every gb_* entry point.
#include "gb_common.h"

#include "../../include/gb.h"

namespace gb {
static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
const char *last_error() { return g_err.c_str(); }
}  // namespace gb

extern "C" {
const char *gb_last_error(void) { return gb::last_error(); }

int gb_device_count(int *count) {
  GB_ARG(count, "gb_device_count: null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    *count = 0;
    gb::set_error("no HIP device visible (%s)", hipGetErrorString(e));
    return GB_ERR_NODEV;
  }
  *count = n;
  return GB_OK;
}

int gb_set_device(int device) {
  int n = 0;
  int st = gb_device_count(&n);
  if (st) return st;
  GB_ARG(device >= 0 && device < n, "gb_set_device: device %d out of range [0,%d)", device, n);
  GB_HIP(hipSetDevice(device));
  return GB_OK;
}

int gb_host_alloc(void **ptr, size_t bytes) {
  GB_ARG(ptr, "gb_host_alloc: null ptr");
  *ptr = nullptr;
  GB_HIP(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault));
  return GB_OK;
}

int gb_host_free(void *ptr) {
  if (ptr) GB_HIP(hipHostFree(ptr));
  return GB_OK;
}
}
