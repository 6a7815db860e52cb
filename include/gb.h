/*
 * gb.h -- common part of the MI355X GenomicsBench C ABI (status codes, device selection).
 * Every gb_* function returns 0 on success or a negative gb_status; gb_last_error() describes the
 * last failure on the calling thread.
 */
#ifndef GB_H
#define GB_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum gb_status {
  GB_OK = 0,
  GB_ERR_ARG = -1,
  GB_ERR_HIP = -2,
  GB_ERR_NODEV = -3,
  GB_ERR_NOMEM = -4,
  GB_ERR_STATE = -5,
};

const char *gb_last_error(void);
int gb_device_count(int *count);
/* Select the HIP device for subsequent gb_* calls on this thread (objects stay bound to the
 * device that was current when they were created). */
int gb_set_device(int device);
/* Page-locked host memory (hipHostMalloc), for the C++ drop-ins' staging buffers: copies from it to
 * the device run at DMA rate instead of through the runtime's pageable bounce buffers. */
int gb_host_alloc(void **ptr, size_t bytes);
int gb_host_free(void *ptr);

#ifdef __cplusplus
}
#endif
#endif /* GB_H */
