/* The C ABI of libgsm_amd.so for the Swift module CGsmAMD (include/ at the repository root), and
 * the few HIP runtime entry points the wrapper uses for device buffers and streams. */
#include "../../../include/gsm_renderer.h"
#include "../../../include/gsm_depthfirst.h"
#include "../../../include/gsm_debug.h"
#include "../../../include/gsm_multigpu.h"

#include <stddef.h>
/* hip_runtime_api.h subset (ROCm 7, C linkage), so the module needs no HIP include path */
typedef int gsm_hip_error;
extern gsm_hip_error hipMalloc(void **ptr, size_t size);
extern gsm_hip_error hipFree(void *ptr);
extern gsm_hip_error hipMemcpy(void *dst, const void *src, size_t size, int kind); /* 1 H2D, 2 D2H */
extern gsm_hip_error hipStreamCreate(void **stream);
extern gsm_hip_error hipStreamDestroy(void *stream);
extern gsm_hip_error hipStreamSynchronize(void *stream);
