// runtime.hip — error plumbing and version for libfedhip.
#include <cstdarg>
#include <cstdio>

#include "fh_common.h"

namespace fh {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}
}  // namespace fh

extern "C" const char* fh_last_error(void) { return fh::g_last_error; }

// Lane streams (fedhip/lanes.py): a HIP stream with a dispatch priority, or restricted to
// a set of CUs.  Concurrent client lanes contend for CU slots; the critical (longest)
// lane's latency-bound kernels are starved behind the wide lanes' full-chip launches
// unless it is either dispatched first (priority) or owns CUs the others never use.
extern "C" int fh_stream_create(int32_t priority, const uint32_t* cu_mask, int32_t mask_words,
                                void** stream_out) {
    if (!stream_out) {
        fh::set_error("fh_stream_create: null output");
        return FH_E_INVALID;
    }
    hipStream_t s = nullptr;
    hipError_t e;
    if (cu_mask && mask_words > 0) {
        e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask);
    } else {
        e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
    }
    if (e != hipSuccess) {
        fh::set_error("fh_stream_create: %s", hipGetErrorString(e));
        return FH_E_LAUNCH;
    }
    *stream_out = (void*)s;
    return FH_OK;
}

extern "C" int fh_stream_destroy(void* stream) {
    hipError_t e = hipStreamDestroy((hipStream_t)stream);
    if (e != hipSuccess) {
        fh::set_error("fh_stream_destroy: %s", hipGetErrorString(e));
        return FH_E_LAUNCH;
    }
    return FH_OK;
}

// 0xMMmmpp
extern "C" int fh_version(void) { return 0x000200; }
