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

// 0xMMmmpp
extern "C" int fh_version(void) { return 0x000100; }
