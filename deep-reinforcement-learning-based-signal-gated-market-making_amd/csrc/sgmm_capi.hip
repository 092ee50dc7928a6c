// sgmm_capi.hip -- ABI version and thread-local error reporting.
#include "sgmm_internal.h"

namespace sgmm {

namespace {
thread_local char g_err[512] = "";
}

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

}  // namespace sgmm

extern "C" int sgmm_abi_version(void) { return SGMM_ABI_VERSION; }

extern "C" const char* sgmm_last_error(void) { return sgmm::g_err; }
