// sgmm_internal.h -- host-side helpers shared by the C-ABI translation units.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/sgmm.h"

namespace sgmm {

void set_error(const char* fmt, ...);
void clear_error();

#define SGMM_REQUIRE(cond, ...)                     \
    do {                                            \
        if (!(cond)) {                              \
            ::sgmm::set_error(__VA_ARGS__);         \
            return SGMM_ERR_ARG;                    \
        }                                           \
    } while (0)

#define SGMM_HIP(call)                                                              \
    do {                                                                            \
        hipError_t err_ = (call);                                                   \
        if (err_ != hipSuccess) {                                                   \
            ::sgmm::set_error("%s failed: %s", #call, hipGetErrorString(err_));     \
            return SGMM_ERR_HIP;                                                    \
        }                                                                           \
    } while (0)

#define SGMM_LAUNCHED()                                                             \
    do {                                                                            \
        hipError_t err_ = hipGetLastError();                                        \
        if (err_ != hipSuccess) {                                                   \
            ::sgmm::set_error("kernel launch failed: %s", hipGetErrorString(err_)); \
            return SGMM_ERR_HIP;                                                    \
        }                                                                           \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel-timing hooks (sgmm_profile_enable).  prof_begin returns a slot
// (or -1 when profiling is off) that prof_end closes on the same stream.
// A kernel launched inside the scope with SGMM_LAUNCH takes the slot's events
// into its own dispatch (hipExtLaunchKernel), so the slot then times the kernel
// itself rather than the span between two stream markers.
int prof_begin(const char* kind, hipStream_t s);
void prof_end(int slot, hipStream_t s);
bool prof_take_events(hipEvent_t* start, hipEvent_t* stop);

#define SGMM_LAUNCH(kernel, grid, block, lds, stream, ...)                                       \
    do {                                                                                         \
        hipEvent_t ev_a_, ev_b_;                                                                 \
        if (::sgmm::prof_take_events(&ev_a_, &ev_b_))                                            \
            hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, ev_a_, ev_b_, 0, __VA_ARGS__); \
        else                                                                                     \
            hipLaunchKernelGGL(kernel, grid, block, lds, stream, __VA_ARGS__);                   \
    } while (0)

struct ProfScope {
    int slot;
    hipStream_t s;
    ProfScope(const char* kind, hipStream_t st) : slot(prof_begin(kind, st)), s(st) {}
    ~ProfScope() { prof_end(slot, s); }
};

inline bool supported_hidden(int h) { return h == 8 || h == 16 || h == 32 || h == 64; }

// Launch-plan override of knob k (SGMM_PLAN_*), or -1 for the default rule
// (sgmm_plan_set; the -DSGMM_EXPERIMENTS build seeds them from SGMM_* variables)
int32_t plan_value(int k);

}  // namespace sgmm
