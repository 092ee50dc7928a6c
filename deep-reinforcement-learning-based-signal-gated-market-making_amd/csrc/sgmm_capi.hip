// sgmm_capi.hip -- ABI version, thread-local error reporting, kernel timing.
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sgmm_internal.h"

namespace sgmm {

namespace {
thread_local char g_err[512] = "";

struct ProfRec {
    const char* kind;
    hipEvent_t a, b;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof;
std::vector<hipEvent_t> g_event_pool;
thread_local int g_open_slot = -1;  // slot of this thread's innermost open scope
thread_local bool g_open_taken = false;

hipEvent_t take_event() {
    if (!g_event_pool.empty()) {
        hipEvent_t e = g_event_pool.back();
        g_event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
}  // namespace

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

int prof_begin(const char* kind, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (!g_prof_on) return -1;
    ProfRec r{kind, take_event(), take_event()};
    if (!r.a || !r.b) return -1;
    (void)hipEventRecord(r.a, s);
    g_prof.push_back(r);
    g_open_slot = (int)g_prof.size() - 1;
    g_open_taken = false;
    return g_open_slot;
}

bool prof_take_events(hipEvent_t* start, hipEvent_t* stop) {
    if (g_open_slot < 0 || g_open_taken) return false;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (g_open_slot >= (int)g_prof.size()) return false;
    *start = g_prof[g_open_slot].a;
    *stop = g_prof[g_open_slot].b;
    g_open_taken = true;
    return true;
}

void prof_end(int slot, hipStream_t s) {
    if (slot < 0) return;
    const bool taken = slot == g_open_slot && g_open_taken;
    if (slot == g_open_slot) g_open_slot = -1;
    if (taken) return;  // the kernel's dispatch records both events
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (slot < (int)g_prof.size()) (void)hipEventRecord(g_prof[slot].b, s);
}

}  // namespace sgmm

using namespace sgmm;

extern "C" int sgmm_abi_version(void) { return SGMM_ABI_VERSION; }

extern "C" const char* sgmm_last_error(void) { return sgmm::g_err; }

extern "C" int sgmm_profile_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = enable != 0;
    return SGMM_OK;
}

extern "C" int sgmm_profile_read(int max_kinds, char* names, double* total_ms, int64_t* count) {
    clear_error();
    std::lock_guard<std::mutex> lk(g_prof_mu);
    std::vector<std::string> kinds;
    std::vector<double> tot;
    std::vector<int64_t> cnt;
    for (auto& r : g_prof) {
        if (hipEventSynchronize(r.b) != hipSuccess) {
            set_error("hipEventSynchronize failed");
            return SGMM_ERR_HIP;
        }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        size_t k = 0;
        while (k < kinds.size() && kinds[k] != r.kind) ++k;
        if (k == kinds.size()) {
            kinds.emplace_back(r.kind);
            tot.push_back(0.0);
            cnt.push_back(0);
        }
        tot[k] += ms;
        cnt[k] += 1;
        g_event_pool.push_back(r.a);
        g_event_pool.push_back(r.b);
    }
    g_prof.clear();
    const int n = (int)kinds.size() < max_kinds ? (int)kinds.size() : max_kinds;
    for (int i = 0; i < n; ++i) {
        if (names) {
            std::strncpy(names + 48 * i, kinds[i].c_str(), 47);
            names[48 * i + 47] = '\0';
        }
        if (total_ms) total_ms[i] = tot[i];
        if (count) count[i] = cnt[i];
    }
    return n;
}
