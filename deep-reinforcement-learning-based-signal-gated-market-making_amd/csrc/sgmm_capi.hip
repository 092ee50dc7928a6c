// sgmm_capi.hip -- ABI version, thread-local error reporting, kernel timing.
#include <atomic>
#include <climits>
#include <cstdlib>
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
// launch-plan overrides (sgmm_plan_set), -1 = the default rule
std::atomic<int32_t> g_plan[SGMM_PLAN_N];
std::once_flag g_plan_once;
void plan_init() {
    for (auto& v : g_plan) v.store(-1, std::memory_order_relaxed);
#ifdef SGMM_EXPERIMENTS
    // the A/B variant build: initial values from the environment (tools/)
    auto env = [](const char* n) -> int32_t {
        const char* v = std::getenv(n);
        return v && *v ? (int32_t)std::atoi(v) : -1;
    };
    if (const char* v = std::getenv("SGMM_TABLE_PATH")) {
        const int32_t p = !std::strcmp(v, "frontier") ? 1 : !std::strcmp(v, "table") ? 2 : !std::strcmp(v, "valu") ? 3 : -1;
        g_plan[SGMM_PLAN_POLICY_PATH].store(p);
    }
    g_plan[SGMM_PLAN_GROUPS].store(env("SGMM_FRONTIER_NW"));
    g_plan[SGMM_PLAN_LANE_SPLIT].store(env("SGMM_FRONTIER_LS"));
    g_plan[SGMM_PLAN_TAIL].store(env("SGMM_FRONTIER_TAIL"));
    g_plan[SGMM_PLAN_FOUR].store(env("SGMM_FRONTIER_FOUR"));
    g_plan[SGMM_PLAN_MIN_EPS].store(env("SGMM_FRONTIER_MIN_EPS"));
    g_plan[SGMM_PLAN_TABLE_SP].store(env("SGMM_TABLE_SP"));
    g_plan[SGMM_PLAN_SCAN_THREADS].store(env("SGMM_SCAN_THREADS"));
    g_plan[SGMM_PLAN_SPILL].store(env("SGMM_FRONTIER_SPILL"));
    g_plan[SGMM_PLAN_SEQ_SUM].store(env("SGMM_SEQ_SUM"));
    g_plan[SGMM_PLAN_FUSED_SCAN].store(env("SGMM_FUSED_SCAN"));
    g_plan[SGMM_PLAN_LANES_SCAN].store(env("SGMM_LANES_SCAN"));
    if (const char* v = std::getenv("SGMM_REORDER_WEIGHTS")) {
        unsigned a = 0, b = 0;
        if (std::sscanf(v, "%u,%u", &a, &b) == 2 && a > 0 && b > 0 && a < 64 && b < 64)
            g_plan[SGMM_PLAN_REORDER_WEIGHTS].store((int32_t)(a << 8 | b));
    }
#endif
}
}  // namespace

int32_t plan_value(int k) {
    std::call_once(g_plan_once, plan_init);
    return (k >= 0 && k < SGMM_PLAN_N) ? g_plan[k].load(std::memory_order_relaxed) : -1;
}

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

extern "C" int sgmm_plan_set(int32_t knob, int32_t value) {
    clear_error();
    SGMM_REQUIRE(knob >= 0 && knob < SGMM_PLAN_N, "unknown plan knob %d", knob);
    (void)plan_value(knob);  // initialised
    g_plan[knob].store(value < 0 ? -1 : value, std::memory_order_relaxed);
    return SGMM_OK;
}

extern "C" int sgmm_plan_get(int32_t knob) {
    clear_error();
    if (knob < 0 || knob >= SGMM_PLAN_N) {
        set_error("unknown plan knob %d", knob);
        return INT32_MIN;
    }
    return plan_value(knob);
}

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
