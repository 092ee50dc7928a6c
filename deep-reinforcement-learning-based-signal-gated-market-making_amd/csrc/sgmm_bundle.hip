// sgmm_bundle.hip -- the signal-bundle builder on gfx950:
// the data path that feeds the rollout, from raw snapshot / trade streams to
// the per-step bundle.  One workgroup per trading day; many days per launch.
//
// Reference semantics (HFTLoader.py / agent_trainer.py, restated and pinned in
// oracle/bundle_oracle.py against the reference's own outputs):
//   event bars   loaders/HFTLoader.py:26-63: a snapshot row is an event when
//                bid/ask price or volume differs from the previous row (the
//                first row always: diff() is NaN); trades are aggregated per
//                trade_time (max buy price, min sell price, volume sums, price
//                count, sum price*volume -- pandas' Kahan group sum, NaN
//                skipped, row order) and joined backward (merge_asof) onto
//                the events.
//   bar mids     loaders/HFTLoader.py:141-169 (SGU2DataPro): per 19-event
//                group 0.5*(max p_buy_max + min p_sell_min) with the pandas
//                mean fallbacks (numpy pairwise sum / 19), ffill, float32,
//                floor 1e-5, returns (m - m_lag)/(m_lag + 1e-9), 10-step
//                windows, nan_to_num.
//   step bundle  pipeline/agent_trainer.py:45-78: for the last n sampled
//                events (every 19th), the window max/min of the traded
//                extremes over the inclusive .loc range between consecutive
//                samples, ask/bid at the sample, mid at the next sample.
// HBM-bound integer/byte work: coalesced column reads, block scans in LDS for
// the compactions, no matrix cores.
#include <cmath>

#include "sgmm_device.h"
#include "sgmm_internal.h"

namespace sgmm {

constexpr int kDayBlock = 1024;

// exclusive block scan of one 0/1 flag per thread; returns the prefix and
// writes the block total to *total (all threads)
__device__ int block_scan_flags(bool flag, int* lds_wave, int& total) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid >> 6, nw = blockDim.x >> 6;
    const uint64_t b = __ballot(flag);
    const int in_wave = __popcll(b & ((1ull << lane) - 1));
    if (lane == 0) lds_wave[w] = __popcll(b);
    __syncthreads();
    int before = 0, tot = 0;
    for (int i = 0; i < nw; ++i) {
        const int c = lds_wave[i];
        before += i < w ? c : 0;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return before + in_wave;
}

__device__ __forceinline__ void kahan_add(double v, double& s, double& c) {
    if (v != v) return;  // NaN skipped
    const double y = v - c;
    const double t = s + y;
    c = (t - s) - y;
    if (c != c) c = 0.0;  // +-inf input (pandas GH#53606)
    s = t;
}

// workspace per tick slot: group start index + group stats
struct GroupWs {
    int32_t* start;   // [ticks] group g of day d starts at tick start[tick_off[d] + g]
    int64_t* time;
    double* st;       // [7][ticks]: bmax, smin, vbuy, vsell, vol, count, vwap
};

__global__ __launch_bounds__(kDayBlock) void k_event_bars(sgmm_day_streams in, sgmm_event_bars out,
                                                          GroupWs ws, int64_t tick_total) {
    __shared__ int lds_wave[kDayBlock / kWave];
    __shared__ int n_groups_s;
    const int d = blockIdx.x, tid = threadIdx.x;
    const int64_t t0 = in.tick_off[d], t1 = in.tick_off[d + 1];
    const int64_t s0 = in.snap_off[d], s1 = in.snap_off[d + 1];
    // 1. tick groups: one per distinct trade_time (ticks sorted by time)
    int ng = 0;
    for (int64_t base = t0; base < t1; base += kDayBlock) {
        const int64_t i = base + tid;
        const bool st = i < t1 && (i == t0 || in.tick_time[i] != in.tick_time[i - 1]);
        int tot;
        const int pos = block_scan_flags(st, lds_wave, tot);
        if (st) {
            ws.start[t0 + ng + pos] = (int32_t)(i - t0);
            ws.time[t0 + ng + pos] = in.tick_time[i];
        }
        ng += tot;
    }
    if (tid == 0) n_groups_s = ng;
    __syncthreads();
    ng = n_groups_s;
    // 2. per-group aggregates (HFTLoader.py:40-55), sequential within a group
    for (int g = tid; g < ng; g += kDayBlock) {
        const int64_t a = t0 + ws.start[t0 + g];
        const int64_t b = g + 1 < ng ? t0 + ws.start[t0 + g + 1] : t1;
        double bmax = NAN, smin = NAN, cnt = 0.0;
        double vb = 0.0, cb = 0.0, vs = 0.0, cs = 0.0, vv = 0.0, cv = 0.0, vw = 0.0, cw = 0.0;
        for (int64_t i = a; i < b; ++i) {
            const double p = in.price[i], v = in.volume[i];
            const int sd = in.side[i];
            if (sd == 1 && p == p) bmax = (bmax != bmax || p > bmax) ? p : bmax;
            if (sd == -1 && p == p) smin = (smin != smin || p < smin) ? p : smin;
            kahan_add(sd == 1 ? v : 0.0, vb, cb);
            kahan_add(sd == -1 ? v : 0.0, vs, cs);
            kahan_add(v, vv, cv);
            kahan_add(p * v, vw, cw);
            cnt += (p == p) ? 1.0 : 0.0;
        }
        double* st = ws.st + t0 + g;
        st[0 * tick_total] = bmax;
        st[1 * tick_total] = smin;
        st[2 * tick_total] = vb;
        st[3 * tick_total] = vs;
        st[4 * tick_total] = vv;
        st[5 * tick_total] = cnt;
        st[6 * tick_total] = vw;
    }
    __syncthreads();
    // 3. event rows (HFTLoader.py:32-36) and the backward as-of join (:60)
    int ne = 0;
    for (int64_t base = s0; base < s1; base += kDayBlock) {
        const int64_t i = base + tid;
        bool ev = false;
        if (i < s1) {
            ev = i == s0 || !(in.bid[i] - in.bid[i - 1] == 0.0) || !(in.ask[i] - in.ask[i - 1] == 0.0) ||
                 !(in.bidvol[i] - in.bidvol[i - 1] == 0.0) || !(in.askvol[i] - in.askvol[i - 1] == 0.0);
        }
        int tot;
        const int pos = block_scan_flags(ev, lds_wave, tot);
        if (ev) {
            const int64_t o = s0 + ne + pos;
            const int64_t t = in.snap_time[i];
            out.trade_time[o] = t;
            out.ask[o] = in.ask[i];
            out.bid[o] = in.bid[i];
            // last group with time <= t
            int lo = 0, hi = ng;  // first group with time > t
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (ws.time[t0 + mid] <= t) lo = mid + 1;
                else hi = mid;
            }
            const int g = lo - 1;
            double* dst[7] = {out.p_buy_max, out.p_sell_min, out.v_buy_sum, out.v_sell_sum, out.vol_sum,
                              out.trade_count, out.vwap_num};
#pragma unroll
            for (int k = 0; k < 7; ++k) dst[k][o] = g >= 0 ? ws.st[k * tick_total + t0 + g] : NAN;
        }
        ne += tot;
    }
    if (tid == 0) out.n_events[d] = ne;
}

// numpy's float64 add.reduce order for n in [8, 128): 8 strided accumulators,
// combined pairwise, then the tail in order
__device__ double pairwise_sum_19(const double* a) {
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = r[j] + a[8 + j];
    double s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    s = s + a[16];
    s = s + a[17];
    s = s + a[18];
    return s;
}

__device__ __forceinline__ double nan_max_run(const double* a, int n) {
    double m = NAN;
    for (int i = 0; i < n; ++i)
        if (a[i] == a[i]) m = (m != m || a[i] > m) ? a[i] : m;
    return m;
}

__device__ __forceinline__ double nan_min_run(const double* a, int n) {
    double m = NAN;
    for (int i = 0; i < n; ++i)
        if (a[i] == a[i]) m = (m != m || a[i] < m) ? a[i] : m;
    return m;
}

constexpr int kEventStep = 19, kTimeSteps = 10;
constexpr int kMaxBars = 4096;  // bars per day held in LDS (4096 * 19 events)

// SGU2DataPro.gen_dataset (HFTLoader.py:139-169) per day: X[w][k] = return
// k of window w (float32), y[w]; n_windows[d] = max(0, bars - 11)
__global__ __launch_bounds__(kDayBlock) void k_bar_windows(sgmm_event_bars ev, const int64_t* snap_off,
                                                           const int64_t* win_off, float* X, float* y,
                                                           int32_t* n_windows) {
    __shared__ double m[kMaxBars];
    __shared__ float ret[kMaxBars];
    __shared__ int last_valid[kMaxBars];
    const int d = blockIdx.x, tid = threadIdx.x;
    const int64_t e0 = snap_off[d];
    const int n_ev = ev.n_events[d];
    const int nb = n_ev > kEventStep ? (n_ev - kEventStep + kEventStep - 1) / kEventStep : 0;  // len(range(0, n-19, 19))
    if (nb > kMaxBars) {  // the host checks max_bars_per_day; never index past the LDS arrays
        if (tid == 0) n_windows[d] = -1;
        return;
    }
    for (int g = tid; g < nb; g += kDayBlock) {
        const int64_t a = e0 + (int64_t)g * kEventStep;
        const double bmax = nan_max_run(ev.p_buy_max + a, kEventStep);
        const double smin = nan_min_run(ev.p_sell_min + a, kEventStep);
        const double am = pairwise_sum_19(ev.ask + a) / kEventStep;
        const double bm = pairwise_sum_19(ev.bid + a) / kEventStep;
        double v;
        if (bmax == bmax && smin == smin) v = 0.5 * (bmax + smin);
        else if (smin == smin) v = 0.5 * (am + smin);
        else if (bmax == bmax) v = 0.5 * (bmax + bm);
        else v = 0.5 * (am + bm);
        m[g] = v;
    }
    __syncthreads();
    if (nb <= kTimeSteps + 1) {
        if (tid == 0) n_windows[d] = 0;
        return;
    }
    // ffill: index of the last non-NaN bar at or before g (sequential chunk scan)
    if (tid == 0) {
        int lv = -1;
        for (int g = 0; g < nb; ++g) {
            if (m[g] == m[g]) lv = g;
            last_valid[g] = lv;
        }
    }
    __syncthreads();
    for (int g = tid; g < nb; g += kDayBlock) {
        auto mf = [&](int k) -> float {
            const int lv = last_valid[k];
            float f = lv >= 0 ? (float)m[lv] : NAN;
            return f < 1e-5f ? 1e-5f : f;  // NaN stays NaN
        };
        if (g == 0) continue;
        const float cur = mf(g), lag = mf(g - 1);
        ret[g - 1] = (cur - lag) / (lag + 1e-9f);  // ret_np = returns[1:]
    }
    __syncthreads();
    const int nr = nb - 1, nw = nr - kTimeSteps;
    const int64_t w0 = win_off[d];
    for (int idx = tid; idx < nw * kTimeSteps; idx += kDayBlock) {
        const int w = idx / kTimeSteps, k = idx % kTimeSteps;
        const float v = ret[w + k];
        X[(w0 + w) * kTimeSteps + k] = v != v ? 0.0f : (isinf(v) ? (v > 0 ? 3.4028234663852886e38f : -3.4028234663852886e38f) : v);
    }
    for (int w = tid; w < nw; w += kDayBlock) {
        const float v = ret[w + kTimeSteps];
        y[w0 + w] = v != v ? 0.0f : (isinf(v) ? (v > 0 ? 3.4028234663852886e38f : -3.4028234663852886e38f) : v);
    }
    if (tid == 0) n_windows[d] = nw;
}

// agent_trainer.py:45-78 per day: the last n_samples sampled events (every
// 19th); step i = samples i -> i+1
__global__ void k_step_bundle(sgmm_event_bars ev, const int64_t* snap_off, const int32_t* n_samples,
                              const int64_t* step_off, double* mid, double* ask, double* bid,
                              double* buy_max, double* sell_min) {
    const int d = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n_ev = ev.n_events[d];
    const int ns = n_samples[d];
    if (i >= ns - 1) return;
    const int total = (n_ev + kEventStep - 1) / kEventStep;  // len(event_df.iloc[::19])
    const int64_t e0 = snap_off[d];
    const int64_t p = e0 + (int64_t)(total - ns + i) * kEventStep, q = p + kEventStep;
    const int64_t o = step_off[d] + i;
    buy_max[o] = nan_max_run(ev.p_buy_max + p, kEventStep + 1);  // .loc[p:q] is inclusive
    sell_min[o] = nan_min_run(ev.p_sell_min + p, kEventStep + 1);
    ask[o] = ev.ask[p];
    bid[o] = ev.bid[p];
    mid[o] = (ev.ask[q] + ev.bid[q]) / 2.0;
}

}  // namespace sgmm

using namespace sgmm;

extern "C" size_t sgmm_event_bars_workspace_size(int64_t total_ticks) {
    const size_t n = (size_t)(total_ticks > 0 ? total_ticks : 1);
    return ((n * sizeof(int32_t) + 255) & ~size_t(255)) + ((n * sizeof(int64_t) + 255) & ~size_t(255)) +
           7 * n * sizeof(double);
}

extern "C" int sgmm_event_bars_build(const sgmm_day_streams* in, const sgmm_event_bars* out,
                                     void* workspace, size_t workspace_bytes, void* stream) {
    clear_error();
    SGMM_REQUIRE(in && out, "null streams / outputs");
    SGMM_REQUIRE(in->n_days >= 0, "n_days < 0");
    if (in->n_days == 0) return SGMM_OK;
    SGMM_REQUIRE(in->snap_off && in->snap_time && in->bid && in->ask && in->bidvol && in->askvol &&
                     in->tick_off && in->tick_time && in->price && in->volume && in->side,
                 "null input column");
    SGMM_REQUIRE(out->n_events && out->trade_time && out->ask && out->bid && out->p_buy_max &&
                     out->p_sell_min && out->v_buy_sum && out->v_sell_sum && out->vol_sum &&
                     out->trade_count && out->vwap_num,
                 "null output column");
    SGMM_REQUIRE(in->tick_total >= 0, "tick_total < 0");
    const size_t need = sgmm_event_bars_workspace_size(in->tick_total);
    if (!workspace || workspace_bytes < need) {
        set_error("workspace %zu bytes < required %zu", workspace_bytes, need);
        return SGMM_ERR_WORKSPACE;
    }
    const size_t n = (size_t)(in->tick_total > 0 ? in->tick_total : 1);
    char* w = reinterpret_cast<char*>(workspace);
    GroupWs ws;
    ws.start = reinterpret_cast<int32_t*>(w);
    w += (n * sizeof(int32_t) + 255) & ~size_t(255);
    ws.time = reinterpret_cast<int64_t*>(w);
    w += (n * sizeof(int64_t) + 255) & ~size_t(255);
    ws.st = reinterpret_cast<double*>(w);
    ProfScope prof("event_bars", as_stream(stream));
    hipLaunchKernelGGL(k_event_bars, dim3(in->n_days), dim3(kDayBlock), 0, as_stream(stream), *in, *out,
                       ws, (int64_t)n);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_bar_windows(const sgmm_event_bars* ev, int32_t n_days, const int64_t* snap_off,
                                const int64_t* win_off, float* X, float* y, int32_t* n_windows,
                                int64_t max_bars_per_day, void* stream) {
    clear_error();
    SGMM_REQUIRE(ev && snap_off && win_off && X && y && n_windows, "null argument");
    SGMM_REQUIRE(max_bars_per_day <= kMaxBars, "more than %d bars per day", kMaxBars);
    if (n_days <= 0) return SGMM_OK;
    ProfScope prof("bar_windows", as_stream(stream));
    hipLaunchKernelGGL(k_bar_windows, dim3(n_days), dim3(kDayBlock), 0, as_stream(stream), *ev, snap_off,
                       win_off, X, y, n_windows);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_step_bundle(const sgmm_event_bars* ev, int32_t n_days, const int64_t* snap_off,
                                const int32_t* n_samples, const int64_t* step_off, int32_t max_steps,
                                double* mid, double* ask, double* bid, double* buy_max, double* sell_min,
                                void* stream) {
    clear_error();
    SGMM_REQUIRE(ev && snap_off && n_samples && step_off && mid && ask && bid && buy_max && sell_min,
                 "null argument");
    if (n_days <= 0 || max_steps <= 0) return SGMM_OK;
    ProfScope prof("step_bundle", as_stream(stream));
    hipLaunchKernelGGL(k_step_bundle, dim3((max_steps + 255) / 256, n_days), dim3(256), 0,
                       as_stream(stream), *ev, snap_off, n_samples, step_off, mid, ask, bid, buy_max,
                       sell_min);
    SGMM_LAUNCHED();
    return SGMM_OK;
}
