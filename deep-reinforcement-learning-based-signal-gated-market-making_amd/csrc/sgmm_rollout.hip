// sgmm_rollout.hip -- the population-rollout hot path on gfx950.
//
// Reference semantics: evaluate_individual (Env/drl_engine.py:9-67) mapped
// over a GA population (drl_engine.py:104-115), FTPEnv.step
// (Env/market_env.py:22-67), TradingPolicy / AdversaryPolicy
// (models/model.py:5-57).
//
// Fitness path (sgmm_rollout_fitness) -- two kernels:
//
//  1. k_policy_table: the inventory feedback makes an episode a serial chain,
//     but the policy only sees (signal_t, inventory) and the inventory takes
//     at most 8 values (caps +-2 -> 5).  So the policy, the FPT fill test and
//     the reward are evaluated for EVERY (tick, inventory[, adversary flags])
//     state in parallel: one lane per tick, weights wave-uniform (scalar
//     loads), the fp32 MLP on the VALU (the f32 MFMA rate equals the VALU rate
//     on gfx950 and the 3->H->H->2 shapes pad badly onto 16x16x4 tiles, so
//     MFMA would add work, not speed).  Output per tick: 2 fill bits per state
//     (u64) and one float64 reward per state.
//
//  2. k_path_scan (one workgroup per episode): chunked parallel walk of the
//     5-state (20 with the adversary) transducer -- every chunk of 64 ticks is
//     walked from every start state, the chunk end-maps are chained, each
//     chunk is replayed from its true start -- and the selected rewards are
//     summed in the reference's sequential float64 order (bit-exact), trades
//     counted with a block reduction.
//
// Trace path (sgmm_rollout_trace): k_rollout_direct, one wave per episode,
// lane = hidden neuron, the literal step loop (independent second
// implementation; the tests require both paths to agree bit for bit).
#include "sgmm_device.h"
#include "sgmm_internal.h"

namespace sgmm {

constexpr int kTableBlock = 256;
constexpr int kChunk = 64;          // ticks per chunk in the path scan
constexpr int kSeg = 4096;          // ticks summed per LDS segment
constexpr int kScanBlock = 256;
constexpr int kMaxLen = 1 << 17;    // max ticks per episode (LDS end-map bound)

struct EpArrays {
    const int32_t* genome;
    const int32_t* adv;
    const int64_t* tick_off;
    const int32_t* len;
    const int64_t* step_off;
    const int32_t* param;
};

__device__ __forceinline__ int next_state(int s, int code, bool arl) {
    const int fb = code & 1, fs = code >> 1;
    if (!arl) return s + fb - fs;
    return (((s >> 2) + fb - fs) << 2) | (fs << 1) | fb;
}

// ------------------------------------------------------------------ table
template <int H, bool ARL>
__global__ __launch_bounds__(kTableBlock) void k_policy_table(
    sgmm_ticks tk, EpArrays ep, const sgmm_env_params* __restrict__ params,
    const float* __restrict__ mm, int64_t mm_stride, const float* __restrict__ adv,
    int64_t adv_stride, int32_t inv_min, int32_t nsi, uint64_t* __restrict__ fills,
    double* __restrict__ rew) {
    using L = GenomeLayout<H>;
    const int e = blockIdx.y;
    const int32_t T = ep.len[e];
    const int32_t t0 = blockIdx.x * kTableBlock;
    if (t0 >= T) return;  // block-uniform
    const int ns = ARL ? 4 * nsi : nsi;
    const sgmm_env_params p = params[ep.param[e]];
    const float* __restrict__ g = mm + (int64_t)ep.genome[e] * mm_stride;

    __shared__ int32_t lut[2][32];  // adversary (delta_a, delta_b) per state
    if (ARL) {
        const int ai = ep.adv ? ep.adv[e] : -1;
        if ((int)threadIdx.x < ns) {
            const int s = threadIdx.x;
            int32_t da = 0, db = 0;
            if (ai >= 0)
                adv_delta(adv + (int64_t)ai * adv_stride, p, inv_min + (s >> 2), (s >> 1) & 1,
                          s & 1, da, db);
            lut[0][s] = da;
            lut[1][s] = db;
        }
        __syncthreads();
    }
    const int32_t t = t0 + threadIdx.x;
    if (t >= T) return;

    const int64_t ti = ep.tick_off[e] + t;
    const float x0 = tk.s1n[ti], x1 = tk.s2n[ti];
    const double mid = tk.mid_next[ti], ask = tk.best_ask[ti], bid = tk.best_bid[ti];
    const double bmax = tk.buy_max[ti], smin = tk.sell_min[ti];

    // tick-dependent part of layer 1 (shared by every inventory state):
    // acc = b1; acc = fma(W1[j,0], s1n, acc); acc = fma(W1[j,1], s2n, acc)
    float pre[H];
#pragma unroll
    for (int j = 0; j < H; ++j)
        pre[j] = __builtin_fmaf(g[L::W1 + 3 * j + 1], x1,
                                __builtin_fmaf(g[L::W1 + 3 * j], x0, g[L::B1 + j]));

    const int64_t row = ep.step_off[e] + t;
    double* __restrict__ R = rew + row * ns;
    uint64_t fw = 0;
    for (int si = 0; si < nsi; ++si) {
        const int32_t inv = inv_min + si;
        const float x2 = (float)((double)inv / 2.0);  // drl_engine.py:35
        float h1[H];
#pragma unroll
        for (int j = 0; j < H; ++j) h1[j] = relu(__builtin_fmaf(g[L::W1 + 3 * j + 2], x2, pre[j]));
        float o0 = g[L::B3], o1 = g[L::B3 + 1];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            float a = g[L::B2 + j];
#pragma unroll
            for (int k = 0; k < H; ++k) a = __builtin_fmaf(g[L::W2 + j * H + k], h1[k], a);
            const float h2 = relu(a);
            o0 = __builtin_fmaf(g[L::W3 + j], h2, o0);
            o1 = __builtin_fmaf(g[L::W3 + H + j], h2, o1);
        }
        const int32_t oa = act_to_int(rintf(o0 * p.act_scale));  // drl_engine.py:38-39
        const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
        if (!ARL) {
            const StepOut so = ftp_step(p, inv, oa, ob, mid, ask, bid, bmax, smin);
            fw |= (uint64_t)(so.fill_buy | (so.fill_sell << 1)) << (2 * si);
            R[si] = so.reward;
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int s = 4 * si + q;
                const StepOut so = ftp_step(p, inv, oa + lut[0][s], ob + lut[1][s], mid, ask, bid,
                                            bmax, smin);
                fw |= (uint64_t)(so.fill_buy | (so.fill_sell << 1)) << (2 * s);
                R[s] = so.reward;
            }
        }
    }
    fills[row] = fw;
}

// ------------------------------------------------------------------ path scan
// Dynamic LDS: [kSeg doubles: selected rewards][nch*ns bytes: end maps][nch bytes: starts]
template <bool ARL>
__global__ __launch_bounds__(kScanBlock) void k_path_scan(
    EpArrays ep, const sgmm_env_params* __restrict__ params, int32_t inv_min, int32_t nsi,
    const uint64_t* __restrict__ fills, const double* __restrict__ rew,
    double* __restrict__ fitness, int32_t* __restrict__ trades_out) {
    extern __shared__ __align__(16) unsigned char lds[];
    double* sel = reinterpret_cast<double*>(lds);
    const int e = blockIdx.x;
    const int32_t T = ep.len[e];
    const int ns = ARL ? 4 * nsi : nsi;
    const int nch = (T + kChunk - 1) / kChunk;
    uint8_t* endmap = lds + kSeg * sizeof(double);
    uint8_t* start = endmap + nch * ns;
    __shared__ int red_trades;
    const int64_t so = ep.step_off[e];
    const uint64_t* __restrict__ F = fills + so;
    const double* __restrict__ R = rew + so * ns;
    const int tid = threadIdx.x;
    if (tid == 0) red_trades = 0;

    // phase 1: end state of every chunk from every start state
    for (int i = tid; i < nch * ns; i += kScanBlock) {
        const int k = i / ns;
        int s = i - k * ns;
        const int ta = k * kChunk, tb = min(T, ta + kChunk);
        for (int t = ta; t < tb; ++t) s = next_state(s, (int)(F[t] >> (2 * s)) & 3, ARL);
        endmap[i] = (uint8_t)s;
    }
    __syncthreads();
    // phase 2: chain the chunk maps from the initial state (inventory 0, no fills)
    if (tid == 0) {
        int s = ARL ? (-inv_min) << 2 : -inv_min;
        for (int k = 0; k < nch; ++k) {
            start[k] = (uint8_t)s;
            s = endmap[k * ns + s];
        }
    }
    __syncthreads();
    // phases 3+4 per segment: replay chunks from their true start selecting the
    // reward of the visited state, then sum in tick order.
    double total = 0.0;
    int my_trades = 0;
    for (int seg0 = 0; seg0 < T; seg0 += kSeg) {
        const int segn = min(kSeg, T - seg0);
        const int segch = (segn + kChunk - 1) / kChunk;
        if (tid < segch) {
            const int k = seg0 / kChunk + tid;
            int s = start[k];
            const int ta = k * kChunk, tb = min(T, ta + kChunk);
            for (int t = ta; t < tb; ++t) {
                const int code = (int)(F[t] >> (2 * s)) & 3;
                sel[t - seg0] = R[(int64_t)t * ns + s];
                my_trades += (code != 0);
                s = next_state(s, code, ARL);
            }
        }
        __syncthreads();
        if (tid == 0) {
            // reference order: total = ((r0 + r1) + r2) + ... (drl_engine.py:54)
            int t = 0;
            for (; t + 8 <= segn; t += 8) {
                const double2 a = *reinterpret_cast<const double2*>(sel + t);
                const double2 b = *reinterpret_cast<const double2*>(sel + t + 2);
                const double2 c = *reinterpret_cast<const double2*>(sel + t + 4);
                const double2 d = *reinterpret_cast<const double2*>(sel + t + 6);
                total += a.x; total += a.y; total += b.x; total += b.y;
                total += c.x; total += c.y; total += d.x; total += d.y;
            }
            for (; t < segn; ++t) total += sel[t];
        }
        __syncthreads();
    }
    // trades: integer, any order
    int w = my_trades;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off, kWave);
    if ((tid & (kWave - 1)) == 0 && w) atomicAdd(&red_trades, w);
    __syncthreads();
    if (tid == 0) {
        const int tr = red_trades;
        if (tr == 0) total -= params[ep.param[e]].idle_penalty;  // drl_engine.py:64-65
        fitness[e] = total;
        trades_out[e] = tr;
    }
}

// ------------------------------------------------------------------ direct (trace) path
struct TraceOut {
    int32_t *off_a, *off_b, *adv_a, *adv_b, *inventory;
    double *cash, *reward, *pnl, *fee_paid;
    uint8_t *fill_buy, *fill_sell;
    float *raw_a, *raw_b;
    double* fitness;
    int32_t* trades;
};

template <int H>
__global__ __launch_bounds__(kWave) void k_rollout_direct(
    sgmm_ticks tk, EpArrays ep, const sgmm_env_params* __restrict__ params,
    const float* __restrict__ mm, int64_t mm_stride, const float* __restrict__ adv,
    int64_t adv_stride, int32_t inv_min, int32_t nsi, TraceOut out) {
    using L = GenomeLayout<H>;
    const int e = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t T = ep.len[e];
    const int64_t to = ep.tick_off[e], so = ep.step_off[e];
    const sgmm_env_params p = params[ep.param[e]];
    const float* __restrict__ g = mm + (int64_t)ep.genome[e] * mm_stride;
    const int ai = (adv && ep.adv) ? ep.adv[e] : -1;

    __shared__ float sh1[H], sh2[H];
    __shared__ int32_t lut[2][32];
    // lane j < H owns hidden neuron j of both hidden layers
    float w1[3] = {0.f, 0.f, 0.f}, b1 = 0.f, b2 = 0.f, w2[H];
#pragma unroll
    for (int k = 0; k < H; ++k) w2[k] = 0.f;
    if (lane < H) {
        w1[0] = g[L::W1 + 3 * lane];
        w1[1] = g[L::W1 + 3 * lane + 1];
        w1[2] = g[L::W1 + 3 * lane + 2];
        b1 = g[L::B1 + lane];
        b2 = g[L::B2 + lane];
#pragma unroll
        for (int k = 0; k < H; ++k) w2[k] = g[L::W2 + lane * H + k];
    }
    if (ai >= 0 && lane < 4 * nsi) {
        int32_t da, db;
        adv_delta(adv + (int64_t)ai * adv_stride, p, inv_min + (lane >> 2), (lane >> 1) & 1,
                  lane & 1, da, db);
        lut[0][lane] = da;
        lut[1][lane] = db;
    }
    __syncthreads();

    int32_t inv = 0, trades = 0, fbp = 0, fsp = 0;
    double cash = 0.0, total = 0.0;
    for (int32_t t = 0; t < T; ++t) {
        const int64_t ti = to + t;
        const float x0 = tk.s1n[ti], x1 = tk.s2n[ti];
        const float x2 = (float)((double)inv / 2.0);
        if (lane < H) {
            float a = b1;
            a = __builtin_fmaf(w1[0], x0, a);
            a = __builtin_fmaf(w1[1], x1, a);
            a = __builtin_fmaf(w1[2], x2, a);
            sh1[lane] = relu(a);
        }
        __syncthreads();
        if (lane < H) {
            float a = b2;
#pragma unroll
            for (int k = 0; k < H; ++k) a = __builtin_fmaf(w2[k], sh1[k], a);
            sh2[lane] = relu(a);
        }
        __syncthreads();
        float o0 = g[L::B3], o1 = g[L::B3 + 1];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float h = sh2[j];
            o0 = __builtin_fmaf(g[L::W3 + j], h, o0);
            o1 = __builtin_fmaf(g[L::W3 + H + j], h, o1);
        }
        const int32_t oa = act_to_int(rintf(o0 * p.act_scale));
        const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
        int32_t da = 0, db = 0;
        if (ai >= 0) {
            const int s = ((inv - inv_min) << 2) | (fsp << 1) | fbp;
            da = lut[0][s];
            db = lut[1][s];
        }
        const StepOut st = ftp_step(p, inv, oa + da, ob + db, tk.mid_next[ti], tk.best_ask[ti],
                                    tk.best_bid[ti], tk.buy_max[ti], tk.sell_min[ti]);
        cash = apply_cash(cash, st);
        inv = st.inv;
        total += st.reward;
        trades += (st.fill_buy | st.fill_sell);
        fbp = st.fill_buy;
        fsp = st.fill_sell;
        if (lane == 0) {
            const int64_t r = so + t;
            if (out.off_a) out.off_a[r] = oa;
            if (out.off_b) out.off_b[r] = ob;
            if (out.adv_a) out.adv_a[r] = da;
            if (out.adv_b) out.adv_b[r] = db;
            if (out.inventory) out.inventory[r] = inv;
            if (out.cash) out.cash[r] = cash;
            if (out.reward) out.reward[r] = st.reward;
            if (out.pnl) out.pnl[r] = st.pnl;
            if (out.fee_paid) out.fee_paid[r] = st.fee_paid;
            if (out.fill_buy) out.fill_buy[r] = (uint8_t)st.fill_buy;
            if (out.fill_sell) out.fill_sell[r] = (uint8_t)st.fill_sell;
            if (out.raw_a) out.raw_a[r] = o0;
            if (out.raw_b) out.raw_b[r] = o1;
        }
    }
    if (lane == 0) {
        if (trades == 0) total -= p.idle_penalty;
        if (out.fitness) out.fitness[e] = total;
        if (out.trades) out.trades[e] = trades;
    }
}

// ------------------------------------------------------------------ batched primitives
template <int H>
__global__ void k_policy_forward(const float* __restrict__ genomes, int64_t stride,
                                 const int32_t* __restrict__ idx, const float* __restrict__ st,
                                 float* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* g = genomes + (int64_t)(idx ? idx[i] : i) * stride;
    float o0, o1;
    mlp_forward<H>(g, st[3 * i], st[3 * i + 1], st[3 * i + 2], o0, o1);
    out[2 * i] = o0;
    out[2 * i + 1] = o1;
}

__global__ void k_adversary_forward(const float* __restrict__ genomes, int64_t stride,
                                    const int32_t* __restrict__ idx, const float* __restrict__ st,
                                    float* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* g = genomes + (int64_t)(idx ? idx[i] : i) * stride;
    float o0, o1;
    adv_forward(g, st[3 * i], st[3 * i + 1], st[3 * i + 2], o0, o1);
    out[2 * i] = o0;
    out[2 * i + 1] = o1;
}

__global__ void k_env_step(const sgmm_env_params* __restrict__ params,
                           const int32_t* __restrict__ pidx, int32_t* __restrict__ inventory,
                           double* __restrict__ cash, const int32_t* __restrict__ action,
                           const int32_t* __restrict__ adv_action,
                           const double* __restrict__ mid, const double* __restrict__ ask,
                           const double* __restrict__ bid, const double* __restrict__ bmax,
                           const double* __restrict__ smin, double* __restrict__ reward,
                           double* __restrict__ pnl, double* __restrict__ inv_reward,
                           double* __restrict__ fee_paid, uint8_t* __restrict__ fill_buy,
                           uint8_t* __restrict__ fill_sell, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const sgmm_env_params p = params[pidx ? pidx[i] : 0];
    int32_t oa = action[2 * i], ob = action[2 * i + 1];
    if (adv_action) {  // market_env.py:25-28
        oa += adv_action[2 * i];
        ob += adv_action[2 * i + 1];
    }
    const StepOut so = ftp_step(p, inventory[i], oa, ob, mid[i], ask[i], bid[i], bmax[i], smin[i]);
    inventory[i] = so.inv;
    cash[i] = apply_cash(cash[i], so);
    if (reward) reward[i] = so.reward;
    if (pnl) pnl[i] = so.pnl;
    if (inv_reward) inv_reward[i] = -(p.phi * (double)(so.inv < 0 ? -so.inv : so.inv));
    if (fee_paid) fee_paid[i] = so.fee_paid;
    if (fill_buy) fill_buy[i] = (uint8_t)so.fill_buy;
    if (fill_sell) fill_sell[i] = (uint8_t)so.fill_sell;
}

// ------------------------------------------------------------------ host helpers
static int check_episodes(const sgmm_ticks* tk, const sgmm_episodes* eps, const void* params,
                          const float* mm, int32_t hidden) {
    SGMM_REQUIRE(tk && eps && params && mm, "null ticks/episodes/params/genomes");
    SGMM_REQUIRE(eps->n >= 0, "n episodes < 0");
    SGMM_REQUIRE(supported_hidden(hidden), "hidden=%d unsupported (8,16,32,64)", hidden);
    SGMM_REQUIRE(eps->max_len >= 0 && eps->max_len <= kMaxLen, "max_len=%d out of [0,%d]",
                 eps->max_len, kMaxLen);
    SGMM_REQUIRE(eps->inv_min <= 0 && eps->inv_max >= 0 && eps->inv_max - eps->inv_min + 1 <= 8,
                 "inventory range [%d,%d] must contain 0 and span <= 8 values", eps->inv_min,
                 eps->inv_max);
    if (eps->n > 0)
        SGMM_REQUIRE(eps->genome && eps->tick_off && eps->len && eps->step_off && eps->param,
                     "null episode array");
    SGMM_REQUIRE(tk->s1n && tk->s2n && tk->mid_next && tk->best_ask && tk->best_bid &&
                     tk->buy_max && tk->sell_min,
                 "null tick column");
    return SGMM_OK;
}

static EpArrays ep_arrays(const sgmm_episodes* e, bool with_adv) {
    return EpArrays{e->genome, with_adv ? e->adv : nullptr, e->tick_off, e->len, e->step_off,
                    e->param};
}

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace sgmm

using namespace sgmm;

extern "C" size_t sgmm_rollout_workspace_size(int32_t n_episodes, int64_t total_steps,
                                              int32_t n_states) {
    (void)n_episodes;
    if (total_steps < 0 || n_states <= 0) return 0;
    return align256((size_t)total_steps * sizeof(uint64_t)) +
           align256((size_t)total_steps * (size_t)n_states * sizeof(double));
}

template <int H>
static void launch_table(bool arl, dim3 grid, hipStream_t s, const sgmm_ticks& tk,
                         const EpArrays& ep, const sgmm_env_params* params, const float* mm,
                         int64_t mm_stride, const float* adv, int64_t adv_stride, int32_t inv_min,
                         int32_t nsi, uint64_t* fills, double* rew) {
    if (arl)
        hipLaunchKernelGGL((k_policy_table<H, true>), grid, dim3(kTableBlock), 0, s, tk, ep,
                           params, mm, mm_stride, adv, adv_stride, inv_min, nsi, fills, rew);
    else
        hipLaunchKernelGGL((k_policy_table<H, false>), grid, dim3(kTableBlock), 0, s, tk, ep,
                           params, mm, mm_stride, adv, adv_stride, inv_min, nsi, fills, rew);
}

extern "C" int sgmm_rollout_fitness(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                                    const sgmm_env_params* params, const float* mm_genomes,
                                    int64_t mm_stride, int32_t hidden, const float* adv_genomes,
                                    int64_t adv_stride, double* fitness, int32_t* trades,
                                    void* workspace, size_t workspace_bytes, void* stream) {
    clear_error();
    if (int rc = check_episodes(ticks, eps, params, mm_genomes, hidden)) return rc;
    SGMM_REQUIRE(fitness && trades, "null fitness/trades output");
    SGMM_REQUIRE(mm_stride >= (int64_t)hidden * hidden + 7 * hidden + 2, "mm_stride too small");
    const bool arl = adv_genomes != nullptr;
    SGMM_REQUIRE(!arl || adv_stride >= 74, "adv_stride < 74");
    if (eps->n == 0) return SGMM_OK;
    const int32_t nsi = eps->inv_max - eps->inv_min + 1;
    const int32_t ns = arl ? 4 * nsi : nsi;
    const size_t need = sgmm_rollout_workspace_size(eps->n, eps->total_steps, ns);
    if (!workspace || workspace_bytes < need) {
        set_error("workspace %zu bytes < required %zu", workspace_bytes, need);
        return SGMM_ERR_WORKSPACE;
    }
    uint64_t* fills = reinterpret_cast<uint64_t*>(workspace);
    double* rew = reinterpret_cast<double*>(reinterpret_cast<char*>(workspace) +
                                            align256((size_t)eps->total_steps * sizeof(uint64_t)));
    hipStream_t s = as_stream(stream);
    const EpArrays ep = ep_arrays(eps, arl);
    if (eps->max_len > 0) {
        dim3 grid((eps->max_len + kTableBlock - 1) / kTableBlock, eps->n);
        switch (hidden) {
            case 8: launch_table<8>(arl, grid, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, fills, rew); break;
            case 16: launch_table<16>(arl, grid, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, fills, rew); break;
            case 32: launch_table<32>(arl, grid, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, fills, rew); break;
            default: launch_table<64>(arl, grid, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, fills, rew); break;
        }
        SGMM_LAUNCHED();
    }
    const int nch_max = (eps->max_len + kChunk - 1) / kChunk;
    const size_t lds = kSeg * sizeof(double) + (size_t)nch_max * ns + nch_max;
    if (arl)
        hipLaunchKernelGGL(k_path_scan<true>, dim3(eps->n), dim3(kScanBlock), lds, s, ep, params,
                           eps->inv_min, nsi, fills, rew, fitness, trades);
    else
        hipLaunchKernelGGL(k_path_scan<false>, dim3(eps->n), dim3(kScanBlock), lds, s, ep, params,
                           eps->inv_min, nsi, fills, rew, fitness, trades);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_rollout_trace(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                                  const sgmm_env_params* params, const float* mm_genomes,
                                  int64_t mm_stride, int32_t hidden, const float* adv_genomes,
                                  int64_t adv_stride, int32_t* off_a, int32_t* off_b,
                                  int32_t* adv_a, int32_t* adv_b, int32_t* inventory,
                                  double* cash, double* reward, double* pnl_reward,
                                  double* fee_paid, uint8_t* fill_buy, uint8_t* fill_sell,
                                  float* raw_a, float* raw_b, double* fitness, int32_t* trades,
                                  void* stream) {
    clear_error();
    if (int rc = check_episodes(ticks, eps, params, mm_genomes, hidden)) return rc;
    SGMM_REQUIRE(mm_stride >= (int64_t)hidden * hidden + 7 * hidden + 2, "mm_stride too small");
    const bool arl = adv_genomes != nullptr;
    SGMM_REQUIRE(!arl || adv_stride >= 74, "adv_stride < 74");
    if (eps->n == 0) return SGMM_OK;
    const int32_t nsi = eps->inv_max - eps->inv_min + 1;
    TraceOut o{off_a, off_b, adv_a, adv_b, inventory, cash, reward, pnl_reward, fee_paid,
               fill_buy, fill_sell, raw_a, raw_b, fitness, trades};
    const EpArrays ep = ep_arrays(eps, arl);
    hipStream_t s = as_stream(stream);
    switch (hidden) {
        case 8: hipLaunchKernelGGL(k_rollout_direct<8>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
        case 16: hipLaunchKernelGGL(k_rollout_direct<16>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
        case 32: hipLaunchKernelGGL(k_rollout_direct<32>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
        default: hipLaunchKernelGGL(k_rollout_direct<64>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
    }
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_policy_forward(const float* genomes, int64_t genome_stride, int32_t hidden,
                                   const int32_t* genome_idx, const float* states, float* out,
                                   int64_t n, void* stream) {
    clear_error();
    SGMM_REQUIRE(genomes && states && out, "null pointer");
    SGMM_REQUIRE(n >= 0, "n < 0");
    SGMM_REQUIRE(supported_hidden(hidden), "hidden=%d unsupported (8,16,32,64)", hidden);
    SGMM_REQUIRE(genome_stride >= (int64_t)hidden * hidden + 7 * hidden + 2, "stride too small");
    if (n == 0) return SGMM_OK;
    const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
    hipStream_t s = as_stream(stream);
    switch (hidden) {
        case 8: hipLaunchKernelGGL(k_policy_forward<8>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
        case 16: hipLaunchKernelGGL(k_policy_forward<16>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
        case 32: hipLaunchKernelGGL(k_policy_forward<32>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
        default: hipLaunchKernelGGL(k_policy_forward<64>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
    }
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_adversary_forward(const float* genomes, int64_t genome_stride,
                                      const int32_t* genome_idx, const float* states, float* out,
                                      int64_t n, void* stream) {
    clear_error();
    SGMM_REQUIRE(genomes && states && out, "null pointer");
    SGMM_REQUIRE(n >= 0 && genome_stride >= 74, "bad n or stride");
    if (n == 0) return SGMM_OK;
    hipLaunchKernelGGL(k_adversary_forward, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), genomes, genome_stride, genome_idx, states, out, n);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_env_step_batch(const sgmm_env_params* params, const int32_t* param_idx,
                                   int32_t* inventory, double* cash, const int32_t* action,
                                   const int32_t* adv_action, const double* mid_next,
                                   const double* best_ask, const double* best_bid,
                                   const double* buy_max, const double* sell_min, double* reward,
                                   double* pnl_reward, double* inventory_reward, double* fee_paid,
                                   uint8_t* fill_buy, uint8_t* fill_sell, int64_t n,
                                   void* stream) {
    clear_error();
    SGMM_REQUIRE(params && inventory && cash && action && mid_next && best_ask && best_bid &&
                     buy_max && sell_min,
                 "null pointer");
    SGMM_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return SGMM_OK;
    hipLaunchKernelGGL(k_env_step, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), params, param_idx, inventory, cash, action, adv_action,
                       mid_next, best_ask, best_bid, buy_max, sell_min, reward, pnl_reward,
                       inventory_reward, fee_paid, fill_buy, fill_sell, n);
    SGMM_LAUNCHED();
    return SGMM_OK;
}
