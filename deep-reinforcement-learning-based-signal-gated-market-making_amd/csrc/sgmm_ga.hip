// sgmm_ga.hip -- the neuroevolution loop's bookkeeping on device, so a whole
// generation (ask -> rollout -> tell -> validation update) is enqueued
// without a host round trip.
//
// Reference: NeuroEvolution.ask/tell (models/model.py:59-76) and the
// generation body of DRLEngine.train (Env/drl_engine.py:92-171).
#include <cmath>

#include "sgmm_device.h"
#include "sgmm_ga_device.h"
#include "sgmm_internal.h"

namespace sgmm {

__global__ void k_ga_ask(const float* __restrict__ master, int64_t n_params,
                         const sgmm_ga_state* __restrict__ st, uint32_t sid, uint64_t seed,
                         int32_t i0, int32_t n, float* __restrict__ out, int64_t out_stride) {
    const int64_t nk4 = (n_params + 3) / 4;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nk4 * n) return;
    const int32_t i = (int32_t)(g / nk4);
    const int64_t k4 = g - (int64_t)i * nk4;
    const float sig = (float)(sid == 0 ? st->sigma_mm : st->sigma_adv);
    float v[4];
    ask_row4(master, n_params, sig, seed, sid, (uint32_t)st->gen, (uint32_t)(i0 + i), k4, v);
    float* row = out + (int64_t)i * out_stride;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (4 * k4 + q < n_params) row[4 * k4 + q] = v[q];
}

constexpr int kTellBlock = 256;

__global__ __launch_bounds__(kTellBlock) void k_ga_tell(
    sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
    const int32_t* __restrict__ trades, int32_t P, float* __restrict__ master_mm,
    const float* __restrict__ pop_mm, int64_t pop_mm_stride, float* __restrict__ master_adv,
    const float* __restrict__ pop_adv, int64_t pop_adv_stride, int64_t n_mm, int64_t n_adv,
    uint64_t seed, sgmm_ga_history* __restrict__ history, int32_t hist_cap) {
    __shared__ double sv[2][kTellBlock];
    const uint32_t gen = (uint32_t)st->gen;
    sgmm_ga_history* hist = (history && st->gen < hist_cap) ? history + st->gen : nullptr;
    __shared__ int si[2][kTellBlock];
    const int tid = threadIdx.x;
    double bv = 0.0, av = 0.0;
    int bi = -1, aj = -1;
    for (int i = tid; i < P; i += kTellBlock) {
        const double f = fit[i];
        if (bi < 0 || better(f, i, bv, bi)) { bv = f; bi = i; }
        if (aj < 0 || better(-f, i, av, aj)) { av = -f; aj = i; }
    }
    sv[0][tid] = bv; si[0][tid] = bi;
    sv[1][tid] = av; si[1][tid] = aj;
    __syncthreads();
    for (int w = kTellBlock / 2; w > 0; w >>= 1) {
        if (tid < w) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int io = si[r][tid + w];
                if (io >= 0 && (si[r][tid] < 0 || better(sv[r][tid + w], io, sv[r][tid], si[r][tid]))) {
                    sv[r][tid] = sv[r][tid + w];
                    si[r][tid] = io;
                }
            }
        }
        __syncthreads();
    }
    const int best = si[0][0], abest = si[1][0];
    const double sig_mm = st->sigma_mm, sig_adv = st->sigma_adv;
    __syncthreads();
    // new masters (model.py:75): copy the host-supplied row, or regenerate
    // the ask() of that individual in place (counter-based RNG)
    const int64_t nk_mm = (n_mm + 3) / 4;
    for (int64_t k4 = tid; k4 < nk_mm; k4 += kTellBlock) {
        if (pop_mm) {
            for (int q = 0; q < 4; ++q)
                if (4 * k4 + q < n_mm) master_mm[4 * k4 + q] = pop_mm[best * pop_mm_stride + 4 * k4 + q];
        } else {
            float v[4];
            ask_row4(master_mm, n_mm, (float)sig_mm, seed, 0u, gen, (uint32_t)best, k4, v);
            for (int q = 0; q < 4; ++q)
                if (4 * k4 + q < n_mm) master_mm[4 * k4 + q] = v[q];
        }
    }
    if (master_adv) {
        const int64_t nk_adv = (n_adv + 3) / 4;
        for (int64_t k4 = tid; k4 < nk_adv; k4 += kTellBlock) {
            if (pop_adv) {
                for (int q = 0; q < 4; ++q)
                    if (4 * k4 + q < n_adv) master_adv[4 * k4 + q] = pop_adv[abest * pop_adv_stride + 4 * k4 + q];
            } else {
                float v[4];
                ask_row4(master_adv, n_adv, (float)sig_adv, seed, 1u, gen, (uint32_t)abest, k4, v);
                for (int q = 0; q < 4; ++q)
                    if (4 * k4 + q < n_adv) master_adv[4 * k4 + q] = v[q];
            }
        }
    }
    if (tid == 0) {
        st->best_idx = best;
        st->adv_best_idx = abest;
        st->last_train_f = fit[best];
        if (hist) {
            hist->train_f = fit[best];
            hist->train_trades = trades ? trades[best] : 0;
            hist->best_idx = best;
        }
    }
}

__global__ __launch_bounds__(kTellBlock) void k_ga_val_update(
    sgmm_ga_state* __restrict__ st, const double* __restrict__ vfit,
    const int32_t* __restrict__ vtrades, int32_t use_best, const float* __restrict__ master,
    float* __restrict__ best_master, int64_t n, sgmm_ga_history* __restrict__ history,
    int32_t hist_cap) {
    __shared__ int improved;
    const int idx = use_best ? st->best_idx : 0;
    val_update_dev(st, vfit[idx], vtrades ? vtrades[idx] : 0, master, best_master, n, history, hist_cap,
                   &improved);
}

__global__ void k_ga_state_init(sgmm_ga_state* st, double sigma, int32_t patience, double decay) {
    st->sigma_mm = sigma;
    st->sigma_adv = sigma;
    st->best_val = -INFINITY;
    st->last_train_f = 0.0;
    st->last_val_f = 0.0;
    st->no_improve = 0;
    st->best_idx = -1;
    st->adv_best_idx = -1;
    st->gen = 0;
    st->improved = 0;
    st->decayed = 0;
    st->patience = patience;
    st->arrivals = 0;
    st->decay = decay;
}

__global__ __launch_bounds__(kStepBlock) void k_ga_step(
    sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
    const int32_t* __restrict__ trades, const double* __restrict__ vfit,
    const int32_t* __restrict__ vtrades, int32_t P, ShardView shard, float* __restrict__ master,
    float* __restrict__ master_adv, float* __restrict__ best_master, int64_t n_mm, int64_t n_adv,
    uint64_t seed, sgmm_ga_history* __restrict__ history, int32_t hist_cap,
    float* __restrict__ next_mm, float* __restrict__ next_adv, int32_t i0, int32_t n) {
    __shared__ double sv[2 * kStepBlock];
    __shared__ int si[2 * kStepBlock];
    __shared__ float lm[kMaxStepParams];
    __shared__ float la[kMaxStepParams];
    ga_step_dev<false>(st, fit, trades, vfit, vtrades, P, shard, master, master_adv, best_master, n_mm,
                n_adv, seed, history, hist_cap, next_mm, next_adv, i0, n, sv, si, lm, la);
}

// One workgroup per population (sgmm_ga_step_multi): population k's records
// at byte offsets k * fit_ps / k * tr_ps, its state / masters / history / key
// at index k.
struct PopsArg {
    sgmm_ga_state* states;
    float* masters_mm;
    float* masters_adv;
    float* best_masters;
    const uint64_t* seeds;
    sgmm_ga_history* history;
    int32_t hist_cap;
    int32_t P;
    int64_t n_mm, n_adv;
};

template <class T>
__device__ __forceinline__ const T* at_bytes(const T* p, int64_t off) {
    return p ? reinterpret_cast<const T*>(reinterpret_cast<const char*>(p) + off) : nullptr;
}

__global__ __launch_bounds__(kStepBlock) void k_ga_step_multi(
    PopsArg pa, const double* __restrict__ fit, const int32_t* __restrict__ trades,
    const double* __restrict__ vfit, const int32_t* __restrict__ vtrades, int64_t fit_ps,
    int64_t tr_ps, ShardView shard, int tell_only) {
    __shared__ double sv[2 * kStepBlock];
    __shared__ int si[2 * kStepBlock];
    __shared__ float lm[kMaxStepParams];
    __shared__ float la[kMaxStepParams];
    const int k = blockIdx.x;
    ga_step_dev<false>(pa.states + k, at_bytes(fit, k * fit_ps), at_bytes(trades, k * tr_ps),
                       at_bytes(vfit, k * fit_ps), at_bytes(vtrades, k * tr_ps), pa.P, shard,
                       pa.masters_mm + k * pa.n_mm, pa.masters_adv ? pa.masters_adv + k * pa.n_adv : nullptr,
                       pa.best_masters ? pa.best_masters + k * pa.n_mm : nullptr, pa.n_mm, pa.n_adv, pa.seeds[k],
                       pa.history ? pa.history + (int64_t)k * pa.hist_cap : nullptr, pa.hist_cap, nullptr,
                       nullptr, 0, 0, sv, si, lm, la, tell_only != 0);
}

}  // namespace sgmm

using namespace sgmm;

extern "C" int sgmm_ga_step_multi(const sgmm_populations* pops, const double* fitness,
                                  const int32_t* trades, const double* val_fitness,
                                  const int32_t* val_trades, int64_t fit_pop_stride,
                                  int64_t trades_pop_stride, int32_t shard_n, int64_t shard_stride,
                                  void* stream) {
    clear_error();
    SGMM_REQUIRE(pops && pops->n_pop > 0 && pops->P > 0, "bad populations");
    SGMM_REQUIRE(supported_hidden(pops->hidden), "hidden=%d unsupported", pops->hidden);
    SGMM_REQUIRE(pops->states && pops->masters_mm && pops->seeds && fitness && val_fitness, "null pointer");
    SGMM_REQUIRE(shard_n <= 0 || shard_stride >= 8LL * shard_n, "shard_stride < 8 * shard_n");
    const int64_t n_mm = (int64_t)pops->hidden * pops->hidden + 7 * pops->hidden + 2;
    SGMM_REQUIRE(n_mm <= kMaxStepParams, "genome too large for the GA step");  // the LDS master stage
    PopsArg pa{pops->states, pops->masters_mm, pops->masters_adv, pops->best_masters, pops->seeds,
               pops->history, pops->history_cap, pops->P, n_mm, pops->masters_adv ? 1250 : 0};
    ProfScope prof("ga_step", as_stream(stream));
    hipLaunchKernelGGL(k_ga_step_multi, dim3(pops->n_pop), dim3(kStepBlock), 0, as_stream(stream), pa,
                       fitness, trades, val_fitness, val_trades, fit_pop_stride, trades_pop_stride,
                       ShardView{shard_n, shard_stride}, 0);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_ga_tell_multi(const sgmm_populations* pops, const double* fitness, const int32_t* trades,
                                  int64_t fit_pop_stride, int64_t trades_pop_stride, int32_t shard_n,
                                  int64_t shard_stride, void* stream) {
    clear_error();
    SGMM_REQUIRE(pops && pops->n_pop > 0 && pops->P > 0, "bad populations");
    SGMM_REQUIRE(supported_hidden(pops->hidden), "hidden=%d unsupported", pops->hidden);
    SGMM_REQUIRE(pops->states && pops->masters_mm && pops->seeds && fitness, "null pointer");
    SGMM_REQUIRE(shard_n <= 0 || shard_stride >= 8LL * shard_n, "shard_stride < 8 * shard_n");
    const int64_t n_mm = (int64_t)pops->hidden * pops->hidden + 7 * pops->hidden + 2;
    SGMM_REQUIRE(n_mm <= kMaxStepParams, "genome too large for the GA step");
    PopsArg pa{pops->states, pops->masters_mm, pops->masters_adv, pops->best_masters, pops->seeds,
               pops->history, pops->history_cap, pops->P, n_mm, pops->masters_adv ? 1250 : 0};
    ProfScope prof("ga_tell", as_stream(stream));
    hipLaunchKernelGGL(k_ga_step_multi, dim3(pops->n_pop), dim3(kStepBlock), 0, as_stream(stream), pa,
                       fitness, trades, nullptr, nullptr, fit_pop_stride, trades_pop_stride,
                       ShardView{shard_n, shard_stride}, 1);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_ga_step(sgmm_ga_state* state, const double* fitness, const int32_t* trades,
                            const double* val_fitness, const int32_t* val_trades, int32_t P,
                            int32_t shard_n, int64_t shard_stride, float* master_mm, float* master_adv, float* best_master,
                            int64_t n_params_mm, int64_t n_params_adv, uint64_t seed,
                            sgmm_ga_history* history, int32_t history_cap, float* next_pop_mm,
                            float* next_pop_adv, int32_t i0, int32_t n, void* stream) {
    clear_error();
    SGMM_REQUIRE(state && fitness && val_fitness && master_mm, "null pointer");
    SGMM_REQUIRE(P > 0 && n_params_mm > 0 && n_params_mm <= kMaxStepParams, "bad P / n_params_mm");
    SGMM_REQUIRE(!master_adv || (n_params_adv > 0 && n_params_adv <= kMaxStepParams), "n_params_adv");
    SGMM_REQUIRE(!next_pop_mm || (n >= 0 && i0 >= 0), "bad next-ask shard");
    SGMM_REQUIRE(shard_n <= 0 || shard_stride >= 8LL * shard_n, "shard_stride < 8 * shard_n");
    ProfScope prof("ga_step", as_stream(stream));
    hipLaunchKernelGGL(k_ga_step, dim3(1), dim3(kStepBlock), 0, as_stream(stream), state,
                       fitness, trades, val_fitness, val_trades, P, ShardView{shard_n, shard_stride},
                       master_mm, master_adv,
                       best_master, n_params_mm, n_params_adv, seed, history, history_cap,
                       next_pop_mm, next_pop_adv, i0, n);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_ga_ask(const float* master, int64_t n_params, const sgmm_ga_state* state,
                           uint32_t stream_id, uint64_t seed, int32_t i0, int32_t n, float* out,
                           int64_t out_stride, void* stream) {
    clear_error();
    SGMM_REQUIRE(master && state && out, "null pointer");
    SGMM_REQUIRE(stream_id <= 1, "stream_id must be 0 (mm) or 1 (adversary)");
    SGMM_REQUIRE(n_params > 0 && n >= 0 && i0 >= 0 && out_stride >= n_params, "bad shape");
    if (n == 0) return SGMM_OK;
    const int64_t work = ((n_params + 3) / 4) * (int64_t)n;
    ProfScope prof("ga_ask", as_stream(stream));
    hipLaunchKernelGGL(k_ga_ask, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                       as_stream(stream), master, n_params, state, stream_id, seed, i0, n, out,
                       out_stride);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_ga_state_init(sgmm_ga_state* state, double sigma, int32_t patience,
                                  double decay, void* stream) {
    clear_error();
    SGMM_REQUIRE(state, "null state");
    hipLaunchKernelGGL(k_ga_state_init, dim3(1), dim3(1), 0, as_stream(stream), state, sigma,
                       patience, decay);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_ga_tell(sgmm_ga_state* state, const double* fitness, const int32_t* trades,
                            int32_t P, float* master_mm, const float* pop_mm,
                            int64_t pop_mm_stride, float* master_adv, const float* pop_adv,
                            int64_t pop_adv_stride, int64_t n_params_mm, int64_t n_params_adv,
                            uint64_t seed, sgmm_ga_history* history, int32_t history_cap,
                            void* stream) {
    clear_error();
    SGMM_REQUIRE(state && fitness && master_mm, "null pointer");
    SGMM_REQUIRE(P > 0 && n_params_mm > 0, "bad P / n_params_mm");
    SGMM_REQUIRE(!pop_mm || pop_mm_stride >= n_params_mm, "pop_mm_stride too small");
    SGMM_REQUIRE(!master_adv || n_params_adv > 0, "n_params_adv");
    SGMM_REQUIRE(!pop_adv || pop_adv_stride >= n_params_adv, "pop_adv_stride too small");
    ProfScope prof("ga_tell", as_stream(stream));
    hipLaunchKernelGGL(k_ga_tell, dim3(1), dim3(kTellBlock), 0, as_stream(stream), state,
                       fitness, trades, P, master_mm, pop_mm, pop_mm_stride, master_adv, pop_adv,
                       pop_adv_stride, n_params_mm, n_params_adv, seed, history, history_cap);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

extern "C" int sgmm_ga_val_update(sgmm_ga_state* state, const double* val_fitness,
                                  const int32_t* val_trades, int32_t use_best_index,
                                  const float* master_mm, float* best_master, int64_t n_params_mm,
                                  sgmm_ga_history* history, int32_t history_cap, void* stream) {
    clear_error();
    SGMM_REQUIRE(state && val_fitness && master_mm, "null pointer");
    SGMM_REQUIRE(n_params_mm > 0, "n_params_mm");
    ProfScope prof("ga_val_update", as_stream(stream));
    hipLaunchKernelGGL(k_ga_val_update, dim3(1), dim3(kTellBlock), 0, as_stream(stream), state,
                       val_fitness, val_trades, use_best_index, master_mm, best_master,
                       n_params_mm, history, history_cap);
    SGMM_LAUNCHED();
    return SGMM_OK;
}
