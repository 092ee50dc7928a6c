// sgmm_ga_device.h -- the generation boundary as device code, shared by the
// standalone GA kernels (sgmm_ga.hip) and the fused rollout launches
// (sgmm_rollout.hip, whose last workgroup runs it).
//
// Reference: NeuroEvolution.tell (models/model.py:73-76) and the validation /
// sigma-decay block of DRLEngine.train (Env/drl_engine.py:119-171).
#pragma once

#include "sgmm_device.h"

namespace sgmm {

// ---------------------------------------------------------------- fused boundary
constexpr int kStepBlock = 1024;

// Loads of the fitness records.  HANDOFF: they were stored in this launch by
// other workgroups with write-through (sc1) stores, so every load of them is a
// global sc1 load (MI355X_MICROARCH.md, inter-workgroup visibility, row 1:
// one storing lane per workgroup, agent-scope arrival ticket, the last
// arriver loads) -- no acquire fence, no L2 invalidate.
template <bool HANDOFF, class T>
__device__ __forceinline__ T ld_rec(const T* p) {
    if constexpr (HANDOFF) {
        typedef __attribute__((address_space(1))) const T gT;
        return __hip_atomic_load((gT*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        return *p;
    }
}

template <bool HANDOFF, class T>
__device__ __forceinline__ T shard_ld(const T* __restrict__ base, ShardView v, int i) {
    if (v.n <= 0) return ld_rec<HANDOFF>(base + i);
    const char* q = reinterpret_cast<const char*>(base) + (int64_t)(i / v.n) * v.stride;
    return ld_rec<HANDOFF>(reinterpret_cast<const T*>(q) + i % v.n);
}

__device__ __forceinline__ void argmax_merge(double& bv, int& bi, double ov, int oi) {
    const bool take = oi >= 0 && (bi < 0 || better(ov, oi, bv, bi));
    bv = take ? ov : bv;
    bi = take ? oi : bi;
}

// np.argmax over one wave (first index on ties, NaN first), lanes with
// valid: a NaN ballot, a max butterfly, a ballot of the lanes equal to the
// max.  Returns the winning lane (-1: no valid lane) and its value.
__device__ __forceinline__ uint64_t argmax_key(double f) {
    // order-preserving unsigned key: -0 == +0, NaN above everything
    if (f != f) return ~0ull;
    const uint64_t b = (uint64_t)__double_as_longlong(f == 0.0 ? 0.0 : f);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}

// wave maximum of an unsigned 64-bit value (DPP row shifts and row
// broadcasts, integer data only), read from lane 63
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#define SGMM_XSTEP(CTRL, RM)                              \
    {                                                     \
        const uint64_t t_ = dpp64<CTRL, RM>(0ull, v);     \
        v = t_ > v ? t_ : v;                              \
    }
    SGMM_XSTEP(0x111, 0xF) SGMM_XSTEP(0x112, 0xF) SGMM_XSTEP(0x114, 0xF)
    SGMM_XSTEP(0x118, 0xF) SGMM_XSTEP(0x142, 0xA) SGMM_XSTEP(0x143, 0xC)
#undef SGMM_XSTEP
    return readlane64(v, kWave - 1);
}

__device__ __forceinline__ int wave_argmax_first(double f, bool valid, double& bv) {
    const uint64_t k = valid ? argmax_key(f) : 0ull;
    const uint64_t m = wave_max_u64(k);
    const uint64_t hit = __ballot(valid && k == m);
    const int l = hit ? __ffsll((unsigned long long)hit) - 1 : -1;
    bv = __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(f), l < 0 ? 0 : l));
    return l;
}

// np.argmax of fit and of -fit (first index on ties, NaN first) over the
// workgroup: strided scan, wave shuffles, one LDS round over the waves.
// LDS scratch: sv[2*nt] doubles, si[2*nt] ints.
template <bool HANDOFF>
__device__ void block_argmax2(const double* __restrict__ fit, ShardView sv_, int P, int& best,
                              int& abest, double* sv, int* si) {
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const int nw = (nt + kWave - 1) / kWave;
    double bv = 0.0, av = 0.0;
    int bi = -1, aj = -1;
    for (int i = tid; i < P; i += nt) {
        const double f = shard_ld<HANDOFF>(fit, sv_, i);
        argmax_merge(bv, bi, f, i);
        argmax_merge(av, aj, -f, i);
    }
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        const double ob = __shfl_down(bv, off, kWave), oa = __shfl_down(av, off, kWave);
        const int oib = __shfl_down(bi, off, kWave), oia = __shfl_down(aj, off, kWave);
        argmax_merge(bv, bi, ob, oib);
        argmax_merge(av, aj, oa, oia);
    }
    if (lane == 0) {
        sv[wv] = bv;
        si[wv] = bi;
        sv[nt + wv] = av;
        si[nt + wv] = aj;
    }
    __syncthreads();
    if (wv == 0) {
        bv = lane < nw ? sv[lane] : 0.0;
        bi = lane < nw ? si[lane] : -1;
        av = lane < nw ? sv[nt + lane] : 0.0;
        aj = lane < nw ? si[nt + lane] : -1;
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) {
            const double ob = __shfl_down(bv, off, kWave), oa = __shfl_down(av, off, kWave);
            const int oib = __shfl_down(bi, off, kWave), oia = __shfl_down(aj, off, kWave);
            argmax_merge(bv, bi, ob, oib);
            argmax_merge(av, aj, oa, oia);
        }
        if (lane == 0) {
            si[0] = bi;
            si[nt] = aj;
        }
    }
    __syncthreads();
    best = si[0];
    abest = si[nt];
}

// master <- ask(best) in place; staged copy to LDS for the next ask
__device__ void regen_master(float* __restrict__ master, float* lds_master, int64_t n, float sig,
                             uint64_t seed, uint32_t sid, uint32_t gen, int best) {
    for (int64_t k4 = threadIdx.x; k4 < (n + 3) / 4; k4 += blockDim.x) {
        float v[4];
        ask_row4(master, n, sig, seed, sid, gen, (uint32_t)best, k4, v);
        for (int q = 0; q < 4; ++q)
            if (4 * k4 + q < n) {
                master[4 * k4 + q] = v[q];
                lds_master[4 * k4 + q] = v[q];
            }
    }
}

__device__ void ask_rows(const float* lds_master, int64_t n, float sig, uint64_t seed,
                         uint32_t sid, uint32_t gen, int32_t i0, int32_t cnt,
                         float* __restrict__ out) {
    const int64_t nk4 = (n + 3) / 4;
    for (int64_t g = threadIdx.x; g < nk4 * cnt; g += blockDim.x) {
        const int32_t i = (int32_t)(g / nk4);
        const int64_t k4 = g - (int64_t)i * nk4;
        float v[4];
        ask_row4(lds_master, n, sig, seed, sid, gen, (uint32_t)(i0 + i), k4, v);
        for (int q = 0; q < 4; ++q)
            if (4 * k4 + q < n) out[(int64_t)i * n + 4 * k4 + q] = v[q];
    }
}

// The tell's bookkeeping when the validation runs after it (reference order,
// drl_engine.py:119-128): best / adversary indices, the best training record,
// the history row's training fields.  One thread.
template <bool HANDOFF>
__device__ __forceinline__ void tell_record(sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
                                            const int32_t* __restrict__ trades, ShardView shard, int best,
                                            int abest, sgmm_ga_history* __restrict__ hist) {
    const double tf = shard_ld<HANDOFF>(fit, shard, best);
    const int32_t ttr = trades ? shard_ld<HANDOFF>(trades, shard, best) : 0;
    st->best_idx = best;
    st->adv_best_idx = abest;
    st->last_train_f = tf;
    if (hist) {
        hist->train_f = tf;
        hist->train_trades = ttr;
        hist->best_idx = best;
    }
}

// Validation bookkeeping of one population (drl_engine.py:129-160): v / vtr
// are the validation record of the post-tell master.  Checkpoint copy
// master -> best_master on improvement (strictly greater; NaN never improves),
// sigma decay after `patience` generations without improvement, the history
// row's validation fields, gen + 1.  Every thread of the workgroup calls
// (v identical in all); `flag` is one int of LDS scratch.
__device__ __forceinline__ void val_update_dev(sgmm_ga_state* __restrict__ st, double v, int32_t vtr,
                                               const float* __restrict__ master, float* __restrict__ best_master,
                                               int64_t n, sgmm_ga_history* __restrict__ history,
                                               int32_t hist_cap, int* flag) {
    if (threadIdx.x == 0) {
        const int32_t gen = st->gen;
        sgmm_ga_history* hist = (history && gen < hist_cap) ? history + gen : nullptr;
        const int improved = v > st->best_val;
        int decayed = 0;
        int32_t no_improve = st->no_improve;
        if (improved) {
            st->best_val = v;
            no_improve = 0;
        } else {
            no_improve += 1;
        }
        double smm = st->sigma_mm, sadv = st->sigma_adv;
        if (no_improve >= st->patience) {  // drl_engine.py:155-160
            smm *= st->decay;
            sadv *= st->decay;
            no_improve = 0;
            decayed = 1;
        }
        st->sigma_mm = smm;
        st->sigma_adv = sadv;
        st->no_improve = no_improve;
        st->improved = improved;
        st->decayed = decayed;
        st->last_val_f = v;
        st->gen = gen + 1;
        if (hist) {
            hist->val_f = v;
            hist->val_trades = vtr;
            hist->sigma_after = smm;
            hist->flags = improved | (decayed << 1);
        }
        *flag = improved;
    }
    __syncthreads();
    if (*flag && best_master)
        for (int64_t k = threadIdx.x; k < n; k += blockDim.x) best_master[k] = master[k];
}

// One generation boundary, executed by one whole workgroup (power-of-two
// size): tell both evolvers, validation bookkeeping, sigma decay, history
// row, and optionally the next generation's ask of [i0, i0+n).
// LDS scratch: sv[2*nt] doubles, si[2*nt] ints, lm[n_mm], la[n_adv] floats.
// HANDOFF: the fitness records come from other workgroups of this launch
// (sc1 loads, see ld_rec).
template <bool HANDOFF>
__device__ void ga_step_dev(sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
                            const int32_t* __restrict__ trades, const double* __restrict__ vfit,
                            const int32_t* __restrict__ vtrades, int32_t P, ShardView shard,
                            float* __restrict__ master, float* __restrict__ master_adv,
                            float* __restrict__ best_master, int64_t n_mm, int64_t n_adv,
                            uint64_t seed, sgmm_ga_history* __restrict__ history, int32_t hist_cap,
                            float* __restrict__ next_mm, float* __restrict__ next_adv, int32_t i0,
                            int32_t n, double* sv, int* si, float* lm, float* la, bool tell_only = false) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const uint32_t gen = (uint32_t)st->gen;
    sgmm_ga_history* hist = (history && st->gen < hist_cap) ? history + st->gen : nullptr;
    int best, abest;
    block_argmax2<HANDOFF>(fit, shard, P, best, abest, sv, si);
    const float sig_mm = (float)st->sigma_mm, sig_adv = (float)st->sigma_adv;
    __syncthreads();  // sv/si are reused below
    // tell (model.py:73-76; drl_engine.py:119-125)
    regen_master(master, lm, n_mm, sig_mm, seed, 0u, gen, best);
    if (master_adv) regen_master(master_adv, la, n_adv, sig_adv, seed, 1u, gen, abest);
    if (tell_only) {  // the validation of the new master follows in its own launches
        if (tid == 0) tell_record<HANDOFF>(st, fit, trades, shard, best, abest, hist);
        return;
    }
    if (tid == 0) {
        // validation of the best (drl_engine.py:129-171); every load issued
        // before the first dependent use
        const double v = shard_ld<HANDOFF>(vfit, shard, best);
        const double tf = shard_ld<HANDOFF>(fit, shard, best);
        const int32_t ttr = trades ? shard_ld<HANDOFF>(trades, shard, best) : 0;
        const int32_t vtr = vtrades ? shard_ld<HANDOFF>(vtrades, shard, best) : 0;
        const double best_val = st->best_val, decay = st->decay;
        double smm = st->sigma_mm, sadv = st->sigma_adv;
        int32_t no_improve = st->no_improve;
        const int32_t patience = st->patience;
        const int improved = v > best_val;
        int decayed = 0;
        if (improved) {
            st->best_val = v;
            no_improve = 0;
        } else {
            no_improve += 1;
        }
        if (no_improve >= patience) {
            smm *= decay;
            sadv *= decay;
            no_improve = 0;
            decayed = 1;
        }
        st->sigma_mm = smm;
        st->sigma_adv = sadv;
        st->no_improve = no_improve;
        st->best_idx = best;
        st->adv_best_idx = abest;
        st->last_train_f = tf;
        st->improved = improved;
        st->decayed = decayed;
        st->last_val_f = v;
        st->gen = (int32_t)gen + 1;
        si[0] = improved;
        sv[0] = smm;
        sv[1] = sadv;
        if (hist) {
            hist->train_f = tf;
            hist->train_trades = ttr;
            hist->best_idx = best;
            hist->val_f = v;
            hist->val_trades = vtr;
            hist->sigma_after = smm;
            hist->flags = improved | (decayed << 1);
        }
    }
    __syncthreads();
    const int improved = si[0];
    const float next_sig_mm = (float)sv[0], next_sig_adv = (float)sv[1];
    if (improved && best_master)
        for (int64_t k = tid; k < n_mm; k += nt) best_master[k] = lm[k];
    // ask of the next generation (model.py:65-71) from the new master / sigma
    if (next_mm) ask_rows(lm, n_mm, next_sig_mm, seed, 0u, gen + 1, i0, n, next_mm);
    if (next_adv && master_adv) ask_rows(la, n_adv, next_sig_adv, seed, 1u, gen + 1, i0, n, next_adv);
}

// The fused generation tail's GA step (sgmm_generation: one workgroup, the
// records contiguous, P <= blockDim.x).  The same results as ga_step_dev, laid
// out for latency: every record (sc1) and the masters are loaded up front, the
// argmax carries the best individual's validation record through its
// shuffles, and the masters are regenerated from registers.
constexpr int kTailSlots = 4;  // float4 master chunks per thread (n <= 16 * blockDim.x)

#ifdef SGMM_STAMPS
static __device__ unsigned long long g_tail[8];  // diagnostic build: tail phase times (thread 0)
#endif
#if defined(SGMM_STAMPS) && !defined(SGMM_NO_TAIL_STAMPS)
// the clock when `dep` is available (its register dependency only: no memory
// wait), kept in registers and stored once at the end (SGMM_TAIL_FLUSH)
#define SGMM_TAIL_DECL unsigned long long tt_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SGMM_TAIL_STAMP(k, dep) \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt_[k]) : "v"(dep) : "memory")
#define SGMM_TAIL_FLUSH                                         \
    do {                                                        \
        if (threadIdx.x == 0)                                   \
            for (int k_ = 0; k_ < 8; ++k_) g_tail[k_] = tt_[k_]; \
    } while (0)
#else
#define SGMM_TAIL_DECL
#define SGMM_TAIL_STAMP(k, dep) \
    do {                        \
    } while (0)
#define SGMM_TAIL_FLUSH \
    do {                \
    } while (0)
#endif

__device__ __forceinline__ void argmax_merge_p(double& bv, int& bi, double& pv, int& pt, int& pvt,
                                               double ov, int oi, double opv, int opt, int opvt) {
    const bool take = oi >= 0 && (bi < 0 || better(ov, oi, bv, bi));
    bv = take ? ov : bv;
    bi = take ? oi : bi;
    pv = take ? opv : pv;
    pt = take ? opt : pt;
    pvt = take ? opvt : pvt;
}

__device__ __forceinline__ void load_master4(const float* __restrict__ m, int64_t n,
                                             float (&r)[kTailSlots][4]) {
#pragma unroll
    for (int j = 0; j < kTailSlots; ++j) {
        const int64_t k4 = threadIdx.x + (int64_t)j * blockDim.x;
#pragma unroll
        for (int q = 0; q < 4; ++q) r[j][q] = 4 * k4 + q < n ? m[4 * k4 + q] : 0.0f;
    }
}

// master <- ask(best) from the registers m; also into best_copy when given
// (the validation improved: the checkpoint copy, drl_engine.py:133-137)
__device__ __forceinline__ void regen_master_regs(float* __restrict__ master, float* __restrict__ best_copy,
                                                  int64_t n, const float (&m)[kTailSlots][4],
                                                  float sig, uint64_t seed, uint32_t sid,
                                                  uint32_t gen, int best) {
#pragma unroll
    for (int j = 0; j < kTailSlots; ++j) {
        const int64_t k4 = threadIdx.x + (int64_t)j * blockDim.x;
        if (4 * k4 >= n) break;
        float z[4];
        normal4(seed, sid, gen, (uint32_t)best, (uint32_t)k4, z);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * k4 + q < n) {
                const float v = m[j][q] + z[q] * sig;  // ask_row4's arithmetic
                master[4 * k4 + q] = v;
                if (best_copy) best_copy[4 * k4 + q] = v;
            }
    }
}

template <bool HANDOFF>
__device__ void ga_step_fused(sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
                              const int32_t* __restrict__ trades, const double* __restrict__ vfit,
                              const int32_t* __restrict__ vtrades, int32_t P,
                              float* __restrict__ master, float* __restrict__ master_adv,
                              float* __restrict__ best_master, int64_t n_mm, int64_t n_adv,
                              uint64_t seed, sgmm_ga_history* __restrict__ history, int32_t hist_cap,
                              double* sv, int* si, float* lm, float* la, bool tell_only = false) {
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & (kWave - 1), wv = tid / kWave;
    const int nw = (nt + kWave - 1) / kWave;
    SGMM_TAIL_DECL
    // ---- every load first
    double f = 0.0, vf = 0.0;
    int tr = 0, vtr = 0;
    const bool mine = tid < P;
    if (mine) {
        f = ld_rec<HANDOFF>(fit + tid);
        if (!tell_only) vf = ld_rec<HANDOFF>(vfit + tid);
        if (trades) tr = ld_rec<HANDOFF>(trades + tid);
        if (vtrades && !tell_only) vtr = ld_rec<HANDOFF>(vtrades + tid);
    }
    float mm[kTailSlots][4], ma[kTailSlots][4];
    load_master4(master, n_mm, mm);
    if (master_adv) load_master4(master_adv, n_adv, ma);
    const int32_t gen_i = st->gen;
    const uint32_t gen = (uint32_t)gen_i;
    const double st_smm = st->sigma_mm, st_sadv = st->sigma_adv, best_val = st->best_val,
                 decay = st->decay;
    const int32_t no_improve0 = st->no_improve, patience = st->patience;
    const float sig_mm = (float)st_smm, sig_adv = (float)st_sadv;
    SGMM_TAIL_STAMP(0, f + vf + mm[0][0] + sig_mm);
    // ---- argmax of fit (payload: the validation record) and of -fit: the
    // waves holding records reduce with shuffles, every thread merges their
    // results from LDS
    const int nwa = (P + kWave - 1) / kWave;
    double bv = f, pv = vf, av = -f;
    int bi = mine ? tid : -1, pt = tr, pvt = vtr, aj = bi;
    if (wv < nwa) {
        const int bl = wave_argmax_first(f, mine, bv);
        const int al = wave_argmax_first(-f, mine, av);
        const int src = bl < 0 ? 0 : bl;  // wave-uniform
        pv = __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(vf), src));
        pt = __builtin_amdgcn_readlane(tr, src);
        pvt = __builtin_amdgcn_readlane(vtr, src);
        bi = bl < 0 ? -1 : wv * kWave + bl;
        aj = al < 0 ? -1 : wv * kWave + al;
        // per-wave results: sv[0..nw) best, sv[nw..2nw) its validation fitness, sv[2nw..3nw)
        // adversary; si[0..nw) best idx, si[nw..2nw) trades, si[2nw..3nw) val trades,
        // si[3nw..4nw) adversary idx
        if (lane == 0) {
            sv[wv] = bv;
            sv[nw + wv] = pv;
            sv[2 * nw + wv] = av;
            si[wv] = bi;
            si[nw + wv] = pt;
            si[2 * nw + wv] = pvt;
            si[3 * nw + wv] = aj;
        }
    }
    SGMM_TAIL_STAMP(6, bv);
    __syncthreads();
    SGMM_TAIL_STAMP(7, bv);
    bv = sv[0];
    pv = sv[nw];
    av = sv[2 * nw];
    bi = si[0];
    pt = si[nw];
    pvt = si[2 * nw];
    aj = si[3 * nw];
    for (int w = 1; w < nwa; ++w) {
        argmax_merge_p(bv, bi, pv, pt, pvt, sv[w], si[w], sv[nw + w], si[nw + w], si[2 * nw + w]);
        argmax_merge(av, aj, sv[2 * nw + w], si[3 * nw + w]);
    }
    const int best = bi, abest = aj;
    // every thread knows whether the validation improved (drl_engine.py:130-131)
    const int improved = !tell_only && pv > best_val;
    SGMM_TAIL_STAMP(1, best + abest);
    // ---- tell (model.py:73-76; drl_engine.py:119-125), the checkpoint copy
    // of the new master written in the same pass
    regen_master_regs(master, improved ? best_master : nullptr, n_mm, mm, sig_mm, seed, 0u, gen, best);
    if (master_adv) regen_master_regs(master_adv, nullptr, n_adv, ma, sig_adv, seed, 1u, gen, abest);
    SGMM_TAIL_STAMP(2, mm[0][0]);
    if (tell_only) {  // the validation of the new master follows in its own launches
        if (tid == 0) {
            st->best_idx = best;
            st->adv_best_idx = abest;
            st->last_train_f = bv;
            if (history && gen_i < hist_cap) {
                sgmm_ga_history* hist = history + gen_i;
                hist->train_f = bv;
                hist->train_trades = pt;
                hist->best_idx = best;
            }
        }
        SGMM_TAIL_FLUSH;
        return;
    }
    if (tid == 0) {  // validation of the best (drl_engine.py:129-171)
        const double v = pv, tf = bv;
        double smm = st_smm, sadv = st_sadv;
        int32_t no_improve = no_improve0;
        int decayed = 0;
        if (improved) {
            st->best_val = v;
            no_improve = 0;
        } else {
            no_improve += 1;
        }
        if (no_improve >= patience) {
            smm *= decay;
            sadv *= decay;
            no_improve = 0;
            decayed = 1;
        }
        st->sigma_mm = smm;
        st->sigma_adv = sadv;
        st->no_improve = no_improve;
        st->best_idx = best;
        st->adv_best_idx = abest;
        st->last_train_f = tf;
        st->improved = improved;
        st->decayed = decayed;
        st->last_val_f = v;
        st->gen = gen_i + 1;
        if (history && gen_i < hist_cap) {
            sgmm_ga_history* hist = history + gen_i;
            hist->train_f = tf;
            hist->train_trades = pt;
            hist->best_idx = best;
            hist->val_f = v;
            hist->val_trades = pvt;
            hist->sigma_after = smm;
            hist->flags = improved | (decayed << 1);
        }
    }
    SGMM_TAIL_STAMP(4, improved);
    SGMM_TAIL_FLUSH;
    (void)lm;
    (void)la;
}

// The tell (tell_only) in a ONE-WAVE workgroup (the path scans above 1024
// episodes): lane l holds records l, l + 64, ... (loaded 16 at a time, sc1),
// the wave's argmax is a DPP maximum of the order-preserving key and a DPP
// minimum of the index among equal keys (np.argmax: first index, NaN first),
// the best's training record comes from its lane's registers, and the masters
// are regenerated from up-front loads.  Same results as ga_step_dev.
constexpr int kWaveRec = 16;     // records per lane loaded together
constexpr int kWaveChunks = 8;   // float4 master chunks per lane: n <= 2048

__device__ __forceinline__ int wave_min_i32(int v) {
#define SGMM_MSTEP(CTRL, RM)                                                  \
    {                                                                         \
        const int t_ = (int)dpp32<CTRL, RM>((uint32_t)INT32_MAX, (uint32_t)v); \
        v = t_ < v ? t_ : v;                                                  \
    }
    SGMM_MSTEP(0x111, 0xF) SGMM_MSTEP(0x112, 0xF) SGMM_MSTEP(0x114, 0xF)
    SGMM_MSTEP(0x118, 0xF) SGMM_MSTEP(0x142, 0xA) SGMM_MSTEP(0x143, 0xC)
#undef SGMM_MSTEP
    return __builtin_amdgcn_readlane(v, kWave - 1);
}

// first index of the largest key over the wave (lane candidates (key, idx),
// idx < 0: none); -1 when no lane has a candidate
__device__ __forceinline__ int wave_best_index(uint64_t key, int idx) {
    const uint64_t m = wave_max_u64(idx >= 0 ? key : 0ull);  // valid keys are > 0
    const int c = wave_min_i32(idx >= 0 && key == m ? idx : INT32_MAX);
    return c == INT32_MAX ? -1 : c;
}

__device__ __forceinline__ void regen_master_wave(float* __restrict__ master, int64_t n, float sig, uint64_t seed,
                                                  uint32_t sid, uint32_t gen, int best) {
    const int lane = threadIdx.x & (kWave - 1);
    float m[kWaveChunks][4];
#pragma unroll
    for (int j = 0; j < kWaveChunks; ++j) {
        const int64_t k4 = lane + (int64_t)j * kWave;
#pragma unroll
        for (int q = 0; q < 4; ++q) m[j][q] = 4 * k4 + q < n ? master[4 * k4 + q] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < kWaveChunks; ++j) {
        const int64_t k4 = lane + (int64_t)j * kWave;
        if (4 * k4 >= n) break;
        float z[4];
        normal4(seed, sid, gen, (uint32_t)best, (uint32_t)k4, z);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * k4 + q < n) master[4 * k4 + q] = m[j][q] + z[q] * sig;  // ask_row4's arithmetic
    }
}

// master <- ask(best) by every thread of the workgroup (4 parameters a thread
// at a time, each read before it is overwritten): the deferred half of the tell
__device__ __forceinline__ void regen_master_block(float* __restrict__ master, int64_t n, float sig, uint64_t seed,
                                                   uint32_t sid, uint32_t gen, int best) {
    for (int64_t k4 = threadIdx.x; 4 * k4 < n; k4 += blockDim.x) {
        float m[4], z[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) m[q] = 4 * k4 + q < n ? master[4 * k4 + q] : 0.0f;
        normal4(seed, sid, gen, (uint32_t)best, (uint32_t)k4, z);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (4 * k4 + q < n) master[4 * k4 + q] = m[q] + z[q] * sig;  // ask_row4's arithmetic
    }
}

// REGEN = false: the argmax and the bookkeeping only; master <- ask(best)
// happens in the validation launch's tail (regen_master_block)
template <bool HANDOFF, bool REGEN = true>
__device__ void tell_wave(sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
                          const int32_t* __restrict__ trades, int32_t P, float* __restrict__ master,
                          float* __restrict__ master_adv, int64_t n_mm, int64_t n_adv, uint64_t seed,
                          sgmm_ga_history* __restrict__ history, int32_t hist_cap) {
    const int lane = threadIdx.x & (kWave - 1);
    const int32_t gen_i = st->gen;
    const uint32_t gen = (uint32_t)gen_i;
    const float sig_mm = (float)st->sigma_mm, sig_adv = (float)st->sigma_adv;
    // this lane's best (ascending indices: the first wins ties) for fit and
    // -fit, over blocks of kWaveRec records per lane, each block's loads issued
    // together
    double bv = 0.0, av = 0.0;
    int bi = -1, aj = -1;
    int32_t btr = 0;
    for (int r0 = 0; r0 * kWave < P; r0 += kWaveRec) {
        double f[kWaveRec];
        int32_t tr[kWaveRec];
#pragma unroll
        for (int r = 0; r < kWaveRec; ++r) {
            const int i = lane + (r0 + r) * kWave;
            f[r] = i < P ? ld_rec<HANDOFF>(fit + i) : 0.0;
            tr[r] = (i < P && trades) ? ld_rec<HANDOFF>(trades + i) : 0;
        }
#pragma unroll
        for (int r = 0; r < kWaveRec; ++r) {
            const int i = lane + (r0 + r) * kWave;
            if (i < P) {
                const bool tb = bi < 0 || better(f[r], i, bv, bi);
                bv = tb ? f[r] : bv;
                btr = tb ? tr[r] : btr;
                bi = tb ? i : bi;
                argmax_merge(av, aj, -f[r], i);
            }
        }
    }
    const int best = wave_best_index(argmax_key(bv), bi);
    const int abest = wave_best_index(argmax_key(av), aj);
    const int src = (best < 0 ? 0 : best) & (kWave - 1);
    const double tf = __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(bv), src));
    const int32_t ttr = __builtin_amdgcn_readlane(btr, src);
    // tell (model.py:73-76; drl_engine.py:119-125)
    if constexpr (REGEN) {
        regen_master_wave(master, n_mm, sig_mm, seed, 0u, gen, best);
        if (master_adv) regen_master_wave(master_adv, n_adv, sig_adv, seed, 1u, gen, abest);
    }
    if (lane == 0) {
        st->best_idx = best;
        st->adv_best_idx = abest;
        st->last_train_f = tf;
        if (history && gen_i < hist_cap) {
            sgmm_ga_history* hist = history + gen_i;
            hist->train_f = tf;
            hist->train_trades = ttr;
            hist->best_idx = best;
        }
    }
}

}  // namespace sgmm
