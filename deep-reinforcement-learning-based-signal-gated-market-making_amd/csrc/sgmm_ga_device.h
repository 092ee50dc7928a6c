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

__device__ void block_argmax2(const double* __restrict__ fit, ShardView sv_, int P, int& best,
                              int& abest, double* sv, int* si) {
    const int tid = threadIdx.x, nt = blockDim.x;
    double bv = 0.0, av = 0.0;
    int bi = -1, aj = -1;
    for (int i = tid; i < P; i += nt) {
        const double f = shard_at(fit, sv_, i);
        if (bi < 0 || better(f, i, bv, bi)) { bv = f; bi = i; }
        if (aj < 0 || better(-f, i, av, aj)) { av = -f; aj = i; }
    }
    sv[tid] = bv; si[tid] = bi;
    sv[nt + tid] = av; si[nt + tid] = aj;
    __syncthreads();
    for (int w = nt / 2; w > 0; w >>= 1) {
        if (tid < w) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int o = r * nt;
                const int io = si[o + tid + w];
                if (io >= 0 && (si[o + tid] < 0 || better(sv[o + tid + w], io, sv[o + tid], si[o + tid]))) {
                    sv[o + tid] = sv[o + tid + w];
                    si[o + tid] = io;
                }
            }
        }
        __syncthreads();
    }
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

// One generation boundary, executed by one whole workgroup (power-of-two
// size): tell both evolvers, validation bookkeeping, sigma decay, history
// row, and optionally the next generation's ask of [i0, i0+n).
// LDS scratch: sv[2*nt] doubles, si[2*nt] ints, lm[n_mm], la[n_adv] floats.
__device__ void ga_step_dev(sgmm_ga_state* __restrict__ st, const double* __restrict__ fit,
                            const int32_t* __restrict__ trades, const double* __restrict__ vfit,
                            const int32_t* __restrict__ vtrades, int32_t P, ShardView shard,
                            float* __restrict__ master, float* __restrict__ master_adv,
                            float* __restrict__ best_master, int64_t n_mm, int64_t n_adv,
                            uint64_t seed, sgmm_ga_history* __restrict__ history, int32_t hist_cap,
                            float* __restrict__ next_mm, float* __restrict__ next_adv, int32_t i0,
                            int32_t n, double* sv, int* si, float* lm, float* la) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const uint32_t gen = (uint32_t)st->gen;
    sgmm_ga_history* hist = (history && st->gen < hist_cap) ? history + st->gen : nullptr;
    int best, abest;
    block_argmax2(fit, shard, P, best, abest, sv, si);
    const float sig_mm = (float)st->sigma_mm, sig_adv = (float)st->sigma_adv;
    __syncthreads();  // sv/si are reused below
    // tell (model.py:73-76; drl_engine.py:119-125)
    regen_master(master, lm, n_mm, sig_mm, seed, 0u, gen, best);
    if (master_adv) regen_master(master_adv, la, n_adv, sig_adv, seed, 1u, gen, abest);
    if (tid == 0) {
        // validation of the best (drl_engine.py:129-171)
        const double v = shard_at(vfit, shard, best);
        const int improved = v > st->best_val;
        int decayed = 0;
        if (improved) {
            st->best_val = v;
            st->no_improve = 0;
        } else {
            st->no_improve += 1;
        }
        if (st->no_improve >= st->patience) {
            st->sigma_mm *= st->decay;
            st->sigma_adv *= st->decay;
            st->no_improve = 0;
            decayed = 1;
        }
        st->best_idx = best;
        st->adv_best_idx = abest;
        st->last_train_f = shard_at(fit, shard, best);
        st->improved = improved;
        st->decayed = decayed;
        st->last_val_f = v;
        st->gen += 1;
        si[0] = improved;
        sv[0] = st->sigma_mm;
        sv[1] = st->sigma_adv;
        if (hist) {
            hist->train_f = shard_at(fit, shard, best);
            hist->train_trades = trades ? shard_at(trades, shard, best) : 0;
            hist->best_idx = best;
            hist->val_f = v;
            hist->val_trades = vtrades ? shard_at(vtrades, shard, best) : 0;
            hist->sigma_after = st->sigma_mm;
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

}  // namespace sgmm
