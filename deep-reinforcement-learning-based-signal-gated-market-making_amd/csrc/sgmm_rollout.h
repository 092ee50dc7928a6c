// sgmm_rollout.h -- device layout and helpers shared by the rollout translation
// units (sgmm_rollout.hip: tables, path scans, host entry points;
// sgmm_frontier.hip: the frontier kernel).
#pragma once

#include "sgmm_device.h"
#include "sgmm_ga_device.h"
#include "sgmm_internal.h"

namespace sgmm {

constexpr int kChunk = 64;          // ticks per chunk in the path scan
constexpr int kSeg = 4096;          // ticks summed per LDS segment
constexpr int kScanBlock = 256;
constexpr int kMaxLen = 1 << 17;    // max ticks per episode of the no-adversary table path (its scan's LDS chunk tables)

struct EpArrays {
    const int32_t* genome;
    const int32_t* adv;
    const int64_t* tick_off;
    const int32_t* len;
    const int64_t* step_off;
    const int32_t* param;
    int64_t rs;  // no adversary: reward table stride, rew[state * rs + row] (SoA)
    const int32_t* order;  // frontier kernel: episode of order position p (NULL: p)
    // frontier kernel: the episodes at order positions [0, whole) are cut into
    // g0 groups of 64 chunks (one wave each, chunks of frontier_len(T, g0)
    // ticks), the rest into gtail groups (frontier_plan); ngrp = the larger,
    // the layout of the records (64 ngrp per episode) and plane padding; the
    // path scan reads an episode's group count from its first record
    int32_t ngrp;
    int32_t g0, gtail, whole;
    // path scans: the episode sums as the plain sequential chain (1) or by the
    // exact parallel binade method (0) -- the same bits either way (rollout_impl's rule)
    int32_t seq_sum = 0;
};

// Where an episode's genomes come from: materialized rows (pop != nullptr) or
// the current generation's ask() of the GA state, generated in the kernel
// (never written to memory): individual i0 + genome[e], values identical to
// what sgmm_ga_ask writes.  With several populations (pop_eps > 0) episode e
// belongs to population k = e / pop_eps, whose state, masters and Philox key
// sit at st + k, master_* + k * *_pstride and seeds[k].
struct GenomeSrc {
    const float* mm;
    int64_t mm_stride;
    const float* adv;
    int64_t adv_stride;
    const sgmm_ga_state* st;
    const float* master_mm;
    const float* master_adv;
    uint64_t seed;            // population 0's key when seeds == nullptr
    int32_t i0;
    int32_t pop_eps;          // episodes per population (0: one population)
    const uint64_t* seeds;    // [K] per-population keys, or nullptr
    int64_t mm_pstride, adv_pstride;
    // asked genomes: 1 = individual st->best_idx of the episode's population (the
    // tell's argmax, its master update deferred to the validation launch's tail)
    int32_t use_best = 0;
};

constexpr int kAdvParams = 74;  // AdversaryPolicy weights = first 74 floats of the genome
constexpr int kAdvGenome = 1250;  // adversary evolver masters are TradingPolicy() genomes (model.py:63)

// Stage the policy genome (n floats) of individual gi of episode e's
// population and, when ga != nullptr and ai >= 0, the adversary weights of
// individual ai into LDS.  Every thread of the block calls; the caller
// synchronizes.
__device__ inline void stage_genomes(const GenomeSrc& src, int e, int gi, int ai, int n, float* gs, float* ga) {
    const int tid = threadIdx.x, nt = blockDim.x;
    if (src.st) {
        const int k = src.pop_eps > 0 ? e / src.pop_eps : 0;
        const sgmm_ga_state* st = src.st + k;
        const uint64_t seed = src.seeds ? src.seeds[k] : src.seed;
        const float* master = src.master_mm + (int64_t)k * src.mm_pstride;
        const uint32_t gen = (uint32_t)st->gen;
        const float sig = (float)st->sigma_mm;
        const uint32_t ind = src.use_best ? (uint32_t)st->best_idx : (uint32_t)(src.i0 + gi);
        for (int k4 = tid; k4 < (n + 3) / 4; k4 += nt) {
            float v[4];
            ask_row4(master, n, sig, seed, 0u, gen, ind, k4, v);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (4 * k4 + q < n) gs[4 * k4 + q] = v[q];
        }
        if (ga && ai >= 0) {
            const float siga = (float)st->sigma_adv;
            const float* amaster = src.master_adv + (int64_t)k * src.adv_pstride;
            for (int k4 = tid; k4 < (kAdvParams + 3) / 4; k4 += nt) {
                float v[4];
                ask_row4(amaster, kAdvParams, siga, seed, 1u, gen, (uint32_t)(src.i0 + ai), k4, v);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (4 * k4 + q < kAdvParams) ga[4 * k4 + q] = v[q];
            }
        }
    } else {
        const float* __restrict__ row = src.mm + (int64_t)gi * src.mm_stride;
        for (int k = tid; k < n; k += nt) gs[k] = row[k];
        if (ga && ai >= 0) {
            const float* __restrict__ arow = src.adv + (int64_t)ai * src.adv_stride;
            for (int k = tid; k < kAdvParams; k += nt) ga[k] = arow[k];
        }
    }
}

// ------------------------------------------------------------------ transition maps
// A step's effect on the (<= 8) inventory states is a map state -> state,
// one byte per state in a u64 (byte x = image of state x).  Composition is
// two v_perm_b32 (byte x of the result = byte a[x] of b), so a wave of 64
// ticks builds the inclusive prefix of its chunk with six DPP steps and the
// path of any start state is one byte lookup.
constexpr uint64_t kIdentityMap = 0x0706050403020100ull;  // x -> x for x = 0..7

__device__ __forceinline__ uint32_t map_get(uint64_t m, uint32_t x) {
    return (uint32_t)(m >> (8u * x)) & 0xFFu;
}

// "first a, then b": (a ; b)[x] = b[a[x]]
__device__ __forceinline__ uint64_t map_then(uint64_t a, uint64_t b) {
    const uint32_t bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint32_t lo = __builtin_amdgcn_perm(bh, bl, (uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_perm(bh, bl, (uint32_t)(a >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// inclusive prefix composition over the wave (row shifts, then row
// broadcasts; a lane without a source composes the identity)
__device__ __forceinline__ uint64_t wave_map_scan(uint64_t m) {
#define SGMM_MSTEP(CTRL, RM) m = map_then(dpp64<CTRL, RM>(kIdentityMap, m), m);
    SGMM_MSTEP(0x111, 0xF) SGMM_MSTEP(0x112, 0xF) SGMM_MSTEP(0x114, 0xF)
    SGMM_MSTEP(0x118, 0xF) SGMM_MSTEP(0x142, 0xA) SGMM_MSTEP(0x143, 0xC)
#undef SGMM_MSTEP
    return m;
}

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, kWave);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, kWave);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t chunk_base(int64_t step_off, int e) {
    // chunk-map slot of episode e: regions of ceil(len/64) never overlap
    return (uint32_t)((step_off + (int64_t)kChunk * e) / kChunk);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int N>
struct IntC {
    static constexpr int value = N;
};
// number of lanes below this one whose bit is set in m
__device__ __forceinline__ int mbcnt64(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
constexpr int kFrontierLanes = 64;     // chunks per wave (one per lane)
#ifndef SGMM_FR_PRIO_EXTRA
#define SGMM_FR_PRIO_EXTRA 160
#endif
constexpr int kFrPrioExtra = SGMM_FR_PRIO_EXTRA;  // a walk's issue priority from 0.625 extra slots per tick on average
constexpr int kFrontierMaxWaves = 16;  // waves (64-chunk groups) per episode
// the chunk records (map, trade counts, merge info) of an episode cut into nw
// groups: 64 nw per episode, chunk c of episode e at e * 64 nw + c
__host__ __device__ __forceinline__ int64_t frontier_rec(int e, int nw, int c) {
    return (int64_t)e * kFrontierLanes * nw + c;
}
constexpr int64_t kFrontierMaxLen = (int64_t)kFrontierLanes * 65532;  // ticks: chunks (multiples of 4) below 2^16 ticks, 16-bit trade counts
typedef __attribute__((address_space(3))) const float lds_cf;
typedef __attribute__((address_space(3))) const f32x4 lds_cf4;
// ticks per chunk with nw waves (64 nw chunks) per episode
__host__ __device__ __forceinline__ int frontier_len(int T, int nw) {
    const int c = (T + kFrontierLanes * nw - 1) / (kFrontierLanes * nw);
    return c < 4 ? 4 : (c + 3) & ~3;  // a multiple of 4: a scan thread's 4 ticks stay in one chunk
}
// the episode's block of plane rows: nw groups of frontier_len(T, nw) x 64 rows
// <= T + 256 nw rows (T rounded up to 64 nw chunks of a multiple of 4),
// starting on a 128-byte line (16 rows), so blocks at step_off + pad e
// (rounded up to 16, pad = 256 nw + 16) never overlap and no two episodes
// share a line; the plane stride covers total_steps + pad n (rew_stride).
// Group g's rows start at base + g * CL * 64 (frontier_row within the group)
__host__ __device__ __forceinline__ int64_t frontier_pad(int nw) { return 256LL * nw + 16; }
__device__ __forceinline__ int64_t frontier_base(int64_t step_off, int e, int nw) {
    return (step_off + frontier_pad(nw) * e + 15) & ~int64_t(15);
}
// Within a group's block, the reward of chunk (lane) l at tick offset u: rows
// of the 64 chunks at one tick offset (u * 64 + l) -- a walk's store of one
// tick is one 512-byte row per plane, four whole 128-byte lines.  (Round 3's
// 4-tick groups, ((u >> 2) * 64 + l) * 4 + (u & 3), gave the scan one line per 4
// ticks but left lines part-written across ticks: 254 vs 155 MB written per
// config-3 launch, profiles/r03_pmc_traffic_c3.json vs r04_pmc_traffic_c3.json.)
__host__ __device__ __forceinline__ int64_t frontier_row(int u, int l) {
    return (int64_t)u * kFrontierLanes + l;
}
// wave b of a frontier launch -> the order position it walks, its chunk group
// and the episode's group count (EpArrays::g0 / gtail / whole)
__device__ __forceinline__ void frontier_wave(const EpArrays& ep, int b, int& pos, int& cg, int& nw) {
    const int nb0 = ep.whole * ep.g0;
    if (b < nb0) {
        pos = b / ep.g0;
        cg = b - pos * ep.g0;
        nw = ep.g0;
    } else {
        const int j = b - nb0, q = j / ep.gtail;
        pos = ep.whole + q;
        cg = j - q * ep.gtail;
        nw = ep.gtail;
    }
}
// chunk record merge info: the merge tick offset (bits 0-15), the episode's
// group count (bits 20-24), the lowest tracked start state (bits 29-31)
constexpr uint32_t kKinfoTick = 0xFFFFu;
__host__ __device__ __forceinline__ uint32_t kinfo_groups(uint32_t k) { return (k >> 20) & 31u; }

// ------------------------------------------------------------------ generation tail
// A fitness launch can end the generation itself: every workgroup publishes
// its episode's result (agent-scope release, arrival ticket); the last one to
// arrive acquires, runs the GA step (tell, validation bookkeeping, sigma
// decay, history) and resets the ticket.  Saves the separate GA launch.
struct StepArgs {
    sgmm_ga_state* st;  // nullptr: no GA step in this launch
    float* master_mm;
    float* master_adv;
    float* best_master;
    int64_t n_mm, n_adv;
    uint64_t seed;
    sgmm_ga_history* history;
    int32_t hist_cap;
    int32_t P;          // per population: fitness[0..P) training, fitness[P..2P) validation
    // several populations: episode e (workgroup e) belongs to population
    // k = e / pop_eps, whose state / masters / history / key sit at st + k,
    // master_* + k * n_*, history + k * hist_cap, seeds[k]; its records at
    // fitness + k * pop_eps.  pop_eps == 0: one population (the whole grid).
    int32_t pop_eps;
    const uint64_t* seeds;
    // 0: the whole boundary (records: P training then P validation results per
    // population); 1: tell only (the validation of the new master follows in its
    // own launches); 2: validation bookkeeping, one episode per population
    // (workgroup k = population k's post-tell master, validation_tail);
    // 3: the tell's argmax only (the last arriver is a one-wave workgroup whose
    // master regeneration took ~17 us, profiles/r05_timeline/sc_tr15d.txt) and
    // 4: its validation launch -- episode k rolls out individual best of
    // population k (GenomeSrc::use_best) and workgroup k regenerates the master
    // (all its threads) before the bookkeeping
    int32_t mode;
};

// The episode's fitness record, stored write-through (sc1) by ONE lane of
// the workgroup: the hand-off to the generation tail needs no release fence.
__device__ __forceinline__ void store_record(double* fitness, int32_t* trades, int e, double f,
                                             int32_t t) {
    typedef __attribute__((address_space(1))) double gdouble;
    typedef __attribute__((address_space(1))) int32_t gint;
    __hip_atomic_store((gdouble*)(fitness + e), f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gint*)(trades + e), t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ frontier kernel launch
struct FrontierArgs {
    sgmm_ticks tk;
    EpArrays ep;
    const sgmm_env_params* params;
    GenomeSrc src;
    int32_t inv_min, nsi;
    uint64_t* cmaps;
    uint32_t* ctr32;
    uint32_t* kinfo;
    double* rew;
    uint32_t* wslots;  // one wave per walk: [e * ngrp + cg] = the MLP slots it ran (walk-order feedback), or null
    // spill (k_frontier_spill): wave b of the launch writes wspill[b] = the tick
    // offset at which it stopped (a multiple of 4, > 0), or 0 when it walked to
    // the end; a walk stops once it has run spill_budget x 10 ns (0: never) and
    // its chunks have at most kSpillTicks ticks left
    uint32_t* wspill;
    uint32_t spill_budget;
    // fused path scan (k_policy_frontier<..., FS = true>): each walk sums its own
    // chunk group; of an episode walked in two groups, group 0 hands the chain on
    // through handoff[e] (or group 1 hands its rows over), hstate[e] the arrival
    // word (zero before the launch, reset by the wave that ends the chain); the
    // chain's last wave stores the record in fitness / trades, and the last record
    // of a population runs the generation tail (step: none or mode 3)
    double* fitness;
    int32_t* trades;
    struct FusedHandoff* handoff;
    uint32_t* hstate;
    int32_t n_eps;
    StepArgs step;
};
// group 0's chain state for group 1: the sum after its chunks, the state the path
// enters chunk 64 in (bits 0-7) and the trades so far (bits 8-31)
struct FusedHandoff {
    double S;
    uint32_t st_tr;
    uint32_t pad;
};
// fused path scan: a frontier walk's LDS holds a 512-tick window of the sum and
// its group's 64 start states / merge infos; at most two groups per episode
constexpr int kFusedWin = 512;
constexpr int kFusedMaxGroups = 2;
constexpr int kSpillTicks = 64;  // a spilled chunk's remaining ticks fit one wave (lane = tick)

// wave_map_scan within segments of SEG = 16, 32 or 64 lanes
template <int SEG>
__device__ __forceinline__ uint64_t wave_map_scan_seg(uint64_t m) {
#define SGMM_MSTEP(CTRL, RM) m = map_then(dpp64<CTRL, RM>(kIdentityMap, m), m);
    SGMM_MSTEP(0x111, 0xF) SGMM_MSTEP(0x112, 0xF) SGMM_MSTEP(0x114, 0xF) SGMM_MSTEP(0x118, 0xF)
    if constexpr (SEG >= 32) { SGMM_MSTEP(0x142, 0xA) }
    if constexpr (SEG >= 64) { SGMM_MSTEP(0x143, 0xC) }
#undef SGMM_MSTEP
    return m;
}

// launches the frontier kernel for hidden = 16 / 32 and nsi inventory states
// (sgmm_frontier.hip): grid = episodes x ep.ngrp waves
// ls: waves per 64-chunk group (1, 2 or 4; the grid is n_waves x ls)
// fa.fitness != nullptr: the fused path scan (ls = 1, ep.ngrp <= kFusedMaxGroups)
int launch_policy_frontier(int hidden, int nsi, unsigned n_waves, int ls, hipStream_t s, const FrontierArgs& fa);
// completes the chunks of the walks that spilled (fa.wspill) tick-parallel; a
// fixed grid (graph-capturable) that exits at once when no walk spilled
int launch_frontier_spill(int hidden, int nsi, unsigned n_waves, int ls, hipStream_t s, const FrontierArgs& fa);

}  // namespace sgmm
