// sgmm_rollout.hip -- the population-rollout hot path on gfx950.
//
// Reference semantics: evaluate_individual (Env/drl_engine.py:9-67) mapped
// over a GA population (drl_engine.py:104-115), FTPEnv.step
// (Env/market_env.py:22-67), TradingPolicy / AdversaryPolicy
// (models/model.py:5-57).
//
// Fitness path (sgmm_rollout_fitness) -- a policy kernel, then a path scan:
//
//  1. policy kernel.  The inventory feedback makes an episode a serial chain,
//     but the policy only sees (signal_t, inventory) and the inventory takes
//     at most 8 values (caps +-2 -> 5), so the per-(tick, state) work can be
//     laid out in parallel:
//     - k_policy_frontier (many episodes, H = 16 / 32): one wave per episode,
//       lane = chunk, only the states the chunk's paths occupy are evaluated;
//     - k_policy_table_v3 (few episodes, and the adversary path): every
//       (tick, inventory[, adversary flags]) state, one wave per 64 ticks, the
//       H x H layer on v_mfma_f32_16x16x4_f32 (its k-ordered fused chain IS
//       the canonical dot-product order); k_policy_table_mfma (round 1's
//       schedule, H = 64) and k_policy_table (VALU, H = 8) likewise.
//     Output: per chunk its transition byte-map and the trade count along the
//     path from each start state, per tick the path planes (the reward along
//     the chunk's path from each start state).  With the adversary: 2 fill
//     bits per (inventory, previous fills) state (u64) and one float64 reward
//     plane per state.
//
//  2. path scan (one workgroup, or one wave, per episode): chunk start states
//     from the chunk maps, each tick's reward = one row of its chunk's path
//     plane, summed in the reference's sequential float64 order (bit-exact,
//     exact_sum_window), trades from the chunk counts.  The adversary variant
//     derives each chunk's transducer from the fill codes, chains them by
//     pointer jumping segment by segment and walks the true path.
//
// Trace path (sgmm_rollout_trace): k_rollout_direct, one wave per episode,
// lane = hidden neuron, the literal step loop (independent second
// implementation; the tests require both paths to agree bit for bit).
#include <algorithm>
#include <climits>
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>

#include "sgmm_rollout.h"

namespace sgmm {




// ------------------------------------------------------------------ adversary state machine
// State (inventory, previous sell fill, previous buy fill) = 4 * inv_index + 2 fs + fb
// (drl_engine.py:42-45, 62-63); a tick's 2-bit code is fill_buy | fill_sell << 1.
__device__ __forceinline__ int next_state_arl(int s, int code) {
    const int fb = code & 1, fs = code >> 1;
    return (((s >> 2) + fb - fs) << 2) | (fs << 1) | fb;
}
// one tick of the walk from state s over the tick's 2-bit fill codes f (state x
// at bits 2x): next_state_arl with the inventory step as a byte lookup
// (code 0, 1, 2, 3 -> 0, +4, -4, 0 on s & ~3) and the trade count
__device__ __forceinline__ int arl_step(int s, uint64_t f, int& cnt) {
    const int c = (int)(f >> (2 * s)) & 3;
    cnt += c != 0;
    const int d = __builtin_amdgcn_sbfe(0x00FC0400, 8 * c, 8);
    return ((s + d) & ~3) | c;
}

// ------------------------------------------------------------------ table
// Block = 64 consecutive ticks of one episode x nsi inventory states: wave w
// evaluates the policy and the FPT step for every tick of the block from
// inventory inv_min + w (one lane per (tick, state)).  The genome is
// wave-uniform, so weights arrive by scalar loads straight into the FMAs'
// SGPR operands, each used once (no loop-invariant hoisting, no SGPR spills,
// ~H+16 VGPRs -> full occupancy).  The 64-tick slice of the tick stream is
// staged once in LDS (coalesced) and read by all waves.  Wave 0 then turns the
// per-state fills into the chunk's transition maps.  Outputs:
//   !ARL: per chunk, cmaps[chunk] = the chunk's full transition map and
//         ctr[chunk] = the trade count along the chunk's path from each start
//         state (8 bits per state); per tick, the path planes
//         rew[s * rs + row] = the reward of the tick along the chunk's path
//         that starts in state s (float64);
//    ARL: fills[row] = 2 fill bits per (inventory, sell flag, buy flag) state
//         and rew[state * rs + row] = the step reward from that state.
template <int H, int NSM, bool ARL>
__global__ __launch_bounds__(kChunk * 8) void k_policy_table(
    sgmm_ticks tk, EpArrays ep, const sgmm_env_params* __restrict__ params,
    GenomeSrc src, int32_t inv_min, int32_t nsi, uint64_t* __restrict__ ctr,
    uint64_t* __restrict__ cmaps, uint64_t* __restrict__ fills, double* __restrict__ rew) {
    const int e = blockIdx.y;
    const int32_t T = ep.len[e];
    const int32_t t0 = blockIdx.x * kChunk;
    if (t0 >= T) return;  // block-uniform
    const int w = threadIdx.x >> 6, lane = threadIdx.x & (kWave - 1);
    const int ns = ARL ? 4 * nsi : nsi;
    const sgmm_env_params p = params[ep.param[e]];
    __shared__ float gsm[GenomeLayout<H>::N];
    __shared__ float gsa[kAdvParams];
    const int ai = (ARL && ep.adv) ? ep.adv[e] : -1;
    stage_genomes(src, e, ep.genome[e], ai, GenomeLayout<H>::N, gsm, ARL ? gsa : nullptr);
    const float* g = gsm;

    __shared__ float sx[2][kChunk];
    __shared__ double spx[5][kChunk];
    __shared__ uint8_t code[32][kChunk];
    __shared__ double rws[ARL ? 1 : NSM][kChunk];  // !ARL: per-state rewards for the path planes
    __shared__ int32_t lut[2][32];
    // stage the tick slice: column c by wave c % nsi
    const int64_t tbase = ep.tick_off[e] + t0;
    const int nvalid = min(kChunk, T - t0);
    for (int c = w; c < 7; c += nsi) {
        if (lane < nvalid) {
            const int64_t ti = tbase + lane;
            switch (c) {
                case 0: sx[0][lane] = tk.s1n[ti]; break;
                case 1: sx[1][lane] = tk.s2n[ti]; break;
                case 2: spx[0][lane] = tk.mid_next[ti]; break;
                case 3: spx[1][lane] = tk.best_ask[ti]; break;
                case 4: spx[2][lane] = tk.best_bid[ti]; break;
                case 5: spx[3][lane] = tk.buy_max[ti]; break;
                default: spx[4][lane] = tk.sell_min[ti]; break;
            }
        }
    }
    __syncthreads();  // staged genomes
    if (ARL) {
        if ((int)threadIdx.x < ns) {
            const int s = threadIdx.x;
            int32_t da = 0, db = 0;
            if (ai >= 0) adv_delta(gsa, p, inv_min + (s >> 2), (s >> 1) & 1, s & 1, da, db);
            lut[0][s] = da;
            lut[1][s] = db;
        }
    }
    __syncthreads();
    const bool valid = lane < nvalid;
    if (valid) {
        const int32_t inv = inv_min + w;
        float o0, o1;
        mlp_forward<H>(g, sx[0][lane], sx[1][lane], (float)((double)inv / 2.0), o0, o1);
        const int32_t oa = act_to_int(rintf(o0 * p.act_scale));  // drl_engine.py:38-39
        const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
        const double mid = spx[0][lane], ask = spx[1][lane], bid = spx[2][lane];
        const double bmax = spx[3][lane], smin = spx[4][lane];
        const int64_t row = ep.step_off[e] + t0 + lane;
        if (!ARL) {
            const StepOut so = ftp_step(p, inv, oa, ob, mid, ask, bid, bmax, smin);
            code[w][lane] = (uint8_t)(so.fill_buy | (so.fill_sell << 1));
            rws[ARL ? 0 : w][lane] = so.reward;
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int s = 4 * w + c;
                const StepOut so = ftp_step(p, inv, oa + lut[0][s], ob + lut[1][s], mid, ask,
                                            bid, bmax, smin);
                code[s][lane] = (uint8_t)(so.fill_buy | (so.fill_sell << 1));
                rew[s * ep.rs + row] = so.reward;  // per-state planes (SoA): coalesced rows
            }
        }
    }
    __syncthreads();
    if (w != 0) return;
    const int64_t row = ep.step_off[e] + t0 + lane;
    if (ARL) {  // the fill codes (the scan derives the chunk transducers from them)
        uint64_t fw = 0;
        for (int s = 0; s < ns; ++s) fw |= (uint64_t)code[s][lane] << (2 * s);
        if (valid) fills[row] = fw;
        return;
    }
    uint64_t map = kIdentityMap;
    uint32_t traded = 0;
    if (valid) {
        for (int s = 0; s < nsi; ++s) {
            const uint32_t c = code[s][lane];
            const uint64_t to = (uint64_t)(s + (int)(c & 1u) - (int)(c >> 1));
            map = (map & ~(0xFFull << (8 * s))) | (to << (8 * s));
            traded |= (uint32_t)(c != 0) << s;
        }
    }
    // exclusive prefix of the chunk's step maps
    const uint64_t inc = wave_map_scan(map);
    uint64_t excl = shfl_up_u64(inc, 1);
    if (lane == 0) excl = kIdentityMap;
    uint64_t cnt = 0;
    for (int s0 = 0; s0 < nsi; ++s0) {
        const uint32_t st = map_get(excl, (uint32_t)s0);
        if (valid) rew[s0 * ep.rs + row] = rws[ARL ? 0 : st][lane];
        cnt |= (uint64_t)__popcll(__ballot(valid && ((traded >> st) & 1u))) << (8 * s0);
    }
    if (lane == kWave - 1) {
        const uint32_t ci = chunk_base(ep.step_off[e], e) + blockIdx.x;
        cmaps[ci] = inc;
        ctr[ci] = cnt;
    }
}

#ifdef SGMM_STAMPS
// diagnostic build only: phase timestamps (s_memtime) of the scan kernel per
// episode and of the table kernel per wave; slot 7 of a table wave holds
// s_memrealtime at entry (a clock common to all XCDs)
__device__ unsigned long long g_stamps[4096][16];
constexpr int kStampWaves = 1 << 16;
__device__ unsigned long long g_tstamps[kStampWaves][8];
__device__ unsigned int g_thwid[kStampWaves][2];  // HW_ID, XCC_ID of each table wave
#define SGMM_STAMP(e, k)                                                           \
    do {                                                                           \
        unsigned long long t_;                                                     \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        if (threadIdx.x == 0 && (e) < 4096) g_stamps[e][k] = t_;                   \
    } while (0)
#define SGMM_TSTAMP(w, k, dep)                                                     \
    do {                                                                           \
        unsigned long long t_;                                                     \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" \
                     : "=s"(t_) : "v"(dep) : "memory");                             \
        if ((threadIdx.x & 63) == 0 && (w) < kStampWaves) g_tstamps[w][k] = t_;    \
    } while (0)
#define SGMM_TSTAMP_REAL(w, k)                                                         \
    do {                                                                               \
        unsigned long long t_;                                                         \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        if ((threadIdx.x & 63) == 0 && (w) < kStampWaves) g_tstamps[w][k] = t_;        \
        unsigned h_, x_;                                                               \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)" \
                     : "=s"(h_), "=s"(x_));                                            \
        if ((threadIdx.x & 63) == 0 && (w) < kStampWaves) { g_thwid[w][0] = h_; g_thwid[w][1] = x_; } \
    } while (0)
#else
#define SGMM_STAMP(e, k) \
    do {                 \
    } while (0)
#define SGMM_TSTAMP(w, k, dep) \
    do {                       \
    } while (0)
#define SGMM_TSTAMP_REAL(w, k) \
    do {                       \
    } while (0)
#endif

// ------------------------------------------------------------------ table on the matrix cores
// gfx950's f32-input MFMA v_mfma_f32_16x16x4_f32 computes, per output, the
// k-ordered fused chain D = fma(a_k3,b_k3, fma(.., fma(a_k0,b_k0, C))) --
// exactly the canonical dot-product order of the numerics contract -- so the
// policy's H x H layer runs on the matrix pipe bit-identically to the
// VALU/oracle chains, with the weights held as compact per-lane fragments
// (loaded once per wave, reused for every tile).
//
// One wave = one 64-tick chunk of one episode; for each inventory state:
//   layer 1 (VALU):  h1[k][n] = relu(b1 + W1[k].(s1n, s2n, inv/2)), the two
//                    signal terms shared by all states;
//   layer 2 (MFMA):  H2^T[j][n] = W2[j][:] . H1^T[:][n] + b2[j], four 16-sample
//                    tiles (A = W2 rows, B = h1 at k = 4i + (lane>>4), C = b2);
//   transpose:       relu(H2) -> LDS as [sample][neuron] (one 16-byte write
//                    per tile and lane);
//   layer 3 (VALU):  lane n = tick n reads its H activations and runs the two
//                    canonical output chains b3[o] + sum_j W3[o][j] h2[j] (the
//                    2-row output would waste 7/8 of a 16-row MFMA tile).
// The lane then holds the policy outputs of its own tick for every state.

template <int H, int NSI, bool ARL>
__global__ __launch_bounds__(kWave * 4, H <= 16 ? 5 : ((ARL && H <= 32) ? 3 : 1)) void k_policy_table_mfma(
    sgmm_ticks tk, EpArrays ep, const sgmm_env_params* __restrict__ params,
    GenomeSrc src, int32_t inv_min, int32_t nsi, uint64_t* __restrict__ ctr,
    uint64_t* __restrict__ cmaps, uint64_t* __restrict__ fills, double* __restrict__ rew) {
    static_assert(H % 16 == 0, "MFMA table needs H multiple of 16");
    using L = GenomeLayout<H>;
    constexpr int NT = H / 16;   // 16-neuron row tiles of layer 2
    constexpr int KS = H / 4;    // k-steps (4 per MFMA)
    constexpr int HP = H + 4;    // LDS row pitch (floats) of the transposed activations
    const int e = blockIdx.y;
    const int32_t T = ep.len[e];
    const int chunk = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int32_t t0 = chunk * kChunk;
    if (blockIdx.x * 4 * kChunk >= T) return;  // block-uniform: no wave of this block has ticks
    const int lane = threadIdx.x & (kWave - 1), grp = lane >> 4, col = lane & 15;
    const int ns = ARL ? 4 * nsi : nsi;
    // this wave's tick data, requested before the genome staging so the loads
    // overlap it (indices clamped into the episode: padded samples are discarded)
    float xs0[4], xs1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t ti = ep.tick_off[e] + min(t0 + 16 * q + col, T - 1);
        xs0[q] = tk.s1n[ti];
        xs1[q] = tk.s2n[ti];
    }
    // the episode's genomes -> LDS (all four waves, before any of them leaves)
    __shared__ __attribute__((aligned(16))) float gsm[GenomeLayout<H>::N];
    __shared__ float gsa[kAdvParams];
    const int ai = (ARL && ep.adv) ? ep.adv[e] : -1;
    stage_genomes(src, e, ep.genome[e], ai, GenomeLayout<H>::N, gsm, ARL ? gsa : nullptr);
    __syncthreads();
    // layer-3 weights interleaved (W3[0][j], W3[1][j]) for the packed output chains
    __shared__ __attribute__((aligned(8))) float w3i[2 * H];
    if (threadIdx.x < 2 * H)
        w3i[threadIdx.x] = gsm[GenomeLayout<H>::W3 + (threadIdx.x & 1) * H + (threadIdx.x >> 1)];
    __syncthreads();
    if (t0 >= T) return;  // wave-uniform; no block barriers below
#ifdef SGMM_STAMPS
    const int wslot = e * (int)(gridDim.x * 4) + chunk;
#endif
    SGMM_TSTAMP_REAL(wslot, 7);
    SGMM_TSTAMP(wslot, 0, 0);
    const sgmm_env_params p = params[ep.param[e]];
    const float* g = gsm;
    const int64_t row = ep.step_off[e] + t0 + lane;  // this lane's output row
    __shared__ __attribute__((aligned(16))) float hb_s[4][kWave * HP];
    float* hb = hb_s[threadIdx.x >> 6];

    // ---- per-lane weight fragments (lane-dependent, tile-independent)
    float w2f[NT][KS];  // A of layer 2: neuron 16rt + col, k = 4i + grp
    f32x4 b2c[NT];      // C of layer 2: neurons 16rt + 4grp + r
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
        for (int i = 0; i < KS; ++i) w2f[rt][i] = g[L::W2 + (16 * rt + col) * H + 4 * i + grp];
#pragma unroll
        for (int r = 0; r < 4; ++r) b2c[rt][r] = g[L::B2 + 16 * rt + 4 * grp + r];
    }
    float w1s[KS];      // layer-1 inventory weight W1[k][2] for k = 4i + grp
    float pre[4][KS];   // b1[k] + W1[k][0] s1n + W1[k][1] s2n of sample 16q + col
    {
#pragma unroll
        for (int i = 0; i < KS; ++i) {
            const int k = 4 * i + grp;
            const float a0 = g[L::W1 + 3 * k], a1 = g[L::W1 + 3 * k + 1], bb = g[L::B1 + k];
            w1s[i] = g[L::W1 + 3 * k + 2];
#pragma unroll
            for (int q = 0; q < 4; ++q) pre[q][i] = __builtin_fmaf(a1, xs1[q], __builtin_fmaf(a0, xs0[q], bb));
        }
    }
    SGMM_TSTAMP(wslot, 1, w2f[0][0] + w1s[KS - 1] + pre[3][KS - 1] + b2c[0][0]);

    // ---- the policy for every (state, tick) of the chunk, software-pipelined:
    // the layer-2 MFMAs of state si+1 are issued beside the layer-3 chains of
    // state si (which read the activations si left in LDS), then state si+1 is
    // transposed.  One accumulator set, one activation buffer.
    float out0[NSI], out1[NSI];
    f32x4 acc[4][NT];
    auto layer12 = [&](int si) {  // layer 1 (packed fma) + layer 2 (MFMA) of state si
        const float x2 = (float)((double)(inv_min + si) / 2.0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int rt = 0; rt < NT; ++rt) acc[q][rt] = b2c[rt];
        // four independent 16-sample chains, issued interleaved (k-step outer);
        // layer 1's last term for two tiles per packed fma
#pragma unroll
        for (int i = 0; i < KS; ++i)
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const f32x2 hh = __builtin_elementwise_fma(f32x2{w1s[i], w1s[i]}, f32x2{x2, x2},
                                                           f32x2{pre[q][i], pre[q + 1][i]});
                const float h1a = relu(hh.x), h1b = relu(hh.y);
#pragma unroll
                for (int rt = 0; rt < NT; ++rt) {
                    acc[q][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[rt][i], h1a, acc[q][rt], 0, 0, 0);
                    acc[q + 1][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[rt][i], h1b, acc[q + 1][rt], 0, 0, 0);
                }
            }
    };
    auto transpose = [&]() {  // relu(H2) through LDS: lane n gets tick n's H activations
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int rt = 0; rt < NT; ++rt) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = relu(acc[q][rt][r]);
                *reinterpret_cast<f32x4*>(&hb[(16 * q + col) * HP + 16 * rt + 4 * grp]) = v;
            }
    };
    layer12(0);
    transpose();
#pragma unroll
    for (int si = 0; si < NSI; ++si) {
        out0[si] = out1[si] = 0.0f;
        if (si >= nsi) continue;
        const bool next = si + 1 < nsi;
        if (next) layer12(si + 1);
        f32x2 o = {g[L::B3], g[L::B3 + 1]};  // both output chains in one packed fma per neuron
#pragma unroll
        for (int j4 = 0; j4 < H / 4; ++j4) {
            const f32x4 h = *reinterpret_cast<const f32x4*>(&hb[lane * HP + 4 * j4]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f32x2 w = *reinterpret_cast<const f32x2*>(&w3i[2 * (4 * j4 + r)]);
                o = __builtin_elementwise_fma(w, f32x2{h[r], h[r]}, o);
            }
        }
        out0[si] = o.x;
        out1[si] = o.y;
        if (next) transpose();
    }
    // this lane's tick prices (loaded after the MLP: registers)
    const int64_t tix = ep.tick_off[e] + min(t0 + lane, T - 1);
    const double tmid = tk.mid_next[tix], task = tk.best_ask[tix], tbid = tk.best_bid[tix];
    const double tbmax = tk.buy_max[tix], tsmin = tk.sell_min[tix];
    SGMM_TSTAMP(wslot, 2, out0[NSI - 1] + out1[0]);

    // ---- FPT step from every state, one lane per tick
    const bool valid = t0 + lane < T;
    __shared__ int32_t lut_s[4][2][32];
    int32_t* lut0 = lut_s[threadIdx.x >> 6][0];
    int32_t* lut1 = lut_s[threadIdx.x >> 6][1];
    if (ARL) {
        if (lane < ns) {
            int32_t da = 0, db = 0;
            if (ai >= 0) adv_delta(gsa, p, inv_min + (lane >> 2), (lane >> 1) & 1, lane & 1, da, db);
            lut0[lane] = da;
            lut1[lane] = db;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    uint64_t map = kIdentityMap;
    uint32_t traded = 0;
    uint64_t fw = 0;
    // [state][lane] rewards, staged in the activation buffer (the MLP is done
    // with it; the asm is a compiler memory barrier: float and double views of
    // the same LDS must not be reordered)
    double* rl = reinterpret_cast<double*>(hb);
    static_assert(NSI * 2 <= HP, "reward staging fits the activation buffer");
    asm volatile("" ::: "memory");
    if (valid) {
        const double mid = tmid, ask = task, bid = tbid, bmax = tbmax, smin = tsmin;
#pragma unroll
        for (int si = 0; si < NSI; ++si) {
            if (si >= nsi) break;
            const int32_t inv = inv_min + si;
            const int32_t oa = act_to_int(rintf(out0[si] * p.act_scale));  // drl_engine.py:38-39
            const int32_t ob = act_to_int(rintf(out1[si] * p.act_scale));
            if (!ARL) {
                const StepOut so = ftp_step(p, inv, oa, ob, mid, ask, bid, bmax, smin);
                map = (map & ~(0xFFull << (8 * si))) |
                      ((uint64_t)(si + so.fill_buy - so.fill_sell) << (8 * si));
                traded |= (uint32_t)(so.fill_buy | so.fill_sell) << si;
                rl[si * kWave + lane] = so.reward;
            } else {
                // the 4 (previous fills) states of this inventory differ only by the
                // adversary's delta (wave-uniform: one adversary per episode); states
                // whose delta equals an earlier one's take that step's result
                // (adv_scale 1: deltas in {-1, 0, 1}, mostly shared)
                int32_t dac[4], dbc[4], fc[4];
                double rc[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int s = 4 * si + c;
                    dac[c] = __builtin_amdgcn_readfirstlane(lut0[s]);
                    dbc[c] = __builtin_amdgcn_readfirstlane(lut1[s]);
                    int dup = -1;
#pragma unroll
                    for (int c2 = c - 1; c2 >= 0; --c2)
                        if (dac[c2] == dac[c] && dbc[c2] == dbc[c]) dup = c2;
                    if (dup < 0) {
                        const StepOut so = ftp_step(p, inv, oa + dac[c], ob + dbc[c], mid, ask, bid, bmax, smin);
                        rc[c] = so.reward;
                        fc[c] = so.fill_buy | (so.fill_sell << 1);
                    } else {
                        rc[c] = dup == 0 ? rc[0] : (dup == 1 ? rc[1] : rc[2]);
                        fc[c] = dup == 0 ? fc[0] : (dup == 1 ? fc[1] : fc[2]);
                    }
                    fw |= (uint64_t)fc[c] << (2 * s);
                    rew[s * ep.rs + row] = rc[c];  // per-state planes (SoA): coalesced rows
                }
            }
        }
    }
    if (ARL) {  // the fill codes (the scan derives the chunk transducers from them)
        if (valid) fills[row] = fw;
        return;
    }
    SGMM_TSTAMP(wslot, 3, map + traded);
    const uint64_t inc = wave_map_scan(map);
    uint64_t excl = shfl_up_u64(inc, 1);
    if (lane == 0) excl = kIdentityMap;
    SGMM_TSTAMP(wslot, 4, excl);
    // path planes: plane s holds the reward along the chunk's path from start
    // state s; per start state the path's trade count (8 bits each)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    uint64_t cnt = 0;
#pragma unroll
    for (int s0 = 0; s0 < NSI; ++s0) {
        if (s0 >= nsi) break;
        const uint32_t st = map_get(excl, (uint32_t)s0);
        if (valid) rew[s0 * ep.rs + row] = rl[st * kWave + lane];
        cnt |= (uint64_t)__popcll(__ballot(valid && ((traded >> st) & 1u))) << (8 * s0);
    }
    if (lane == kWave - 1) {
        const uint32_t ci = chunk_base(ep.step_off[e], e) + chunk;
        cmaps[ci] = inc;
        ctr[ci] = cnt;
    }
#ifdef SGMM_STAMPS
    SGMM_TSTAMP(wslot, 5, 0);
    SGMM_TSTAMP_REAL(wslot, 6);
#endif
}

// ------------------------------------------------------------------ table v3: one state per MFMA stream
// Same outputs and arithmetic as k_policy_table_mfma (no adversary),
// re-scheduled: one accumulator set; per inventory state a vector block
// (relu + LDS transpose of state si, layer 1 of si+1, layer 3 and the FPT step
// of si) and a pure MFMA block (layer 2 of si+1).  f32 MFMAs and vector ops of
// ONE wave do not overlap on gfx950 (tools/mb/mb_mfma_valu.hip), so the blocks
// are kept apart and the overlap comes from the other waves of the SIMD.
// Every lane computes every state (padded lanes read a clamped tick and are
// masked out of the maps afterwards).  (Round 2's alternative with two
// accumulator sets interleaved, "v3i", and this schedule for the adversary
// table measured slower: tools/experiments/round3_opt_in_paths.patch.)
template <int H, int NSI>
__global__ __launch_bounds__(kWave * 4, H <= 16 ? (NSI <= 5 ? 5 : 4) : 2) void k_policy_table_v3(
    sgmm_ticks tk, EpArrays ep, const sgmm_env_params* __restrict__ params, GenomeSrc src,
    int32_t inv_min, int32_t nsi, uint64_t* __restrict__ ctr, uint64_t* __restrict__ cmaps,
    double* __restrict__ rew) {
    static_assert(H % 16 == 0 && H <= 32, "v3 table: H = 16 or 32");
    using L = GenomeLayout<H>;
    constexpr int NT = H / 16;   // 16-neuron row tiles of layer 2
    constexpr int KS = H / 4;    // k-steps (4 per MFMA)
    constexpr int HP = H + 4;    // LDS row pitch (floats) of the transposed activations
    const int e = blockIdx.y;
    const int32_t T = ep.len[e];
    const int wv = threadIdx.x >> 6;
    const int chunk = blockIdx.x * 4 + wv;
    const int32_t t0 = chunk * kChunk;
    if (blockIdx.x * 4 * kChunk >= T) return;  // block-uniform
    const int lane = threadIdx.x & (kWave - 1), grp = lane >> 4, col = lane & 15;
    const int64_t tb = ep.tick_off[e];
    // tick data requested before the genome staging so the loads overlap it
    // (indices clamped into the episode: padded samples are discarded)
    float xs0[4], xs1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t ti = tb + min(t0 + 16 * q + col, T - 1);
        xs0[q] = tk.s1n[ti];
        xs1[q] = tk.s2n[ti];
    }
    const int64_t tix = tb + min(t0 + lane, T - 1);
    const double tmid = tk.mid_next[tix], task = tk.best_ask[tix], tbid = tk.best_bid[tix];
    const double tbmax = tk.buy_max[tix], tsmin = tk.sell_min[tix];
    // the genome is staged in the reward buffer: it is dead once every wave
    // holds its weights in registers (the barrier below).  The LDS saved keeps
    // the H = 16 workgroup at 30.8 KB, so five fit a CU (96 VGPRs: five waves
    // per SIMD; config 2's table 21.3 -> 19.4 us)
    __shared__ __attribute__((aligned(16))) double rl_s[4][NSI][kWave];  // [state][lane] path-plane rewards
    static_assert(sizeof(rl_s) >= sizeof(float) * L::N, "genome fits the reward buffer");
    float* gsm = reinterpret_cast<float*>(&rl_s[0][0][0]);
    stage_genomes(src, e, ep.genome[e], -1, L::N, gsm, nullptr);
    __syncthreads();
    __shared__ __attribute__((aligned(16))) float w3i[2 * H];  // (W3[0][j], W3[1][j]) pairs
    if (threadIdx.x < 2 * H) w3i[threadIdx.x] = gsm[L::W3 + (threadIdx.x & 1) * H + (threadIdx.x >> 1)];
    const float* g = gsm;
    float w2f[NT][KS];  // A of layer 2: neuron 16rt + col, k = 4i + grp
    f32x4 b2c[NT];      // C of layer 2: neurons 16rt + 4grp + r
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
        for (int i = 0; i < KS; ++i) w2f[rt][i] = g[L::W2 + (16 * rt + col) * H + 4 * i + grp];
#pragma unroll
        for (int r = 0; r < 4; ++r) b2c[rt][r] = g[L::B2 + 16 * rt + 4 * grp + r];
    }
    float w1s[KS];      // W1[k][2], k = 4i + grp
    float pre[4][KS];   // b1[k] + W1[k][0] s1n + W1[k][1] s2n of sample 16q + col
#pragma unroll
    for (int i = 0; i < KS; ++i) {
        const int k = 4 * i + grp;
        const float a0 = g[L::W1 + 3 * k], a1 = g[L::W1 + 3 * k + 1], bb = g[L::B1 + k];
        w1s[i] = g[L::W1 + 3 * k + 2];
#pragma unroll
        for (int q = 0; q < 4; ++q) pre[q][i] = __builtin_fmaf(a1, xs1[q], __builtin_fmaf(a0, xs0[q], bb));
    }
    const float b30 = g[L::B3], b31 = g[L::B3 + 1];
    __syncthreads();      // the genome is dead: rl_s holds rewards from here
    if (t0 >= T) return;  // wave-uniform; no block barriers below
#ifdef SGMM_STAMPS
    // slots: 7 realtime at entry, 0 start, 1 weights + layer 1 of state 0,
    // 2 states done, 3 map scan, 4 end, 5 / 6 summed MFMA / vector blocks
    const int wslot = e * (int)(gridDim.x * 4) + chunk;
    unsigned long long st_m = 0, st_v = 0, st_a, st_b;
#define SGMM_V3T(var) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory")
#endif
    SGMM_TSTAMP_REAL(wslot, 7);
    SGMM_TSTAMP(wslot, 0, 0);
    const sgmm_env_params p = params[ep.param[e]];
    __shared__ __attribute__((aligned(16))) float hb_s[4][kWave * HP];
    float* hb = hb_s[wv];
    double* rl = &rl_s[wv][0][0];

    f32x4 acc[4][NT];
    uint64_t map = kIdentityMap;
    uint32_t traded = 0;
    const bool valid = t0 + lane < T;
    const int64_t row = ep.step_off[e] + t0 + lane;
    auto transpose = [&]() {  // relu(H2) -> LDS [sample][neuron]
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int rt = 0; rt < NT; ++rt) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = relu(acc[q][rt][r]);
                *reinterpret_cast<f32x4*>(&hb[(16 * q + col) * HP + 16 * rt + 4 * grp]) = v;
            }
    };
    auto layer3_env = [&](int si) {  // layer 3 of this lane's tick, then its FPT step from state si
        float o0 = b30, o1 = b31;
#pragma unroll
        for (int j4 = 0; j4 < H / 4; ++j4) {
            const f32x4 h = *reinterpret_cast<const f32x4*>(&hb[lane * HP + 4 * j4]);
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(&w3i[2 * (4 * j4 + 2 * r2)]);
                o0 = __builtin_fmaf(w[0], h[2 * r2], o0);
                o1 = __builtin_fmaf(w[1], h[2 * r2], o1);
                o0 = __builtin_fmaf(w[2], h[2 * r2 + 1], o0);
                o1 = __builtin_fmaf(w[3], h[2 * r2 + 1], o1);
            }
        }
        const int32_t oa = act_to_int(rintf(o0 * p.act_scale));  // drl_engine.py:38-39
        const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
        const StepOut so = ftp_step(p, inv_min + si, oa, ob, tmid, task, tbid, tbmax, tsmin);
        const bool live = si < nsi;  // states past the caps keep the identity byte
        const uint64_t to = live ? (uint64_t)(si + so.fill_buy - so.fill_sell) : (uint64_t)si;
        map = (map & ~(0xFFull << (8 * si))) | (to << (8 * si));
        traded |= (uint32_t)(live && (so.fill_buy | so.fill_sell)) << si;
        rl[si * kWave + lane] = so.reward;
    };
    {
        float h1[KS][4];
        auto layer1 = [&](int si) {
            const float x2 = (float)((double)(inv_min + si) / 2.0);
#pragma unroll
            for (int i = 0; i < KS; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) h1[i][q] = relu(__builtin_fmaf(w1s[i], x2, pre[q][i]));
        };
        auto layer2 = [&]() {
#pragma unroll
            for (int i = 0; i < KS; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int rt = 0; rt < NT; ++rt)
                        acc[q][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[rt][i], h1[i][q],
                                                                          i == 0 ? b2c[rt] : acc[q][rt], 0, 0, 0);
        };
        layer1(0);
        SGMM_TSTAMP(wslot, 1, h1[KS - 1][3] + pre[0][0] + w2f[0][0] + b2c[0][0]);
#ifdef SGMM_STAMPS
        SGMM_V3T(st_b);
#endif
        __builtin_amdgcn_sched_barrier(0);
        layer2();
#pragma unroll
        for (int si = 0; si < NSI; ++si) {
            __builtin_amdgcn_sched_barrier(0);
#ifdef SGMM_STAMPS
            SGMM_V3T(st_a);
            st_m += st_a - st_b;
#endif
            transpose();
            if (si + 1 < NSI) layer1(si + 1);
            layer3_env(si);
            __builtin_amdgcn_sched_barrier(0);
#ifdef SGMM_STAMPS
            SGMM_V3T(st_b);
            st_v += st_b - st_a;
#endif
            if (si + 1 < NSI) layer2();
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    SGMM_TSTAMP(wslot, 2, map + traded);
    if (!valid) {  // padded lanes: identity steps, no trades
        map = kIdentityMap;
        traded = 0;
    }
    const uint64_t inc = wave_map_scan(map);
    uint64_t excl = shfl_up_u64(inc, 1);
    if (lane == 0) excl = kIdentityMap;
    SGMM_TSTAMP(wslot, 3, excl);
    // path planes: plane s holds the reward along the chunk's path from start
    // state s; per start state the path's trade count (8 bits each)
    uint64_t cnt = 0;
#pragma unroll
    for (int s0 = 0; s0 < NSI; ++s0) {
        if (s0 >= nsi) break;
        const uint32_t st = map_get(excl, (uint32_t)s0);
        if (valid) rew[s0 * ep.rs + row] = rl[st * kWave + lane];
        cnt |= (uint64_t)__popcll(__ballot(valid && ((traded >> st) & 1u))) << (8 * s0);
    }
    if (lane == kWave - 1) {
        const uint32_t ci = chunk_base(ep.step_off[e], e) + chunk;
        cmaps[ci] = inc;
        ctr[ci] = cnt;
    }
#ifdef SGMM_STAMPS
    SGMM_TSTAMP(wslot, 4, 0);
    if (lane == 0 && wslot < kStampWaves) {
        g_tstamps[wslot][5] = st_m;
        g_tstamps[wslot][6] = st_v;
    }
#undef SGMM_V3T
#endif
}

// ------------------------------------------------------------------ walk order feedback
// A launch with whole walks and walks in halves (frontier_plan's four-walk
// rule, config 3: 1 024 whole + 1 536 in halves) ends with its heaviest whole
// walk: the walks of a GA-trained population differ in how long their paths
// stay apart, and the populations differ in how heavy their tails are
// (config 3 after 15 generations: the heaviest whole walk of population 0 ran
// 167 slots / 557 us, population 1's 116; every half walk ended by 430 us;
// profiles/r05_timeline/tlo_*).  After each training launch of
// sgmm_generation_multi_best this kernel ranks the populations by the heaviest
// episode they just ran -- a whole walk's slots x 5, an episode in halves the
// sum of its halves' slots x 4 (the halves' extra chunk starts: ~25 % more
// slots for the same episode) -- and rewrites the order so the next launch
// walks the lightest populations whole and cuts the heaviest into halves.
// Scheduling only: every result is per episode and independent of the order.
// (SGMM_FRONTIER_REORDER=0 keeps the caller's order.)
// The job rides along as one extra workgroup of the validation table launch
// that follows (k_policy_table_sp), which hides its ~6 us of latency; alone
// (k_walk_reorder) where that launch takes another path.
constexpr int kReorderMaxPops = 64;
struct ReorderJob {
    const uint32_t* wslots;
    int32_t* order;  // null: no job
    int32_t n, whole, gtail, pop_eps;
    uint32_t w_whole = 5, w_split = 4;  // score weights (SGMM_PLAN_REORDER_WEIGHTS for experiments)
    int32_t len = 0;                    // the episodes' (common) length: groups past the last chunk have no count
};
__device__ __forceinline__ void walk_reorder_block(const ReorderJob rj) {
    const uint32_t* __restrict__ wslots = rj.wslots;
    int32_t* __restrict__ order = rj.order;
    const int32_t n = rj.n, whole = rj.whole, gtail = rj.gtail, pop_eps = rj.pop_eps;
    const int nt = (int)blockDim.x;
    // an episode in gtail groups has chunks in the first ceil(nch / 64) only (the
    // frontier kernel writes no slot count for an empty group)
    const int cl = frontier_len(max(rj.len, 1), gtail);
    const int gused = min(gtail, (((rj.len + cl - 1) / cl) + kFrontierLanes - 1) / kFrontierLanes);
    __shared__ uint32_t score[kReorderMaxPops];
    __shared__ int32_t rank[kReorderMaxPops];
    const int npop = n / pop_eps;
    if ((int)threadIdx.x < npop) score[threadIdx.x] = 0;
    __syncthreads();
    // four positions per thread in flight: the order loads, then the slot loads (two
    // dependent load rounds per 4 096 positions instead of two per 1 024)
    constexpr int kPer = 4;
    for (int base = 0; base < n; base += nt * kPer) {
        int e[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int pos = base + j * nt + (int)threadIdx.x;
            e[j] = pos < n ? order[pos] : -1;
        }
        uint32_t sc[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j) {  // the episode's walks' slots at wslots[e * gtail + g]
            const int pos = base + j * nt + (int)threadIdx.x;
            sc[j] = 0;
            if (e[j] < 0) continue;
            if (pos < whole) {
                sc[j] = rj.w_whole * wslots[e[j] * gtail];
            } else {
                uint32_t sum = 0;
                for (int g = 0; g < gused; ++g) sum += wslots[e[j] * gtail + g];
                sc[j] = rj.w_split * sum;
            }
        }
        // one LDS atomic per wave where its 64 positions are one population (the usual
        // case: the order is population blocks), per lane otherwise
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int k = e[j] < 0 ? -1 : e[j] / pop_eps;
            const int k0 = __builtin_amdgcn_readfirstlane(k);
            if (__all(k == k0)) {
                uint32_t m = sc[j];
#pragma unroll
                for (int d = 1; d < kWave; d <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, kWave));
                if ((threadIdx.x & (kWave - 1)) == 0 && k0 >= 0) atomicMax(&score[k0], m);
            } else if (k >= 0) {
                atomicMax(&score[k], sc[j]);
            }
        }
    }
    __syncthreads();  // every read of the old order precedes the writes below
    if (threadIdx.x == 0) {  // populations by (score, index), lightest first
        for (int k = 0; k < npop; ++k) rank[k] = k;
        for (int i = 1; i < npop; ++i)
            for (int j = i; j > 0 && score[rank[j]] < score[rank[j - 1]]; --j) {
                const int t = rank[j];
                rank[j] = rank[j - 1];
                rank[j - 1] = t;
            }
    }
    __syncthreads();
    for (int pos = threadIdx.x; pos < n; pos += blockDim.x) order[pos] = rank[pos / pop_eps] * pop_eps + pos % pop_eps;
}
__global__ __launch_bounds__(1024) void k_walk_reorder(ReorderJob rj) { walk_reorder_block(rj); }
// ------------------------------------------------------------------ table, one state per wave (small launches)
// The v3 table's arithmetic with its state loop spread over the workgroup: one
// workgroup per 64-tick chunk, wave si runs layers 1-3 and the FPT step from
// inventory state si, and wave 0 assembles the chunk's map, path planes and
// trade counts from the states' successor bytes and rewards in LDS.  For
// launches with few chunks (the validation rollouts: 5 x 15 chunks at config
// 3) the v3 wave's serial five-state chain is the launch's latency; here it is
// one state deep.  Outputs are identical to v3's (same per-tick arithmetic).
template <int H, int NSI>
__global__ __launch_bounds__(kWave * NSI) void k_policy_table_sp(
    sgmm_ticks tk, EpArrays ep, const sgmm_env_params* __restrict__ params, GenomeSrc src,
    int32_t inv_min, int32_t nsi, uint64_t* __restrict__ ctr, uint64_t* __restrict__ cmaps,
    double* __restrict__ rew, ReorderJob rj) {
    static_assert(H % 16 == 0 && H <= 32, "state-parallel table: H = 16 or 32");
    using L = GenomeLayout<H>;
    constexpr int NT = H / 16, KS = H / 4, HP = H + 4;
    if (rj.order && blockIdx.y == gridDim.y - 1) {  // the extra workgroup: the walk-order job
        if (blockIdx.x == 0) walk_reorder_block(rj);
        return;
    }
    const int e = blockIdx.y;
    const int32_t T = ep.len[e];
    const int chunk = blockIdx.x;
    const int32_t t0 = chunk * kChunk;
    if (t0 >= T) return;  // block-uniform
    const int si = threadIdx.x >> 6;  // this wave's inventory state (blockDim = 64 nsi)
    const int lane = threadIdx.x & (kWave - 1), grp = lane >> 4, col = lane & 15;
    const int64_t tb = ep.tick_off[e];
    float xs0[4], xs1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t ti = tb + min(t0 + 16 * q + col, T - 1);
        xs0[q] = tk.s1n[ti];
        xs1[q] = tk.s2n[ti];
    }
    const int64_t tix = tb + min(t0 + lane, T - 1);
    const double tmid = tk.mid_next[tix], task = tk.best_ask[tix], tbid = tk.best_bid[tix];
    const double tbmax = tk.buy_max[tix], tsmin = tk.sell_min[tix];
    __shared__ __attribute__((aligned(16))) float gsm[L::N];
    __shared__ __attribute__((aligned(16))) float w3i[2 * H];
    __shared__ __attribute__((aligned(16))) float hb_s[NSI][kWave * HP];
    __shared__ __attribute__((aligned(16))) double rl_s[NSI][kWave];  // [state][lane] rewards
    __shared__ uint8_t to_s[NSI][kWave];  // successor state | traded << 7
    stage_genomes(src, e, ep.genome[e], -1, L::N, gsm, nullptr);
    __syncthreads();
    if (threadIdx.x < 2 * H) w3i[threadIdx.x] = gsm[L::W3 + (threadIdx.x & 1) * H + (threadIdx.x >> 1)];
    const float* g = gsm;
    float w2f[NT][KS];
    f32x4 b2c[NT];
#pragma unroll
    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
        for (int i = 0; i < KS; ++i) w2f[rt][i] = g[L::W2 + (16 * rt + col) * H + 4 * i + grp];
#pragma unroll
        for (int r = 0; r < 4; ++r) b2c[rt][r] = g[L::B2 + 16 * rt + 4 * grp + r];
    }
    const float x2 = (float)((double)(inv_min + si) / 2.0);
    float h1[KS][4];
#pragma unroll
    for (int i = 0; i < KS; ++i) {
        const int k = 4 * i + grp;
        const float a0 = g[L::W1 + 3 * k], a1 = g[L::W1 + 3 * k + 1], bb = g[L::B1 + k], w1s = g[L::W1 + 3 * k + 2];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            h1[i][q] = relu(__builtin_fmaf(w1s, x2, __builtin_fmaf(a1, xs1[q], __builtin_fmaf(a0, xs0[q], bb))));
    }
    const float b30 = g[L::B3], b31 = g[L::B3 + 1];
    __syncthreads();  // w3i complete
    const sgmm_env_params p = params[ep.param[e]];
    float* hb = hb_s[si];
    f32x4 acc[4][NT];
#pragma unroll
    for (int i = 0; i < KS; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int rt = 0; rt < NT; ++rt)
                acc[q][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[rt][i], h1[i][q], i == 0 ? b2c[rt] : acc[q][rt],
                                                                  0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int rt = 0; rt < NT; ++rt) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = relu(acc[q][rt][r]);
            *reinterpret_cast<f32x4*>(&hb[(16 * q + col) * HP + 16 * rt + 4 * grp]) = v;
        }
    float o0 = b30, o1 = b31;
#pragma unroll
    for (int j4 = 0; j4 < H / 4; ++j4) {
        const f32x4 h = *reinterpret_cast<const f32x4*>(&hb[lane * HP + 4 * j4]);
#pragma unroll
        for (int r2 = 0; r2 < 2; ++r2) {
            const f32x4 w = *reinterpret_cast<const f32x4*>(&w3i[2 * (4 * j4 + 2 * r2)]);
            o0 = __builtin_fmaf(w[0], h[2 * r2], o0);
            o1 = __builtin_fmaf(w[1], h[2 * r2], o1);
            o0 = __builtin_fmaf(w[2], h[2 * r2 + 1], o0);
            o1 = __builtin_fmaf(w[3], h[2 * r2 + 1], o1);
        }
    }
    const int32_t oa = act_to_int(rintf(o0 * p.act_scale));  // drl_engine.py:38-39
    const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
    const StepOut so = ftp_step(p, inv_min + si, oa, ob, tmid, task, tbid, tbmax, tsmin);
    to_s[si][lane] = (uint8_t)((si + so.fill_buy - so.fill_sell) | ((so.fill_buy | so.fill_sell) << 7));
    rl_s[si][lane] = so.reward;
    __syncthreads();
    if (si != 0) return;
    // wave 0: the chunk's map, path planes and trade counts (v3's tail)
    const bool valid = t0 + lane < T;
    uint64_t map = kIdentityMap;
    uint32_t traded = 0;
    if (valid) {
        for (int s = 0; s < nsi; ++s) {
            const uint32_t b = to_s[s][lane];
            map = (map & ~(0xFFull << (8 * s))) | ((uint64_t)(b & 0x7Fu) << (8 * s));
            traded |= (b >> 7) << s;
        }
    }
    const uint64_t inc = wave_map_scan(map);
    uint64_t excl = shfl_up_u64(inc, 1);
    if (lane == 0) excl = kIdentityMap;
    const int64_t row = ep.step_off[e] + t0 + lane;
    uint64_t cnt = 0;
#pragma unroll
    for (int s0 = 0; s0 < NSI; ++s0) {
        if (s0 >= nsi) break;
        const uint32_t st = map_get(excl, (uint32_t)s0);
        if (valid) rew[s0 * ep.rs + row] = rl_s[st][lane];
        cnt |= (uint64_t)__popcll(__ballot(valid && ((traded >> st) & 1u))) << (8 * s0);
    }
    if (lane == kWave - 1) {
        const uint32_t ci = chunk_base(ep.step_off[e], e) + chunk;
        cmaps[ci] = inc;
        ctr[ci] = cnt;
    }
}


// ------------------------------------------------------------------ exact ordered sum
// The episode total is the reference's sequential float64 sum
// (drl_engine.py:53: total = ((0 + r0) + r1) + ...).  It is evaluated in
// parallel, bit-exactly, from one property of IEEE addition: while the running
// sum S stays inside one binade [2^e, 2^(e+1)) (either sign) it is an integer
// multiple M of u = 2^(e-52), and fl(S + r) = (M + rint(r/u)) * u exactly as
// long as the exact S + r stays inside the binade and r/u is not a tie (x.5).
// So a stretch of ticks that keeps one binade adds up as 64-bit integers.
//
// A window of 4 NT values, cut into NT/4 blocks of 16 values, one block per
// lane of the first NT/256 waves:
//   a. float32 approximate block starts (wave scan + the waves' totals);
//   b. per block: the binade predicted from its approximate start, its integer
//      steps d = rint(r/u), their prefix range and a flag for ties / huge
//      steps / a predicted range near the binade's edges.  Blocks of one wave
//      that share a predicted binade form a run; every block gets the record
//      of the rest of its run (segmented suffix min / max of the integer
//      prefixes, the run's integer sum, its end); wave 0 extends each wave's
//      head record over the following waves;
//   c. one lane walks the blocks from the exact S, kept as (binade, integer
//      M) between fallback blocks: if S's binade is the block's prediction
//      and M plus the run's prefix range stays strictly inside [2^52, 2^53),
//      the whole rest of the run is added as one integer; otherwise the block
//      is added with the reference's float64 additions and the walk moves to
//      the next block.
// Every accepted shortcut is exact by the property above, so the result is
// the sequential sum bit for bit.  On a bench episode the walk takes ~10
// fallback blocks (the sum's doublings: ticks 2, 3, 6, 16, 22, 43, 85, ...)
// and ~11 run jumps.
constexpr int kSumBlk = 16;
constexpr int kSumTpt = 4;          // rewards gathered per path-scan thread
constexpr int kScanThreads = 1024;  // path-scan workgroup
constexpr int kScanWin = kScanThreads * kSumTpt;
constexpr int kScanAt1024 = 256;  // path-scan workgroup: 1024 threads up to this many episodes,
constexpr int kScanAt512 = 512;   // 256 up to this many, one wave above
constexpr int kScanArlAt1024 = 1024;  // adversary path scan: 1024 threads up to this many, kScanBlock above
constexpr int64_t kMLo = (1LL << 52) + 1, kMHi = (1LL << 53) - 1;
constexpr int32_t kZeroRun = INT32_MAX;  // a block's prediction: all its values are +-0.0
constexpr int kHeadBlocks = 8;           // blocks added the reference way when a sum starts at +0.0
constexpr int64_t kEdge = 1LL << 40;  // prediction margin at the binade edges (2^-12 relative)
static_assert(kChunk % kSumTpt == 0, "a thread's ticks lie in one chunk");

// S = M * 2^(e-52) with |M| in [2^52, 2^53); false unless S is normal with
// |e| <= 900 (the shortcut's range: 2^(52-e) and its inverse stay normal)
__device__ __forceinline__ bool binade_of(double s, int& e, int64_t& m) {
    const int64_t bits = __double_as_longlong(s);
    const int be = (int)((bits >> 52) & 0x7FF);
    e = be - 1023;
    const int64_t mag = (bits & 0xFFFFFFFFFFFFFLL) | (1LL << 52);
    m = bits < 0 ? -mag : mag;
    return be >= 1023 - 900 && be <= 1023 + 900;
}

__device__ __forceinline__ double from_binade(int64_t m, int e) {
    const int64_t mag = m < 0 ? -m : m;  // in [2^52, 2^53)
    const int64_t bits = ((int64_t)(e + 1023) << 52) | (mag - (1LL << 52));
    return __longlong_as_double(m < 0 ? (bits | INT64_MIN) : bits);
}

__device__ __forceinline__ double uniform_f64(double v) {
    const long long b = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ double pow2(int k) {  // k in [-1022, 1023]
    return __longlong_as_double((int64_t)(k + 1023) << 52);
}

__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {
    const int lo = __shfl((int)(uint32_t)v, src, kWave);
    const int hi = __shfl((int)(uint32_t)((uint64_t)v >> 32), src, kWave);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// inclusive float32 prefix sum over the wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ float wave_scan_add_f32(float v) {
#define SGMM_FSTEP(CTRL, RM) \
    v += __int_as_float((int)dpp32<CTRL, RM>(0u, (uint32_t)__float_as_int(v)));
    SGMM_FSTEP(0x111, 0xF) SGMM_FSTEP(0x112, 0xF) SGMM_FSTEP(0x114, 0xF)
    SGMM_FSTEP(0x118, 0xF) SGMM_FSTEP(0x142, 0xA) SGMM_FSTEP(0x143, 0xC)
#undef SGMM_FSTEP
    return v;
}

// the walk's view of block b: the rest of its run [b, rend)
struct SumRec {
    int64_t mn, mx;  // min / max of the integer prefixes over the run, relative to b's start
    int64_t dsum;    // integer sum of blocks b .. rend-1
    int32_t be;      // predicted binade (INT32_MIN: none, tie, huge step, or past the end)
    int32_t rend;    // first block after b (window index) with another prediction, or the wave's end
};

template <int NT>
struct SumLds {
    SumRec rec[NT / 4];
    float w_ap[NT / kWave];
    double S;
};

// All NT threads call once sel[0, n) holds the window's values (n <= 4 NT)
// and a barrier has passed; returns S + sel[0] + ... + sel[n-1] in sequential
// float64 order in every thread.  S must be the same in every thread.  Ends
// with a barrier (sel may then be refilled).
// A block without a prediction takes the rest of its run with it: one loop of
// reference additions, no walk step per block (see the walk below).
template <int NT>
__device__ __forceinline__ double exact_sum_window(const double* sel, int n, double S, SumLds<NT>& L,
                                                   bool seq = false) {
    static_assert(NT % (4 * kWave) == 0, "whole block waves");
    if (seq) {
        // the plain sequential chain: wave 0's lanes add the window from LDS
        // broadcast reads in the reference's order, one dependent add per value
        // (32 values per LDS round trip: 71 against 75 us with 16 on config 3, 64
        // need 226 VGPRs -- two waves per SIMD).  Faster than the parallel method below
        // where its fallbacks are many or its window phases are not hidden (the
        // one-wave scans of thousands of GA-trained episodes, the validation
        // scans); rollout_impl chooses (scan_seq_sum)
        if (threadIdx.x < kWave) {
            double s = S;
            const double2* p = reinterpret_cast<const double2*>(sel);
            const int n16 = n & ~15;
            int i = 0;
            // (pinning the next 16 values ahead of this 16's adds -- asm operands, which
            // wait for them -- measured slower: 99 against 76 us on config 3,
            // profiles/r06_seq2_*)
#ifndef SGMM_SEQ_CHUNK
#define SGMM_SEQ_CHUNK 32
#endif
            constexpr int kC = SGMM_SEQ_CHUNK;
            const int nc = n & ~(kC - 1);
            for (; i < nc; i += kC) {
                double2 v[kC / 2];
#pragma unroll
                for (int j = 0; j < kC / 2; ++j) v[j] = p[i / 2 + j];
#pragma unroll
                for (int j = 0; j < kC / 2; ++j) {
                    s += v[j].x;
                    s += v[j].y;
                }
            }
            (void)n16;
            for (; i < n; ++i) s += sel[i];
            if (threadIdx.x == 0) L.S = s;
        }
        __syncthreads();
        return L.S;
    }
    constexpr int NB = NT / 4;         // 16-value blocks per window
    constexpr int NWB = NB / kWave;    // waves holding one block per lane
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid >> 6;
    const int b = tid;                 // this lane's block (waves < NWB)
    const int i0 = b * kSumBlk;
    const bool blk = wv < NWB;         // wave-uniform
    const bool live = blk && i0 < n;
    double r[kSumBlk];
    float fex = 0.0f;
    if (blk) {
        // the block's values; the last block padded with -0.0 in LDS (x + -0.0
        // == x for every x, -0.0 and NaN included), so a fallback block always
        // adds 16 values
#pragma unroll
        for (int j = 0; j < kSumBlk; j += 2) {
            const double2 v = live ? *reinterpret_cast<const double2*>(sel + i0 + j) : double2{0.0, 0.0};
            r[j] = i0 + j < n ? v.x : 0.0;
            r[j + 1] = i0 + j + 1 < n ? v.y : 0.0;
        }
        if (live && i0 + kSumBlk > n)
            for (int j = n - i0; j < kSumBlk; ++j) const_cast<double*>(sel)[i0 + j] = -0.0;
        // a. approximate block starts (binade predictions only: float32 is enough)
        double a = 0.0;
#pragma unroll
        for (int j = 0; j < kSumBlk; ++j) a += r[j];
        const float fv = (float)a;
        const float finc = wave_scan_add_f32(fv);
        fex = finc - fv;
        if (lane == kWave - 1) L.w_ap[wv] = finc;
    }
    __syncthreads();
    SGMM_STAMP(blockIdx.x, 8);
    if (blk) {
        float woff = 0.0f;  // the preceding block waves' totals (broadcast reads, in order)
#pragma unroll
        for (int k = 0; k < NWB; ++k) woff += k < wv ? L.w_ap[k] : 0.0f;
        // b. integer steps of the block in its predicted binade
        int eb = 0;
        int64_t ma = 0;  // the approximate start's mantissa
        const bool fast = live && binade_of(S + (double)(woff + fex), eb, ma);
        const double sc52 = pow2(52 - (fast ? eb : 0));
        bool bad = !fast;
        int64_t P = 0, mn = INT64_MAX, mx = INT64_MIN;
        // rint by the 1.5 * 2^52 shifter: for |q| < 2^51, q + 1.5 * 2^52 lands
        // in [2^52, 2^53) (ulp 1), so the addition rounds q half-to-even and the
        // integer is the difference of the bit patterns; a tie is |rint(q) - q|
        // == 0.5 (exact: both are multiples of ulp(q) <= 1/4).  Larger steps
        // leave the binade anyway: the block is flagged.
        constexpr double kShift = 0x1.8p52;
#pragma unroll
        for (int j = 0; j < kSumBlk; ++j) {
            const double qv = r[j] * sc52;
            const double t = qv + kShift;
            const bool bj = !(fabs(qv) < 0x1p51) || fabs((t - kShift) - qv) == 0.5;
            const bool use = fast && i0 + j < n;
            bad |= use && bj;
            const int64_t d = (use && !bj) ? __double_as_longlong(t) - __double_as_longlong(kShift) : 0;
            P += d;
            mn = min(mn, P);
            mx = max(mx, P);
        }
        // a block whose predicted prefix comes within 2^-12 of the binade's
        // edges (the float32 start's error is far below that) most likely
        // crosses it: no prediction, so the runs before it stay fast and it is
        // added the reference way
        const bool edge = fast && (ma > 0 ? (ma + mx > kMHi - kEdge || ma + mn < kMLo + kEdge)
                                          : (ma + mn < -kMHi + kEdge || ma + mx > -kMLo - kEdge));
        // a block of exact zeros (either sign) leaves any S unchanged (S is
        // never -0.0: the sum starts at +0.0 and round-to-nearest cancels to
        // +0.0), whatever its binade -- runs of them are skipped whole, which is
        // what keeps an idle individual's walk (S = 0 for the whole episode:
        // every block was a fallback) as short as a trading one's
        bool allz = true;
#pragma unroll
        for (int j = 0; j < kSumBlk; ++j) allz &= r[j] == 0.0;
        const int32_t be = allz ? kZeroRun : (fast && !bad && !edge) ? eb : INT32_MIN;
#ifdef SGMM_STAMPS
        {   // why blocks have no prediction: [6] += no binade | bad step << 20 | binade edge << 40, [7] += zero blocks
            const unsigned long long nf = __popcll(__ballot(live && !allz && !fast));
            const unsigned long long nb = __popcll(__ballot(live && !allz && fast && bad));
            const unsigned long long ne = __popcll(__ballot(live && !allz && fast && !bad && edge));
            const unsigned long long nz = __popcll(__ballot(live && allz));
            if (lane == 0 && blockIdx.x < 4096) {
                atomicAdd(&g_stamps[blockIdx.x][6], nf | nb << 20 | ne << 40);
                atomicAdd(&g_stamps[blockIdx.x][7], nz);
            }
        }
#endif
        // block sums -> wave-local exclusive prefix zl
        const uint64_t zinc = wave_scan_add((uint64_t)P);
        const int64_t zl = (int64_t)(zinc - (uint64_t)P);
        const int64_t wtot = (int64_t)readlane64(zinc, kWave - 1);
        // runs inside the wave: a block starts a run when its prediction
        // differs from the previous block's
        const int32_t bprev = __shfl_up(be, 1, kWave);
        const uint64_t starts = __ballot(lane == 0 || be != bprev);
        const uint64_t later = lane == kWave - 1 ? 0ull : starts & (~0ull << (lane + 1));
        const int rq = later ? __ffsll((unsigned long long)later) - 1 : kWave;
        // segmented suffix min / max of the in-wave prefix extremes over [lane, rq)
        int64_t amn = zl + mn, amx = zl + mx;
#ifndef SGMM_SUFFIX_BPERMUTE
        // inside each 16-lane row by DPP row shifts (lane i reads lane i + d of its
        // row: no LDS round trip), then across rows from the three row heads
        // (readlane): a lane whose run goes on into row k > its row takes row k's
        // head, which covers [16k, min(rq, 16k + 16)) of the same run
        {
            const int rl_ = lane & 15;
#define SGMM_SEG_STEP(D)                                                                   \
    {                                                                                      \
        const int64_t omn = (int64_t)dpp64<0x100 + D>((uint64_t)INT64_MAX, (uint64_t)amn); \
        const int64_t omx = (int64_t)dpp64<0x100 + D>((uint64_t)INT64_MIN, (uint64_t)amx); \
        if (rl_ + D < 16 && lane + D < rq) {                                               \
            amn = min(amn, omn);                                                           \
            amx = max(amx, omx);                                                           \
        }                                                                                  \
    }
            SGMM_SEG_STEP(1) SGMM_SEG_STEP(2) SGMM_SEG_STEP(4) SGMM_SEG_STEP(8)
#undef SGMM_SEG_STEP
            const int row = lane >> 4;
#pragma unroll
            for (int k = 1; k < 4; ++k) {
                const int64_t hmn = (int64_t)readlane64((uint64_t)amn, 16 * k);
                const int64_t hmx = (int64_t)readlane64((uint64_t)amx, 16 * k);
                if (row < k && rq > 16 * k) {
                    amn = min(amn, hmn);
                    amx = max(amx, hmx);
                }
            }
        }
#else
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int64_t omn = shfl_i64(amn, min(lane + d, kWave - 1));
            const int64_t omx = shfl_i64(amx, min(lane + d, kWave - 1));
            if (lane + d < rq) {
                amn = min(amn, omn);
                amx = max(amx, omx);
            }
        }
#endif
        const int64_t zr = shfl_i64(zl, min(rq, kWave - 1));
        SumRec rc;
        rc.mn = amn - zl;
        rc.mx = amx - zl;
        rc.dsum = (rq < kWave ? zr : wtot) - zl;
        rc.be = be;
        rc.rend = wv * kWave + rq;
        L.rec[b] = rc;
    }
    __syncthreads();
    SGMM_STAMP(blockIdx.x, 9);
    // c. the walk (wave 0, scalar control flow, every lane carries S)
    if (wv == 0) {
        const int nblk = (n + kSumBlk - 1) / kSumBlk;
        // runs across waves: the head record of wave w (its run starts at the
        // wave's first block) is extended over the following waves while each
        // is one run with the same prediction -- a segmented suffix scan of
        // (min, max, sum) over the heads, lanes w < NT/64
        constexpr int NW = NT / (4 * kWave);  // block waves
        if (lane < NW) {
            const SumRec h = L.rec[lane * kWave];
            const int32_t bnext = __shfl_down(h.be, 1, kWave);
            const bool link = lane + 1 < NW && h.rend == (lane + 1) * kWave && bnext == h.be;
            const uint64_t brk = __ballot(!link) & ((1ull << NW) - 1);
            const uint64_t atl = brk & (~0ull << lane);  // the first break at or after this wave
            const int k = __ffsll((unsigned long long)atl) - 1;
            int64_t mn = h.mn, mx = h.mx, ds = h.dsum;
            int32_t re = h.rend;
#pragma unroll
            for (int d = 1; d < NW; d <<= 1) {
                const int src = min(lane + d, NW - 1);
                const int64_t omn = shfl_i64(mn, src), omx = shfl_i64(mx, src), ods = shfl_i64(ds, src);
                const int32_t ore = __shfl(re, src, kWave);
                if (lane + d <= k) {
                    mn = min(mn, ds + omn);
                    mx = max(mx, ds + omx);
                    ds += ods;
                    re = ore;
                }
            }
            SumRec& hw = L.rec[lane * kWave];
            hw.mn = mn;
            hw.mx = mx;
            hw.dsum = ds;
            hw.rend = re;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
#ifdef SGMM_STAMPS
        unsigned long long n_iter = 0, n_slow = 0;
#endif
        // One lane walks, carrying S as (binade e, integer M) between
        // fallback blocks: a run jump is integer work only (M += the run's
        // sum), S is rebuilt as a double just for a fallback block's reference
        // additions.  Both possible next records (pos + 1 and the run end) are
        // requested as soon as the current one arrives.
        constexpr int NB = NT / 4;
        // the walk is the episode's serial chain: first call on its SIMD's issue
        // while it runs (the other waves there are in their window phases)
#ifndef SGMM_NO_WALK_PRIO
        __builtin_amdgcn_s_setprio(3);
#endif
        if (lane == 0 && nblk > 0) {
            int pos = 0;
            int e = 0;
            int64_t M = 0;
            bool ib = binade_of(S, e, M);  // S = M * 2^(e-52) exactly while ib
#ifndef SGMM_NO_HEAD_STREAK
            // an episode's sum starts at +0.0 and doubles every few ticks at first
            // (ticks 2, 3, 6, 16, 22, 43, 85, ...): its first kHeadBlocks blocks
            // are walk steps that almost all fall back, so they are added the
            // reference way in one loop
            if (__double_as_longlong(S) == 0) {
                const int pe = min(kHeadBlocks, nblk);
                const double2* hp = reinterpret_cast<const double2*>(sel);
                double s = S;
                for (int b = 0; b < pe; ++b) {
                    double2 v[kSumBlk / 2];
#pragma unroll
                    for (int j = 0; j < kSumBlk / 2; ++j) v[j] = hp[b * (kSumBlk / 2) + j];
#pragma unroll
                    for (int j = 0; j < kSumBlk / 2; ++j) {
                        s += v[j].x;
                        s += v[j].y;
                    }
                }
#ifdef SGMM_STAMPS
                n_slow += pe;
#endif
                S = s;
                ib = binade_of(s, e, M);
                pos = pe;
            }
#endif
            SumRec cur = L.rec[min(pos, NB - 1)];
            while (pos < nblk) {
#ifdef SGMM_STAMPS
                ++n_iter;
#endif
                const SumRec rn = L.rec[min(pos + 1, NB - 1)];
                const SumRec rj = L.rec[min(cur.rend, NB - 1)];
                // (a zero run is skipped unless S is -0.0: only the API's init can make it so)
                // every term evaluated, combined bitwise: no branch per term on the
                // walk's serial chain (the short-circuit form compiled to 4-5 branches;
                // measured the same, profiles/r04_ab/r04af*)
                const int64_t lo_ = M + cur.mn, hi_ = M + cur.mx;
                const bool pos_ok = (lo_ >= kMLo) & (hi_ <= kMHi);
                const bool neg_ok = (hi_ <= -kMLo) & (lo_ >= -kMHi);
                const bool zero_ok = (cur.be == kZeroRun) & (ib | (__double_as_longlong(S) != INT64_MIN));
                const bool ok = zero_ok | (ib & (cur.be == e) & (M > 0 ? pos_ok : neg_ok));
                const int64_t Mj = M + cur.dsum;
                const int pj = cur.rend;
                // a block without a prediction is added the reference way whatever
                // S is, and so is the rest of its run (every block of [pos, rend)
                // has none): the whole streak in one loop of 8 values per LDS
                // round trip (a sum crossing zero or sitting on a binade edge makes
                // such streaks: the slowest episodes' walks were 70-171 one-block
                // fallbacks)
                const bool streak = !ok && cur.be == INT32_MIN;
                const int pend = streak ? min(pj, nblk) : pos + 1;
                if (!ok) {  // blocks [pos, pend) the reference way (the last block padded with -0.0)
#ifdef SGMM_STAMPS
                    n_slow += pend - pos;
#endif
                    const double2* vp = reinterpret_cast<const double2*>(sel + pos * kSumBlk);
                    double2 v[kSumBlk / 2];
#pragma unroll
                    for (int j = 0; j < kSumBlk / 2; ++j) v[j] = vp[j];
                    double s = ib ? from_binade(M, e) : S;
#pragma unroll
                    for (int j = 0; j < kSumBlk / 2; ++j) {
                        s += v[j].x;
                        s += v[j].y;
                    }
                    // the rest of a streak, 8 values per LDS round trip
                    const double2* __restrict__ sp = vp + kSumBlk / 2;
                    const double2* const se = vp + (pend - pos) * (kSumBlk / 2);
                    for (; sp < se; sp += 4) {
                        const double2 a = sp[0], b = sp[1], c = sp[2], d = sp[3];
                        s += a.x;
                        s += a.y;
                        s += b.x;
                        s += b.y;
                        s += c.x;
                        s += c.y;
                        s += d.x;
                        s += d.y;
                    }
                    S = s;
                    ib = binade_of(s, e, M);
                }
                // both successors' records were requested before the decision
                // (a streak ends at the run's end: its record is rj)
                const bool to_end = ok || streak;
                M = ok ? Mj : M;
                pos = ok ? pj : pend;
                // field by field: a whole-struct select was lowered to a scratch
                // round trip per step
                cur.mn = to_end ? rj.mn : rn.mn;
                cur.mx = to_end ? rj.mx : rn.mx;
                cur.dsum = to_end ? rj.dsum : rn.dsum;
                cur.be = to_end ? rj.be : rn.be;
                cur.rend = to_end ? rj.rend : rn.rend;
                if (pos >= nblk) break;
            }
            L.S = ib ? from_binade(M, e) : S;
        }
#ifdef SGMM_STAMPS
        if (threadIdx.x == 0 && blockIdx.x < 4096) { g_stamps[blockIdx.x][13] += n_iter; g_stamps[blockIdx.x][14] += n_slow; }
#endif
        if (lane == 0 && nblk == 0) L.S = S;
#ifndef SGMM_NO_WALK_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
    }
    __syncthreads();
    SGMM_STAMP(blockIdx.x, 10);
    return L.S;
}



// LDS bytes the tail needs (aliased onto the kernel's dynamic LDS)
static inline size_t step_lds_bytes(int threads, const StepArgs& sa) {
    return (size_t)threads * 2 * (sizeof(double) + sizeof(int)) +
           sizeof(float) * (size_t)(sa.n_mm + (sa.master_adv ? sa.n_adv : 0));
}


// Thread 0 stored the workgroup's record with store_record.  It drains the
// stores, takes an arrival ticket (agent-scope atomic); the workgroup that
// draws the last ticket reads every record with sc1 loads (ga_step_dev
// <HANDOFF = true>) -- MI355X_MICROARCH.md inter-workgroup visibility, row 1
// -- runs the GA step and resets the ticket for the next launch.  e = the
// episode whose record was stored (its population's ticket), n_total = the
// launch's episodes (one population when pop_eps == 0).
// The GA step of population k once all its records are stored (the last
// arriver's part of generation_tail; the fused frontier launch's cleanup runs
// it directly).
__device__ __forceinline__ void tail_run(const StepArgs& sa0, const double* fitness0, const int32_t* trades0, unsigned char* lds,
                         int k, int n_eps) {
    StepArgs sa = sa0;
    sa.st = sa0.st + k;
    sa.master_mm = sa0.master_mm + (int64_t)k * sa0.n_mm;
    if (sa0.master_adv) sa.master_adv = sa0.master_adv + (int64_t)k * sa0.n_adv;
    if (sa0.best_master) sa.best_master = sa0.best_master + (int64_t)k * sa0.n_mm;
    if (sa0.history) sa.history = sa0.history + (int64_t)k * sa0.hist_cap;
    const double* fitness = fitness0 + (int64_t)k * n_eps;
    const int32_t* trades = trades0 + (int64_t)k * n_eps;
    if (sa0.seeds) sa.seed = sa0.seeds[k];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: loads after the ticket
    SGMM_STAMP(blockIdx.x, 4);
#ifdef SGMM_STAMPS
    if (threadIdx.x == 0) g_stamps[4095][0] = g_stamps[blockIdx.x][4];
#endif
    const int nt = blockDim.x;
    double* sv = reinterpret_cast<double*>(lds);
    int* si = reinterpret_cast<int*>(sv + 2 * nt);
    float* lm = reinterpret_cast<float*>(si + 2 * nt);
    float* la = lm + sa.n_mm;
    const bool tell_only = sa.mode == 1;
    if (sa.mode == 3) {
        if (threadIdx.x < kWave)
            tell_wave<true, false>(sa.st, fitness, trades, sa.P, sa.master_mm, sa.master_adv, sa.n_mm, sa.n_adv,
                                   sa.seed, sa.history, sa.hist_cap);
    } else if (tell_only && nt == kWave && sa.n_mm <= 4 * kWave * kWaveChunks && sa.n_adv <= 4 * kWave * kWaveChunks)
        tell_wave<true>(sa.st, fitness, trades, sa.P, sa.master_mm, sa.master_adv, sa.n_mm, sa.n_adv, sa.seed,
                        sa.history, sa.hist_cap);
    else if (sa.P <= nt && sa.n_mm <= 16 * nt && sa.n_adv <= 16 * nt)
        ga_step_fused<true>(sa.st, fitness, trades, fitness + sa.P, trades + sa.P, sa.P, sa.master_mm,
                            sa.master_adv, sa.best_master, sa.n_mm, sa.n_adv, sa.seed, sa.history,
                            sa.hist_cap, sv, si, lm, la, tell_only);
    else
        ga_step_dev<true>(sa.st, fitness, trades, fitness + sa.P, trades + sa.P, sa.P, ShardView{0, 0},
                          sa.master_mm, sa.master_adv, sa.best_master, sa.n_mm, sa.n_adv, sa.seed,
                          sa.history, sa.hist_cap, nullptr, nullptr, 0, 0, sv, si, lm, la, tell_only);
    if (threadIdx.x == 0) sa.st->arrivals = 0;
    SGMM_STAMP(blockIdx.x, 5);
}

__device__ __forceinline__ void generation_tail(const StepArgs& sa0, const double* fitness0, const int32_t* trades0,
                                unsigned char* lds, int* s_last, int e, int n_total) {
    // this episode's population (one arrival ticket per population)
    const int n_eps = sa0.pop_eps > 0 ? sa0.pop_eps : n_total;
    const int k = sa0.pop_eps > 0 ? e / sa0.pop_eps : 0;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int prev = __hip_atomic_fetch_add(&sa0.st[k].arrivals, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        *s_last = prev == n_eps - 1;
    }
    __syncthreads();
    if (!*s_last) return;
    tail_run(sa0, fitness0, trades0, lds, k, n_eps);
}

// The validation launch's tail (StepArgs::mode 2): episode k holds the
// validation record (v, vtr: thread 0's values) of population k's post-tell
// master and runs its bookkeeping -- no other episode's record is needed.
__device__ __forceinline__ void validation_tail(const StepArgs& sa, double v, int32_t vtr, int* flag, int k) {
    __syncthreads();  // flag aliases LDS the caller has just read
    if (sa.mode == 4) {
        // the deferred tell: master <- ask(best) with the generation's sigma and
        // counter (the bookkeeping below decays sigma and advances gen)
        const sgmm_ga_state* st = sa.st + k;
        const uint32_t gen = (uint32_t)st->gen;
        const int best = st->best_idx, abest = st->adv_best_idx;
        const float smm = (float)st->sigma_mm, sadv = (float)st->sigma_adv;
        const uint64_t seed = sa.seeds ? sa.seeds[k] : sa.seed;
        regen_master_block(sa.master_mm + (int64_t)k * sa.n_mm, sa.n_mm, smm, seed, 0u, gen, best);
        if (sa.master_adv) regen_master_block(sa.master_adv + (int64_t)k * sa.n_adv, sa.n_adv, sadv, seed, 1u, gen, abest);
        __syncthreads();  // the new master before the checkpoint copy reads it
    }
    val_update_dev(sa.st + k, v, vtr, sa.master_mm + (int64_t)k * sa.n_mm,
                   sa.best_master ? sa.best_master + (int64_t)k * sa.n_mm : nullptr, sa.n_mm,
                   sa.history ? sa.history + (int64_t)k * sa.hist_cap : nullptr, sa.hist_cap, flag);
}

// ------------------------------------------------------------------ path scan (no adversary)
// Per episode (one workgroup, or one wave of the fused frontier launch):
//   1. wave 0: chunk start states from a wave-level scan of the chunk maps,
//      and the episode's trades: each chunk's count along the path from its
//      start state (8 bits per start state, written by the table);
//   2. every thread: the rewards of its 4 ticks from the path plane of their
//      chunk's start state (one coalesced row per chunk) -> LDS;
//   3. the rewards' sequential float64 sum, bit-exact (exact_sum_window).
// FR: the frontier kernel's chunks (frontier_len(T, nw) ticks, 64 per wave,
// records e * 256 + c, u32 trade counts, kinfo = merge tick | p0 << 29).
// TPB < NT: a TPB-thread workgroup with NT's window and block layout (TPB =
// 64, NT = 256: one wave -- the only one exact_sum_window<256> gives blocks
// to -- gathers 1024 values, so many more episodes run per CU).
template <int NT>
struct ScanShared {
    double* sel;          // [NT * kSumTpt] the window (the last block padded in place)
    SumLds<NT>* L;
    uint8_t* start;       // chunk start states
    uint32_t* kin;        // FR: the chunks' merge info
    int* red;             // trades, then the tail's "last arriver" flag
    unsigned char* tail;  // generation-tail scratch (aliases sel)
};

template <int NSM, int NT, bool FR, int TPB>
__device__ __forceinline__ void scan_episode(int e, int nw, const EpArrays& ep, const sgmm_env_params* __restrict__ params,
                                             int32_t inv_min, const uint64_t* __restrict__ cmaps,
                                             const uint64_t* __restrict__ ctr, const uint32_t* __restrict__ kinfo,
                                             const double* __restrict__ rew, double* __restrict__ fitness,
                                             int32_t* __restrict__ trades_out, const StepArgs& step, int n_total,
                                             const ScanShared<NT>& sh) {
    static_assert(TPB == NT || (TPB == kWave && NT == 4 * kWave), "TPB = NT or one wave with NT = 256");
    constexpr int kWin = NT * kSumTpt;
    double* sel = sh.sel;
    uint8_t* start = sh.start;
    uint32_t* kin = sh.kin;
    const int32_t T = ep.len[e];
    const int64_t so = ep.step_off[e];
    // FR: records laid out for nw (ep.ngrp) groups; the episode's own group
    // count is in its first record
    const int64_t cb = FR ? frontier_rec(e, nw, 0) : (int64_t)chunk_base(so, e);
    const int nwe = (FR && T > 0) ? (int)kinfo_groups(kinfo[cb]) : 1;
    const int CL = FR ? frontier_len(T, nwe) : kChunk;
    const int nch = (T + CL - 1) / CL;
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    SGMM_STAMP(e, 0);
    if (tid < kWave) {  // chunk start states, 64 chunks per round, carried across rounds
        uint32_t s = (uint32_t)(-inv_min);
        int tr = 0;
        for (int c0 = 0; c0 < nch; c0 += kWave) {
            const int c = c0 + lane;
            const uint64_t m = c < nch ? cmaps[cb + c] : kIdentityMap;
            const uint64_t k = (!FR && c < nch) ? ctr[cb + c] : 0;
            const uint64_t inc = wave_map_scan(m);
            uint64_t excl = shfl_up_u64(inc, 1);
            if (lane == 0) excl = kIdentityMap;
            const uint32_t st = map_get(excl, s);
            if (c < nch) start[c] = (uint8_t)st;
            if (FR) {
                if (c < nch) {
                    tr += (int)reinterpret_cast<const uint32_t*>(ctr)[(cb + c) * 8 + st];
                    kin[c] = kinfo[cb + c];
                }
            } else {
                tr += (int)((k >> (8 * st)) & 0xFFu);
            }
            s = map_get(readlane64(inc, kWave - 1), s);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) tr += __shfl_xor(tr, off, kWave);
        if (lane == 0) *sh.red = tr;
    }
    __syncthreads();
    SGMM_STAMP(e, 1);
#ifdef SGMM_STAMPS
    // per episode, summed over the windows: 11 gather cycles, 12 sum cycles,
    // 15 windows; 13 / 14 walk iterations / fallback blocks
    unsigned long long sw_a, sw_b, sw_g = 0, sw_s = 0, sw_n = 0;
    if (tid == 0 && e < 4096) g_stamps[e][13] = g_stamps[e][14] = g_stamps[e][6] = g_stamps[e][7] = 0;
#define SGMM_SW(var) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory")
#endif
    double S = 0.0;  // exact running sum (identical in every thread between windows)
    // a window's rewards: each thread's NT / TPB groups of kSumTpt ticks (4
    // ticks of one chunk, CL % kSumTpt == 0) gathered into registers; the next
    // window's loads are issued before this window's exact sum, so their
    // latency hides behind the sum's serial walk
    double r[NT / TPB][kSumTpt];
    auto gather = [&](int w0) {
        const int n = min(kWin, T - w0);
#pragma unroll
        for (int g = 0; g < NT / TPB; ++g) {
            const int i0 = (g * TPB + tid) * kSumTpt;
            if (i0 < n) {
                if (FR) {  // plane of the start state before the chunk's paths merge, plane p0 after
                    const int c = (w0 + i0) / CL, u = w0 + i0 - c * CL;
                    const uint32_t ki = kin[c];
                    const int kc = (int)(ki & kKinfoTick);
                    const int64_t pst = start[c], pp0 = ki >> 29;
                    const int64_t rb = frontier_base(so, e, nw) + (int64_t)(c / kFrontierLanes) * CL * kFrontierLanes +
                                       frontier_row(u, c % kFrontierLanes);
#pragma unroll
                    for (int j = 0; j < kSumTpt; ++j) {
                        const int jj = min(j, n - 1 - i0);
                        r[g][j] = rew[(u + jj >= kc ? pp0 : pst) * ep.rs + rb + (int64_t)jj * kFrontierLanes];
                    }
                } else {
                    const double* __restrict__ src = rew + (int64_t)start[(w0 + i0) / kChunk] * ep.rs + so + w0 + i0;
#pragma unroll
                    for (int j = 0; j < kSumTpt; ++j) r[g][j] = src[min(j, n - 1 - i0)];
                }
            }
        }
    };
    if (T > 0) gather(0);
    for (int w0 = 0; w0 < T; w0 += kWin) {
        const int n = min(kWin, T - w0);
#ifdef SGMM_STAMPS
        SGMM_SW(sw_a);
#endif
#pragma unroll
        for (int g = 0; g < NT / TPB; ++g) {
            const int i0 = (g * TPB + tid) * kSumTpt;
#pragma unroll
            for (int j = 0; j < kSumTpt; ++j)
                if (i0 + j < n) sel[i0 + j] = r[g][j];
        }
        __syncthreads();
        SGMM_STAMP(e, 2);
#ifdef SGMM_STAMPS
        SGMM_SW(sw_b);
        sw_g += sw_b - sw_a;
#endif
        if (w0 + kWin < T) gather(w0 + kWin);  // in flight during the sum
        S = exact_sum_window<NT>(sel, n, S, *sh.L, ep.seq_sum != 0);
#ifdef SGMM_STAMPS
        SGMM_SW(sw_a);
        sw_s += sw_a - sw_b;
        sw_n += 1;
#endif
    }
#ifdef SGMM_STAMPS
    if (tid == 0 && e < 4096) {
        g_stamps[e][11] = sw_g;
        g_stamps[e][12] = sw_s;
        g_stamps[e][15] = sw_n;
    }
#undef SGMM_SW
#endif
    SGMM_STAMP(e, 3);
    int tr = 0;  // thread 0's record (the tails read it there only)
    double total = S;
    if (tid == 0) {
        tr = *sh.red;
        if (tr == 0) total -= params[ep.param[e]].idle_penalty;  // drl_engine.py:64-65
        store_record(fitness, trades_out, e, total, tr);
    }
    if (step.st) {
        if (step.mode == 2 || step.mode == 4) validation_tail(step, total, tr, sh.red, e);
        else generation_tail(step, fitness, trades_out, sh.tail, sh.red, e, n_total);
    }
}

// one workgroup per episode (the table path, and the frontier path unfused)
template <int NSM, int NT, bool FR, int TPB = NT>
__global__ __launch_bounds__(TPB) void k_path_scan(
    EpArrays ep, const sgmm_env_params* __restrict__ params, int32_t inv_min,
    const uint64_t* __restrict__ cmaps, const uint64_t* __restrict__ ctr,
    const uint32_t* __restrict__ kinfo, const double* __restrict__ rew, double* __restrict__ fitness,
    int32_t* __restrict__ trades_out, StepArgs step) {
    extern __shared__ __align__(16) unsigned char lds[];
    __shared__ SumLds<NT> L;
    __shared__ uint8_t start_t[FR ? 1 : kMaxLen / kChunk];
    __shared__ int red_trades;
    const int e = blockIdx.x;
    // frontier chunks (64 per group): their start states and merge info follow
    // the window in the dynamic LDS (scan_lds_bytes)
    uint8_t* start = FR ? lds + NT * kSumTpt * sizeof(double) : start_t;
    uint32_t* kin = reinterpret_cast<uint32_t*>(lds + NT * kSumTpt * sizeof(double) + kFrontierLanes * ep.ngrp);
    const ScanShared<NT> sh{reinterpret_cast<double*>(lds), &L, start, kin, &red_trades, lds};
    scan_episode<NSM, NT, FR, TPB>(e, FR ? ep.ngrp : 1, ep, params, inv_min, cmaps, ctr, kinfo, rew, fitness, trades_out,
                                   step, (int)gridDim.x, sh);
}


// ------------------------------------------------------------------ path scan, W episodes per workgroup
// The frontier path scan for many episodes, the sums as sequential chains: wave w
// of the workgroup takes episode e0 + w through the scan's first two phases (chunk
// start states and trades; the rewards of its path, kLanesWin ticks per window,
// into LDS row w, padded with -0.0), and wave 0 adds the W windows, lane w episode
// e0 + w, one dependent v_add_f64 advancing all W chains.  The one-wave scan ran
// one chain per wave on all 64 lanes: with 2-3 scans per SIMD its float64 adds
// shared the vector pipe (trained config 3: ~20 cycles per tick and episode,
// against ~10 for a lone chain, tools/mb_trained_timeline.py SCAN=1).  x + -0.0 == x
// for every x, so the padding leaves each episode's sum its reference-order chain.
// The generation tail: the workgroup's W records, one arrival of W (the tell's
// argmax, StepArgs mode 3, when its last population record arrives).
// W and the window measured (profiles/r06_lanes/, scan of config 3 / of config 5's
// 1-of-8 shard): W = 16 57.8 / 40.5 us, 8 59.5 / 33.9, 4 55.5 / 31.1, 2 53.5 / 33.5;
// 1024-tick windows 56.5-59.6 / 33.8 (one episode per wave: 72.2 / 37.5)
#ifndef SGMM_LANES_W
#define SGMM_LANES_W 4
#endif
constexpr int kLanesW = SGMM_LANES_W;       // episodes per workgroup (lanes_w picks 2 or 4 per launch)
#ifndef SGMM_LANES_WIN
#define SGMM_LANES_WIN 512
#endif
constexpr int kLanesWin = SGMM_LANES_WIN;   // ticks per window
constexpr int kLanesPitch = kLanesWin + 2;  // doubles per LDS row (16-byte bank offset per row)
static size_t lanes_scan_lds(int ngrp, int w) {
    return (size_t)w * kLanesPitch * sizeof(double) + (size_t)w * kFrontierLanes * ngrp * (sizeof(uint32_t) + 1) + 64;
}
template <int NSM, int kLanesW>
__global__ __launch_bounds__(kWave * kLanesW) void k_path_scan_lanes(
    EpArrays ep, const sgmm_env_params* __restrict__ params, int32_t inv_min, const uint64_t* __restrict__ cmaps,
    const uint32_t* __restrict__ ctr32, const uint32_t* __restrict__ kinfo, const double* __restrict__ rew,
    double* __restrict__ fitness, int32_t* __restrict__ trades_out, StepArgs step, int32_t n) {
    extern __shared__ __align__(16) unsigned char lds[];
    const int nw = ep.ngrp;
    double* win = reinterpret_cast<double*>(lds);  // [kLanesW][kLanesPitch]
    uint32_t* kin_all = reinterpret_cast<uint32_t*>(win + kLanesW * kLanesPitch);
    uint8_t* start_all = reinterpret_cast<uint8_t*>(kin_all + kLanesW * kFrontierLanes * nw);
    __shared__ int32_t red_s[kLanesW];
    __shared__ int32_t len_s[kLanesW];
    const int w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & (kWave - 1));
    const int e0 = (int)blockIdx.x * kLanesW, e = e0 + w;
    constexpr int wc = 0;  // the chain wave (rotating it over the SIMDs measured no different)
    SGMM_STAMP(blockIdx.x, 0);
#ifdef SGMM_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_stamps[blockIdx.x][12] = 0;
#endif
    const bool has = e < n;
    const int32_t T = has ? ep.len[e] : 0;
    uint32_t* kin = kin_all + w * kFrontierLanes * nw;
    uint8_t* start = start_all + w * kFrontierLanes * nw;
    double* row = win + w * kLanesPitch;
    // 1. (wave w) chunk start states and the trades along the path
    const int64_t cb = frontier_rec(has ? e : 0, nw, 0);
    const int nwe = T > 0 ? (int)kinfo_groups(kinfo[cb]) : 1;
    const int CL = frontier_len(T, nwe);
    const int nch = T > 0 ? (T + CL - 1) / CL : 0;
    {
        uint32_t s = (uint32_t)(-inv_min);
        int tr = 0;
        for (int c0 = 0; c0 < nch; c0 += kWave) {
            const int c = c0 + lane;
            const uint64_t m = c < nch ? cmaps[cb + c] : kIdentityMap;
            const uint64_t inc = wave_map_scan(m);
            uint64_t excl = shfl_up_u64(inc, 1);
            if (lane == 0) excl = kIdentityMap;
            const uint32_t st = map_get(excl, s);
            if (c < nch) {
                start[c] = (uint8_t)st;
                kin[c] = kinfo[cb + c];
                tr += (int)ctr32[(cb + c) * 8 + st];
            }
            s = map_get(readlane64(inc, kWave - 1), s);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, kWave);
        if (lane == 0) {
            red_s[w] = tr;
            len_s[w] = T;
        }
    }
    __syncthreads();
    SGMM_STAMP(blockIdx.x, 1);
    int tmax = 0;
#pragma unroll
    for (int i = 0; i < kLanesW; ++i) tmax = max(tmax, len_s[i]);
    // 2. windows: every wave gathers its episode's next window while wave 0 adds
    const int64_t base = frontier_base(has ? ep.step_off[e] : 0, has ? e : 0, nw);
    constexpr int kG = kLanesWin / (4 * kWave);
    double r[kG][4];
    auto gather = [&](int w0) {
        const int cnt = min(kLanesWin, T - w0);  // <= 0 past the episode's end
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int i0 = (q * kWave + lane) * 4;
            if (i0 < cnt) {
                const int c = (w0 + i0) / CL, u = w0 + i0 - c * CL;
                const uint32_t ki = kin[c];
                const int kc = (int)(ki & kKinfoTick);
                const int64_t pst = start[c], pp0 = ki >> 29;
                const int64_t rb = base + (int64_t)(c / kFrontierLanes) * CL * kFrontierLanes +
                                   frontier_row(u, c % kFrontierLanes);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int jj = min(j, cnt - 1 - i0);
                    r[q][j] = rew[(u + jj >= kc ? pp0 : pst) * ep.rs + rb + (int64_t)jj * kFrontierLanes];
                }
            }
        }
    };
    gather(0);
    double S = 0.0;  // wave 0, lane v < kLanesW: episode e0 + v
    const double* mine = win + min(lane, kLanesW - 1) * kLanesPitch;
    for (int w0 = 0; w0 < tmax; w0 += kLanesWin) {
        const int cnt = T - w0;
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int i0 = (q * kWave + lane) * 4;
            double2 a, b;
            a.x = i0 < cnt ? r[q][0] : -0.0;
            a.y = i0 + 1 < cnt ? r[q][1] : -0.0;
            b.x = i0 + 2 < cnt ? r[q][2] : -0.0;
            b.y = i0 + 3 < cnt ? r[q][3] : -0.0;
            *reinterpret_cast<double2*>(row + i0) = a;
            *reinterpret_cast<double2*>(row + i0 + 2) = b;
        }
        __syncthreads();
#ifdef SGMM_STAMPS
        if (w0 == 0) SGMM_STAMP(blockIdx.x, 2);
        unsigned long long ch0;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ch0)::"memory");
#endif
        if (w0 + kLanesWin < T) gather(w0 + kLanesWin);
        if (w == wc) {
            // this window's length over the workgroup's episodes
            const int m = min(kLanesWin, tmax - w0);
            const double2* p = reinterpret_cast<const double2*>(mine);
            int i = 0;
            for (; i + 32 <= m; i += 32) {
                double2 v[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = p[i / 2 + j];
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    S += v[j].x;
                    S += v[j].y;
                }
            }
            for (; i < m; ++i) S += mine[i];
#ifdef SGMM_STAMPS
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            unsigned long long ch1;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ch1)::"memory");
            if (threadIdx.x == 0 && blockIdx.x < 4096) g_stamps[blockIdx.x][12] += ch1 - ch0;
#endif
        }
        __syncthreads();  // the windows are read before the next ones are written
    }
    SGMM_STAMP(blockIdx.x, 3);
    // 3. records (the chain wave, lane v: episode e0 + v) and the generation tail
    if (w == wc) {
        const int nv = min(kLanesW, n - e0);
        if (lane < nv) {
            const int ev = e0 + lane;
            const int32_t tr = red_s[lane];
            double total = S;
            if (tr == 0) total -= params[ep.param[ev]].idle_penalty;  // drl_engine.py:64-65
            store_record(fitness, trades_out, ev, total, tr);
        }
        if (step.st) {
            const int n_eps = step.pop_eps > 0 ? step.pop_eps : n;
            const int k = step.pop_eps > 0 ? e0 / step.pop_eps : 0;
            int last = 0;
            if (lane == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's record stores
                last = __hip_atomic_fetch_add(&step.st[k].arrivals, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                       n_eps - nv;
            }
            if (__shfl(last, 0, kWave)) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: loads after the ticket
                sgmm_ga_state* st = step.st + k;
                tell_wave<true, false>(st, fitness + (int64_t)k * n_eps, trades_out + (int64_t)k * n_eps, step.P,
                                       step.master_mm + (int64_t)k * step.n_mm,
                                       step.master_adv ? step.master_adv + (int64_t)k * step.n_adv : nullptr,
                                       step.n_mm, step.n_adv, step.seeds ? step.seeds[k] : step.seed,
                                       step.history ? step.history + (int64_t)k * step.hist_cap : nullptr,
                                       step.hist_cap);
                if (lane == 0) st->arrivals = 0;
            }
        }
    }
    SGMM_STAMP(blockIdx.x, 4);
}


// ------------------------------------------------------------------ ordered sum (standalone)
// init + x[0] + x[1] + ... in sequential float64 order, one workgroup.
__global__ __launch_bounds__(kScanThreads) void k_ordered_sum(const double* __restrict__ x, int64_t n,
                                                              double init, double* __restrict__ out) {
    __shared__ __align__(16) double sel[kScanWin];
    __shared__ SumLds<kScanThreads> L;
    double S = init;
    for (int64_t w0 = 0; w0 < n; w0 += kScanWin) {
        const int m = (int)min((int64_t)kScanWin, n - w0);
        for (int i = threadIdx.x; i < m; i += kScanThreads) sel[i] = x[w0 + i];
        __syncthreads();
        S = exact_sum_window<kScanThreads>(sel, m, S, L);
    }
    if (threadIdx.x == 0) *out = S;
}


// ------------------------------------------------------------------ path scan (adversary)
// 4 nsi-state machine (inventory x previous fill flags).  Per episode, one
// NT-thread workgroup, segment by segment (kSeg ticks = 128 pieces of 32), the
// state entering a segment carried over -- no bound on the episode length:
//   1. the segment's fill codes -> LDS (coalesced);
//   2. every (piece, start state) pair walks its piece over the LDS codes (8
//      per round trip): the piece's transducer, end state and trade count per
//      start state (all NT threads: 3 rounds of 32 steps at config 4, where
//      one serial walker per table wave cost the table ~25 us; 64-tick pieces
//      took 2 rounds of 64 steps, and twice as long in step 4);
//   3. the end maps chained by pointer jumping (log2(128) rounds over all
//      (piece, state) pairs) -> each piece's start state; trades = the sum of
//      every piece's count from its start state;
//   4. one thread per piece walks its 32 ticks from the start state and
//      records the state of every tick;
//   5. every thread gathers its ticks' rewards from the per-state planes
//      rew[state * rs + row] (independent loads: one latency per segment;
//      consecutive ticks in one state are consecutive addresses);
//   6. the exact sequential float64 sum (exact_sum_window).
// Dynamic LDS: [kSeg u64 codes / f64 rewards][kSeg states][2][128][ns] maps
// [128][ns] trade counts [128] starts.
constexpr int kArlSub = 32;                 // ticks per transducer piece (half a table chunk)
constexpr int kSegChunks = kSeg / kArlSub;  // pieces per segment
static size_t arl_scan_lds(int ns) { return (size_t)kSeg * 9 + (size_t)3 * kSegChunks * ns + kSegChunks; }
template <int NT>
__global__ __launch_bounds__(NT) void k_path_scan_arl(
    EpArrays ep, const sgmm_env_params* __restrict__ params, int32_t inv_min, int32_t nsi,
    const uint64_t* __restrict__ fills, const double* __restrict__ rew,
    double* __restrict__ fitness, int32_t* __restrict__ trades_out, StepArgs step) {
    extern __shared__ __align__(16) unsigned char lds[];
    uint64_t* fl = reinterpret_cast<uint64_t*>(lds);  // the segment's fill codes, then
    double* sel = reinterpret_cast<double*>(lds);     // its rewards (the codes are dead by then)
    uint8_t* stt = lds + kSeg * sizeof(double);       // [kSeg] the state at each tick
    const int ns = 4 * nsi;
    uint8_t* jm = stt + kSeg;                         // [2][segch][ns] jump maps (double-buffered)
    uint8_t* tr = jm + 2 * kSegChunks * ns;           // [segch][ns] trades from each start state
    uint8_t* start = tr + kSegChunks * ns;            // [segch]
    __shared__ SumLds<NT> L;
    __shared__ int red_trades;
    const int e = blockIdx.x;
    const int32_t T = ep.len[e];
    const int64_t so = ep.step_off[e];
    const uint64_t* __restrict__ F = fills + so;
    const int tid = threadIdx.x;
    if (tid == 0) red_trades = 0;
    SGMM_STAMP(e, 0);
    int carry = (-inv_min) << 2;  // the state entering the segment (episode start: inventory 0, no fills)
    int my_trades = 0;
    double total = 0.0;
    for (int seg0 = 0; seg0 < T; seg0 += kSeg) {
        const int segn = min(kSeg, T - seg0);
        const int segch = (segn + kArlSub - 1) / kArlSub;
        for (int i = tid; i < segn; i += NT) fl[i] = F[seg0 + i];
        __syncthreads();
        SGMM_STAMP(e, 1);
        // chunk k's transducer from start state s (padded ticks: none, the walk stops at the chunk's end)
        for (int i = tid; i < segch * ns; i += NT) {
            const int k = i / ns;
            int st = i - k * ns, cnt = 0;
            const int ta = k * kArlSub, tb = min(segn, ta + kArlSub);
            if (tb - ta == kArlSub) {  // a whole piece: no per-tick bound check
#pragma unroll 1
                for (int t8 = ta; t8 < tb; t8 += 8) {
                    uint64_t f[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) f[j] = fl[t8 + j];
#pragma unroll
                    for (int j = 0; j < 8; ++j) st = arl_step(st, f[j], cnt);
                }
            } else
            for (int t8 = ta; t8 < tb; t8 += 8) {
                uint64_t f[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = fl[t8 + j];  // < kSeg: in the buffer
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (t8 + j < tb) {
                        const int c = (int)(f[j] >> (2 * st)) & 3;
                        cnt += c != 0;
                        st = next_state_arl(st, c);
                    }
            }
            jm[i] = (uint8_t)st;
            tr[i] = (uint8_t)cnt;
        }
        __syncthreads();
        SGMM_STAMP(e, 6);
        // jm[k][s] = state after chunks k-2^r+1 .. k from state s at chunk k-2^r+1's start
        int cur = 0;
        for (int d = 1; d < segch; d <<= 1) {
            const uint8_t* a = jm + cur * segch * ns;
            uint8_t* b = jm + (cur ^ 1) * segch * ns;
            for (int i = tid; i < segch * ns; i += NT) {
                const int k = i / ns, st = i - k * ns;
                b[i] = k >= d ? a[k * ns + a[(k - d) * ns + st]] : a[i];
            }
            cur ^= 1;
            __syncthreads();
        }
        // start of chunk k = the inclusive prefix of chunks 0 .. k-1 applied to the carry
        const uint8_t* pre = jm + cur * segch * ns;
        for (int k = tid; k < segch; k += NT) {
            const int st = k == 0 ? carry : pre[(k - 1) * ns + carry];
            start[k] = (uint8_t)st;
            my_trades += tr[k * ns + st];
        }
        __syncthreads();
        SGMM_STAMP(e, 7);
        carry = pre[(segch - 1) * ns + carry];
        if (tid < segch) {  // piece tid's state path
            int st = start[tid];
            const int ta = tid * kArlSub, tb = min(segn, ta + kArlSub);
            if (tb - ta == kArlSub) {  // a whole piece: no per-tick bound check
                int unused = 0;
#pragma unroll 1
                for (int t8 = ta; t8 < tb; t8 += 8) {
                    uint64_t f[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) f[j] = fl[t8 + j];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        stt[t8 + j] = (uint8_t)st;
                        st = arl_step(st, f[j], unused);
                    }
                }
            } else
            for (int t8 = ta; t8 < tb; t8 += 8) {
                uint64_t f[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = fl[t8 + j];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (t8 + j < tb) {
                        stt[t8 + j] = (uint8_t)st;
                        st = next_state_arl(st, (int)(f[j] >> (2 * st)) & 3);
                    }
            }
        }
        __syncthreads();  // the codes are dead: sel takes their place
        SGMM_STAMP(e, 11);
        for (int i = tid; i < segn; i += NT) sel[i] = rew[(int64_t)stt[i] * ep.rs + so + seg0 + i];
        __syncthreads();
        SGMM_STAMP(e, 12);
        for (int k = 0; k < segn; k += 4 * NT)  // windows of 4 values per thread
            total = exact_sum_window<NT>(sel + k, min(4 * NT, segn - k), total, L, ep.seq_sum != 0);
    }
    int w = my_trades;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off, kWave);
    if ((tid & (kWave - 1)) == 0 && w) atomicAdd(&red_trades, w);
    __syncthreads();
    if (tid == 0) {
        const int tr_ = red_trades;
        if (tr_ == 0) total -= params[ep.param[e]].idle_penalty;
        store_record(fitness, trades_out, e, total, tr_);
    }
    SGMM_STAMP(e, 3);
    if (step.st) generation_tail(step, fitness, trades_out, lds, &red_trades, e, (int)gridDim.x);
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
    SGMM_REQUIRE(eps->max_len >= 0, "max_len=%d < 0", eps->max_len);
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

// Chunk groups per episode in the frontier kernel (one wave each).  A walk's
// time is set by its serial chain of ticks, not by its SIMD's load, so when the
// launch has fewer than two walks per SIMD the episodes are cut into 2-4
// groups of 64 chunks of proportionally fewer ticks;
// each extra group pays for tracking every start state of its chunks until
// their paths merge.  SGMM_PLAN_GROUPS = 1..16 forces the count (records and
// plane padding are laid out for the launch's count, frontier_rec / frontier_pad).
constexpr int kFrontierAutoWaves = 8;  // the default rule's cap
// SIMDs of the current device (cached per device id; 256 CUs if the query fails)
static int simd_count() {
    constexpr int kMaxDev = 64;
    static std::atomic<int> cache[kMaxDev];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    std::atomic<int>& c = cache[dev < kMaxDev ? dev : kMaxDev - 1];
    int n = c.load(std::memory_order_relaxed);
    if (n == 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        n = 4 * cus;
        c.store(n, std::memory_order_relaxed);
    }
    return n;
}
// The launch's chunk-group plan: g0 groups for the episodes at order positions
// [0, whole), gtail groups for the rest; gmax = the record / padding layout.
struct FrontierPlan {
    int32_t g0, gtail, whole, gmax;
    int64_t waves;  // walks (64-chunk groups)
    int32_t ls;     // waves per walk (lane split, k_policy_frontier<H, NSI, LS>)
};
static FrontierPlan frontier_plan(int32_t n) {
    FrontierPlan p{1, 1, std::max(n, 0), 1, std::max<int64_t>(n, 0), 1};
    const int ls_force = plan_value(SGMM_PLAN_LANE_SPLIT);  // tests / experiments: waves per walk
    if (ls_force == 2 || ls_force == 4) p.ls = ls_force;
    {
        const int g = plan_value(SGMM_PLAN_GROUPS);
        if (g >= 1 && g <= kFrontierMaxWaves) {
            p.g0 = p.gtail = p.gmax = g;
            p.waves = (int64_t)n * g;
            return p;
        }
    }
    if (n <= 0) return p;
    // two walks per SIMD (measured, config 5's 1-of-8 shard, 1024 episodes of
    // 3600 ticks: 317 / 274 / 313 / 336 us at 1 / 2 / 3 / 4 groups, round 4;
    // 270 / 272 / 331 us at 2 / 4 / 8 groups, round 5; splitting lanes instead,
    // 283-311 us, profiles/r05_small)
    const int64_t S = simd_count();
    p.g0 = p.gtail = p.gmax = (int32_t)std::max<int64_t>(1, std::min<int64_t>(kFrontierAutoWaves, 2 * S / n));
    // from half as many episodes as SIMDs down, two waves per walk (lane split):
    // four waves per SIMD without more chunk starts (the 1-of-16 shard, 512
    // episodes: frontier + scan 248.5 us at G = 4 with two waves per walk against
    // 255.9 us at G = 8 and 270.6 us at G = 4 with one, profiles/r05_small/ls_*, c5s16_fr4)
    if (n <= S / 2 && ls_force < 0) p.ls = 2;
    // Whole walks are dispatched one per SIMD per run of S waves, so n = a S + r
    // leaves r SIMDs with a walk more than the others, and the walks on those
    // SIMDs end last.  The r episodes at the end of the order are cut into
    // ~S / r groups instead: the last run of waves becomes ~S shorter walks,
    // one per SIMD (1536 = 1024 + 512 -> 1024 whole walks and 512 episodes in 2
    // groups; config 3's 2560 = 2 x 1024 + 512 -> 2048 + 512 in 2 groups took
    // the policy kernel from 547 to 525 us, before the four-walk rule below).
    // SGMM_PLAN_TAIL = 0 keeps every walk whole.
    const bool tail = plan_value(SGMM_PLAN_TAIL) != 0;
    const int64_t r = n % S;
    const int fourv = plan_value(SGMM_PLAN_FOUR);
    const bool four = fourv != 0;  // experiments: 0 = no four-walk rule, 2 = whole walks and quarters
    if (tail && fourv == 2 && p.g0 == 1 && 4 * n - 4 * S >= 3 * (S / 2) && n < 4 * S) {
        // experiment: four walks per SIMD as whole walks and quarters, (4n - 4S) / 3
        // whole (config 3: 2048 whole + 512 episodes in quarters)
        p.whole = (int32_t)((4 * n - 4 * S) / 3);
        p.gtail = p.gmax = 4;
    } else if (tail && four && p.g0 == 1 && 2 * n - 4 * S >= S / 2 && n < 4 * S) {
        // from 2.5 episodes per SIMD up to 4: four walks per SIMD, 2n - 4S whole
        // and the rest in halves, one whole and three half walks per SIMD (config
        // 3: 2560 = 1024 whole + 1536 in halves; 660.5-668.0 against 670.3-670.6 us
        // per generation for 2048 whole + 512 in halves, and 690-699 us for all in
        // halves, profiles/r05_ab/ab20_*, ab21_*)
        p.whole = (int32_t)(2 * n - 4 * S);
        p.gtail = p.gmax = 2;
    } else if (tail && p.g0 == 1 && n > S && r > 0) {
        const int64_t gt = std::max<int64_t>(1, std::min<int64_t>(kFrontierMaxWaves, (S + r / 2) / r));
        if (gt > 1) {
            p.whole = (int32_t)(n - r);
            p.gtail = p.gmax = (int32_t)gt;
        }
    }
    p.waves = (int64_t)p.whole * p.g0 + (int64_t)(n - p.whole) * p.gtail;
    return p;
}
// the record / plane-padding layout of a launch of n episodes
static int32_t frontier_groups(int32_t n) { return frontier_plan(n).gmax; }

// Spill deadline of a frontier launch (FrontierArgs::spill_budget, 10 ns units):
// SGMM_PLAN_SPILL microseconds after a walk's start, 0 = no spill.  A walk
// still running then stops once its chunks have <= kSpillTicks ticks left;
// k_frontier_spill runs the rest tick-parallel.
constexpr int kSpillDefault = 0;
static uint32_t spill_budget(const sgmm_episodes* eps, const FrontierPlan&) {
    int v = plan_value(SGMM_PLAN_SPILL);
    if (v < 0) v = kSpillDefault;
    if (v == 0 || eps->max_len <= 0) return 0;
    return (uint32_t)std::min<int64_t>((int64_t)v * 100, 0x7FFFFFFF);
}


// plane stride: every tick, plus (no adversary: the frontier kernel may run)
// the frontier layout's padding rows per episode, frontier_pad(G) with G the
// launch's chunk groups; the adversary planes are table rows only
static int64_t rew_stride(int64_t steps, int32_t n, bool arl) {
    const int64_t pad = arl ? 0 : frontier_pad(frontier_groups(n)) * n;
    return (steps + pad + 31) & ~int64_t(31);
}

static EpArrays ep_arrays(const sgmm_episodes* e, bool with_adv) {
    return EpArrays{e->genome, with_adv ? e->adv : nullptr, e->tick_off, e->len, e->step_off,
                    e->param, rew_stride(e->total_steps, e->n, with_adv), e->order, 1, 1, 1, e->n};
}

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Policy kernel selection, SGMM_PLAN_POLICY_PATH: default = the frontier
// kernel for many episodes, else the f32-MFMA table; 1 / 2 force either; 3
// forces the VALU table (one lane per (tick, state)), an independent
// cross-check in the tests.
static bool table_valu() { return plan_value(SGMM_PLAN_POLICY_PATH) == 3; }

}  // namespace sgmm

using namespace sgmm;

#ifdef SGMM_STAMPS
extern "C" int sgmm_debug_stamps(unsigned long long* host, int n_eps) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16 * n_eps);
}
extern "C" int sgmm_debug_tail(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tail), sizeof(unsigned long long) * 8);
}
extern "C" int sgmm_debug_thwid(unsigned int* host, int n_waves) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_thwid), sizeof(unsigned int) * 2 * n_waves);
}
extern "C" int sgmm_debug_tstamps(unsigned long long* host, int n_waves) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tstamps), sizeof(unsigned long long) * 8 * n_waves);
}
#endif

// Workspace layout (256-byte aligned sections), per batch of total_steps ticks:
//   no adversary: u64 cmaps[nc] | u64 ctr[nc] (nc = total_steps/64 + n + 1 chunk
//                 slots) | u32 kinfo[n * 64 G] | u32 wslots[n * 64] | u32 wspill[n * 64] | f64 path planes
//                 rew[n_states][rs] (rs = total_steps + frontier_pad(G) n,
//                 rounded up to 32; G = frontier_groups(n))
//   adversary:    u64 fills[total_steps] | f64 rew[n_states][rs] (rs =
//                 total_steps rounded up to 32)
//   (frontier kernel: cmaps / ctr hold u64 maps / u32[8] trade counts at the
//   records e * 64 G + c, kinfo the merge tick | p0 << 29 of each record; the
//   sections are sized for both the table and the frontier layout)
static size_t n_chunk_slots(int32_t n, int64_t steps) { return (size_t)steps / kChunk + (size_t)n + 1; }
static size_t n_frontier_slots(int32_t n) { return (size_t)n * kFrontierLanes * frontier_groups(n); }  // chunk records
static size_t ws_cmaps(int32_t n, int64_t steps) {
    return align256(std::max(n_chunk_slots(n, steps), n_frontier_slots(n)) * sizeof(uint64_t));
}
static size_t ws_ctr(int32_t n, int64_t steps) {
    return align256(std::max(n_chunk_slots(n, steps) * sizeof(uint64_t), n_frontier_slots(n) * 8 * sizeof(uint32_t)));
}
// u32 kinfo[n * 256]: per chunk record the merge tick | p0 << 29
static size_t ws_kinfo(int32_t n) { return align256(n_frontier_slots(n) * sizeof(uint32_t)); }
static size_t ws_fills(int64_t steps) { return align256((size_t)steps * sizeof(uint64_t)); }
// u32 wslots[n * 64]: the frontier launch's MLP slots per walk, [e * G + group] (G <= 16)
static size_t ws_wslots(int32_t n) { return align256((size_t)n * 64 * sizeof(uint32_t)); }
// u32 wspill[n * 64]: per frontier wave (<= 16 groups x 4 waves per episode) the
// tick offset at which it spilled, 0 if it did not
static size_t ws_wspill(int32_t n) { return align256((size_t)n * 64 * sizeof(uint32_t)); }
// the fused scan's per-episode arrival words and chain hand-offs (FrontierArgs::hstate, handoff)
static size_t ws_arrive(int32_t n) {
    return align256((size_t)n * sizeof(uint32_t)) + align256((size_t)n * sizeof(FusedHandoff));
}

// The workspace of a batch with n_inventory inventory values, with or
// without the adversary (then 4 * n_inventory states: inventory x previous
// fill flags).  The adversary flag is explicit: 4 * n_inventory <= 8 for one
// or two inventory values, so a state count alone cannot tell the layouts apart.
static size_t rollout_ws_bytes(int32_t n_episodes, int64_t total_steps, int32_t nsi, bool arl) {
    if (total_steps < 0 || nsi <= 0 || nsi > 8 || n_episodes < 0) return 0;
    if (arl)  // fill codes, per-state planes rew[state * rs + row]
        return ws_fills(total_steps) + (size_t)rew_stride(total_steps, n_episodes, true) * (size_t)(4 * nsi) * sizeof(double);
    return ws_cmaps(n_episodes, total_steps) + ws_ctr(n_episodes, total_steps) + ws_kinfo(n_episodes) +
           ws_wslots(n_episodes) + ws_wspill(n_episodes) + ws_arrive(n_episodes) +
           (size_t)rew_stride(total_steps, n_episodes, false) * (size_t)nsi * sizeof(double);
}

extern "C" size_t sgmm_rollout_workspace_bytes(int32_t n_episodes, int64_t total_steps, int32_t n_inventory,
                                               int32_t with_adversary) {
    return rollout_ws_bytes(n_episodes, total_steps, n_inventory, with_adversary != 0);
}

// ABI 3 form: n_states > 8 means the adversary layout with n_states / 4
// inventory values (use sgmm_rollout_workspace_bytes for an adversary batch
// with fewer than 3 inventory values)
extern "C" size_t sgmm_rollout_workspace_size(int32_t n_episodes, int64_t total_steps,
                                              int32_t n_states) {
    if (n_states > 8) return n_states % 4 ? 0 : rollout_ws_bytes(n_episodes, total_steps, n_states / 4, true);
    return rollout_ws_bytes(n_episodes, total_steps, n_states, false);
}

// Frontier kernel or table: the frontier kernel does ~1/3 of the table's
// matrix work but walks each episode serially (one wave per episode), so it
// needs many episodes to fill the chip; it is also the only path for episodes
// longer than kMaxLen.  SGMM_PLAN_POLICY_PATH forces either,
// SGMM_PLAN_MIN_EPS moves the threshold.  Measured crossover (one rank's
// shard of config 5, H = 32, 3600 ticks, per generation, profiles/r03_c5_shard*):
// 256 episodes table 235 / frontier 363 us, 512: 365 / 435, 1024: 633 / 525,
// 2048: 1078 / 572 -- the lines crossed near 700 episodes.  With 2-4 chunk
// groups per episode (round 4, training launch alone, profiles/r04_ab/r04m_*,
// r04n_*): 256 episodes table 167 / frontier 162 us, 512: 255-263 / 195-204.
constexpr int kFrontierMinEps = 512;
static bool use_frontier(bool arl, int hidden, const sgmm_episodes* eps) {
    if (arl || (hidden != 16 && hidden != 32)) return false;
    if (eps->max_len > kMaxLen) return true;
    const int path = plan_value(SGMM_PLAN_POLICY_PATH);
    if (path == 1) return true;
    if (path > 1) return false;
    const int m = plan_value(SGMM_PLAN_MIN_EPS);
    return eps->n >= (m > 0 ? m : kFrontierMinEps);
}

// The one-state-per-wave table for launches of at most kTableSpChunks chunks
// (SGMM_PLAN_TABLE_SP = 0 / 1 forces v3 / it, for A/B and the tests)
constexpr int64_t kTableSpChunks = 256;
static bool table_sp(int nch, int n_ep) {
    if (const int v = plan_value(SGMM_PLAN_TABLE_SP); v >= 0) return v != 0;
    return (int64_t)nch * n_ep <= kTableSpChunks;
}

// rj (may be null): a walk-order job to run as the state-parallel table's extra
// workgroup; *rj_done tells whether it did
template <int H>
static void launch_table_mfma(bool arl, int nsi, int max_len, int n_ep, hipStream_t s,
                              const sgmm_ticks& tk, const EpArrays& ep,
                              const sgmm_env_params* params, const GenomeSrc& src, int32_t inv_min,
                              uint64_t* ctr, uint64_t* cmaps, uint64_t* fills, double* rew,
                              const ReorderJob* rj = nullptr, bool* rj_done = nullptr) {
    const int nch = (max_len + kChunk - 1) / kChunk;
    const dim3 grid((nch + 3) / 4, n_ep), block(kWave * 4);  // 4 chunks (waves) per block
    if constexpr (H <= 32) {
        if (!arl && table_sp(nch, n_ep)) {
            const ReorderJob job = rj ? *rj : ReorderJob{nullptr, nullptr, 0, 0, 0, 1};
            const dim3 g2(nch, n_ep + (job.order ? 1 : 0)), b2(kWave * nsi);  // one workgroup per chunk, one wave per state
            if (nsi <= 5)
                SGMM_LAUNCH((k_policy_table_sp<H, 5>), g2, b2, 0, s, tk, ep, params, src, inv_min, nsi, ctr, cmaps,
                            rew, job);
            else
                SGMM_LAUNCH((k_policy_table_sp<H, 8>), g2, b2, 0, s, tk, ep, params, src, inv_min, nsi, ctr, cmaps,
                            rew, job);
            if (rj_done) *rj_done = job.order != nullptr;
            return;
        }
        if (!arl) {
            if (nsi <= 5)
                SGMM_LAUNCH((k_policy_table_v3<H, 5>), grid, block, 0, s, tk, ep, params, src, inv_min, nsi, ctr, cmaps,
                            rew);
            else
                SGMM_LAUNCH((k_policy_table_v3<H, 8>), grid, block, 0, s, tk, ep, params, src, inv_min, nsi, ctr, cmaps,
                            rew);
            return;
        }
    }
#define SGMM_TABLE_MFMA(NSI_, ARL_)                                                               \
    SGMM_LAUNCH((k_policy_table_mfma<H, NSI_, ARL_>), grid, block, 0, s, tk, ep, params,  \
                       src, inv_min, nsi, ctr, cmaps, fills, rew)
    if (arl) {
        if (nsi <= 5) SGMM_TABLE_MFMA(5, true);
        else SGMM_TABLE_MFMA(8, true);
    } else if (nsi <= 5) {
        SGMM_TABLE_MFMA(5, false);
    } else {
        SGMM_TABLE_MFMA(8, false);
    }
#undef SGMM_TABLE_MFMA
}

template <int H>
static void launch_table(bool arl, int nsi, dim3 grid, hipStream_t s, const sgmm_ticks& tk,
                         const EpArrays& ep, const sgmm_env_params* params, const GenomeSrc& src,
                         int32_t inv_min, uint64_t* ctr, uint64_t* cmaps, uint64_t* fills,
                         double* rew) {
    const dim3 block(kChunk * nsi);  // one wave per inventory state
#define SGMM_TABLE(NSM_, ARL_)                                                                  \
    SGMM_LAUNCH((k_policy_table<H, NSM_, ARL_>), grid, block, 0, s, tk, ep, params, src, \
                       inv_min, nsi, ctr, cmaps, fills, rew)
    if (arl) SGMM_TABLE(8, true);
    else if (nsi <= 5) SGMM_TABLE(5, false);
    else SGMM_TABLE(8, false);
#undef SGMM_TABLE
}

extern "C" int sgmm_ordered_sum(const double* values, int64_t n, double init, double* out,
                                void* stream) {
    clear_error();
    SGMM_REQUIRE(out && (values || n == 0) && n >= 0, "bad arguments");
    ProfScope prof("ordered_sum", as_stream(stream));
    SGMM_LAUNCH(k_ordered_sum, dim3(1), dim3(kScanThreads), 0, as_stream(stream), values, n,
                       init, out);
    SGMM_LAUNCHED();
    return SGMM_OK;
}

// path-scan workgroup size for n episodes (256 CUs): one 16-wave workgroup per
// CU while they fit, then 8-wave, then 4-wave workgroups
static int scan_threads(int64_t n) {
    {
        const int t = plan_value(SGMM_PLAN_SCAN_THREADS);
        if (t == 64 || t == 256 || t == 512 || t == 1024) return t;
    }
    // beyond 512 episodes one-wave workgroups: the exact-sum walk is serial,
    // so many episodes resident per CU beat fewer wider workgroups (config 3:
    // 193 -> 145 us per scan, tools/gpu_sc1.sh; config 5's 1-of-8 shard, 1024
    // episodes: 110 -> 74 us, profiles/r04_ab/r04k_*; round 6: 54.7 against 69.3 /
    // 94.6 us for 256 / 512 threads, profiles/r06_scanw/).  From 257 to 512
    // episodes 4-wave workgroups (1024-tick windows): config 5's 1-of-16 shard
    // (512 episodes) 49.8 against 61.7 us with 512 threads, 52.4 with one wave
    return n <= kScanAt1024 ? kScanThreads : (n <= kScanAt512 ? 256 : kWave);
}

template <int NSM, bool FR>
static void launch_path_scan(int nt, int64_t n, size_t lds, hipStream_t s, const EpArrays& ep,
                             const sgmm_env_params* params, int32_t inv_min, const uint64_t* cmaps,
                             const uint64_t* ctr, const uint32_t* kinfo, const double* rew, double* fitness,
                             int32_t* trades, const StepArgs& step) {
    if (nt == kWave)
        SGMM_LAUNCH((k_path_scan<NSM, 4 * kWave, FR, kWave>), dim3(n), dim3(nt), lds, s, ep, params, inv_min, cmaps,
                    ctr, kinfo, rew, fitness, trades, step);
    else if (nt == kScanThreads)
        SGMM_LAUNCH((k_path_scan<NSM, kScanThreads, FR, kScanThreads>), dim3(n), dim3(nt), lds, s, ep, params, inv_min,
                    cmaps, ctr, kinfo, rew, fitness, trades, step);
    else if (nt == 512)
        SGMM_LAUNCH((k_path_scan<NSM, 512, FR, 512>), dim3(n), dim3(nt), lds, s, ep, params, inv_min, cmaps, ctr, kinfo,
                    rew, fitness, trades, step);
    else
        SGMM_LAUNCH((k_path_scan<NSM, 256, FR, 256>), dim3(n), dim3(nt), lds, s, ep, params, inv_min, cmaps, ctr, kinfo,
                    rew, fitness, trades, step);
}

// Episode sums of a path scan: the plain sequential chain or the exact parallel
// binade method (exact_sum_window); both give the reference's bits.  Measured per
// shape, 20 generations each (profiles/r06_seq/): the sequential chain wins in the
// one-wave and 4-wave scans of many GA-trained episodes -- config 3 89.0 -> 75.7 us,
// config 5's 8 192 / 4 096 / 2 048 / 1 024 / 512 episodes 187.9 / 112.8 / 68.0 /
// 55.9 / 50.7 -> 177.4 / 102.4 / 61.8 / 40.1 / 32.9 us -- and in the validation
// scans (11.5-12.7 -> 10.3-11.4 us); the parallel method wins where one 16-wave
// workgroup sums each long episode (config 2 15.7 vs 26.8 us, config 6 18.5 vs
// 27.0) and in the adversary scan (config 4 39.9 vs 44.9, its 1-of-4 shard 32.5 vs
// 41.9).  SGMM_PLAN_SEQ_SUM forces either.
static bool scan_seq_sum(int nt, bool arl, bool validation) {
    if (const int v = plan_value(SGMM_PLAN_SEQ_SUM); v >= 0) return v != 0;
    if (validation) return true;
    return !arl && nt <= 256;
}

// The path scan fused into the frontier launch (k_policy_frontier<..., FS>): each
// walk sums its own episode (the sequential chain) while the launch's longer walks
// still run, and the last record of a population runs the tell -- no separate
// scan launch.  Where it applies: one wave per walk, <= kFusedMaxGroups groups, no
// spill, no tail or the tell's argmax (mode 3), not where the parallel sum is forced.
// The default takes it for launches of whole walks only (round 6, profiles/r06_fused/,
// per generation: config 5 1.344-1.360 -> 1.327-1.332 ms, its 1-of-2 shard
// 0.789-0.794 -> 0.759-0.761, 1-of-4 0.489-0.490 -> 0.469-0.471); with halves the
// chain hand-offs and the in-kernel sums on SIMDs shared with walks cost more than
// the separate scan (config 3 0.639-0.641 -> 0.646-0.650, the 1-of-8 shard 0.333 ->
// 0.372 ms).  SGMM_PLAN_FUSED_SCAN forces it off (0) or on where it applies (1).
static bool fused_scan_plan(const FrontierPlan& plan, uint32_t spill, const StepArgs& step, bool vt) {
    const int v = plan_value(SGMM_PLAN_FUSED_SCAN);
    if (v == 0 || vt || spill || plan.ls != 1 || plan.gmax > kFusedMaxGroups) return false;
    if (plan_value(SGMM_PLAN_SEQ_SUM) == 0) return false;  // the parallel method forced
    if (step.st && step.mode != 3) return false;
    return v == 1 || plan.gmax == 1;
}

// zero n words (the fused scan's arrival counters)
__global__ __launch_bounds__(1024) void k_zero_u32(uint32_t* __restrict__ p, int32_t n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) p[i] = 0u;
}

// The frontier path scan with kLanesW episodes per workgroup and their chains in
// the lanes of one wave (k_path_scan_lanes): where the one-wave scan would run the
// sequential chain, with no tail or the tell's argmax (mode 3) and populations of
// whole workgroups (config 3: scan 72 -> 55.5 us, 0.627-0.639 -> 0.605-0.612 ms
// per generation; config 5's 1-of-8 shard 37.5 -> 31.1 us).  SGMM_PLAN_LANES_SCAN forces it off (0) or on where it applies (1).
static bool lanes_scan(int nt, bool seq, const StepArgs& step, int32_t pop_eps) {
    const int v = plan_value(SGMM_PLAN_LANES_SCAN);
    if (v == 0 || !seq || (step.st && step.mode != 3)) return false;
    if (step.st && step.pop_eps > 0 && step.pop_eps % 4 != 0) return false;
    (void)pop_eps;
    return v > 0 || nt == kWave;
}
// episodes per lanes-scan workgroup: 2 from 2 048 episodes, 4 below (config 3 / 2 560
// episodes: scan 53.5 against 55.5 us; config 5's 1-of-8 shard / 1 024: 31.1 against
// 33.5 us with 2, profiles/r06_lanes/); SGMM_PLAN_LANES_SCAN = 2 or 4 forces it
static int lanes_w(int32_t n, const StepArgs& step) {
    const int v = plan_value(SGMM_PLAN_LANES_SCAN);
    if (v == 2 || v == 4) return v;
    (void)step;
    return n >= 2048 ? 2 : kLanesW;
}

// the launches the feedback applies to: a mixed whole / halves plan of one wave
// per walk, whole populations of equal-length episodes, the caller's writable
// walk order (sgmm_populations::walk_order)
static bool walk_reorder(const sgmm_episodes* eps, const FrontierPlan& plan, const GenomeSrc& src,
                         const int32_t* walk_order) {
    const int P = src.pop_eps;
    return walk_order && eps->order == walk_order && P > 0 && eps->n % P == 0 && eps->n / P >= 2 &&
           eps->n / P <= kReorderMaxPops &&
           plan.ls == 1 && plan.g0 == 1 && (plan.gtail == 2 || plan.gtail == 4) && plan.whole > 0 && plan.whole < eps->n &&
           eps->total_steps == (int64_t)eps->n * eps->max_len;
}

// table + path scan (+ the generation tail when step.st) for one batch
// walk_order: the caller's writable walk order (eps->order points at it) for the
// walk-order feedback; rj_out: a training launch with the feedback hands its job
// here instead of launching it; rj_in: a job to run inside (or before) this launch
static int rollout_impl(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                        const sgmm_env_params* params, const GenomeSrc& src, bool arl,
                        int32_t hidden, double* fitness, int32_t* trades, void* workspace,
                        size_t workspace_bytes, const StepArgs& step, hipStream_t s,
                        ReorderJob* rj_out = nullptr, const ReorderJob* rj_in = nullptr,
                        int32_t* walk_order = nullptr) {
    SGMM_REQUIRE(fitness && trades, "null fitness/trades output");
    if (eps->n == 0) return SGMM_OK;
    const int32_t nsi = eps->inv_max - eps->inv_min + 1;
    const int32_t ns = arl ? 4 * nsi : nsi;
    const size_t need = rollout_ws_bytes(eps->n, eps->total_steps, nsi, arl);
    if (!workspace || workspace_bytes < need) {
        set_error("workspace %zu bytes < required %zu", workspace_bytes, need);
        return SGMM_ERR_WORKSPACE;
    }
    char* w = reinterpret_cast<char*>(workspace);
    uint64_t* ctr = nullptr;
    uint64_t* cmaps = nullptr;
    uint64_t* fills = nullptr;
    uint32_t* kinfo = nullptr;
    uint32_t* wslots = nullptr;
    uint32_t* wspill = nullptr;
    uint32_t* arrive = nullptr;
    double* rew;
    if (arl) {
        fills = reinterpret_cast<uint64_t*>(w);
        rew = reinterpret_cast<double*>(w + ws_fills(eps->total_steps));
    } else {
        const size_t a = ws_cmaps(eps->n, eps->total_steps), b = ws_ctr(eps->n, eps->total_steps);
        cmaps = reinterpret_cast<uint64_t*>(w);
        ctr = reinterpret_cast<uint64_t*>(w + a);
        kinfo = reinterpret_cast<uint32_t*>(w + a + b);
        wslots = reinterpret_cast<uint32_t*>(w + a + b + ws_kinfo(eps->n));
        const size_t c = a + b + ws_kinfo(eps->n) + ws_wslots(eps->n);
        wspill = reinterpret_cast<uint32_t*>(w + c);
        arrive = reinterpret_cast<uint32_t*>(w + c + ws_wspill(eps->n));
        rew = reinterpret_cast<double*>(w + c + ws_wspill(eps->n) + ws_arrive(eps->n));
    }
    EpArrays ep = ep_arrays(eps, arl);
    const ReorderJob* rj_fold = nullptr;
    bool rj_done = false;
    const bool fr = use_frontier(arl, hidden, eps);
    const FrontierPlan plan = frontier_plan(eps->n);
    if (fr) {
        ep.ngrp = plan.gmax;
        ep.g0 = plan.g0;
        ep.gtail = plan.gtail;
        ep.whole = plan.whole;
    }
    const bool vt = step.st && (step.mode == 2 || step.mode == 4);  // the validation launches (profiled separately)
    SGMM_REQUIRE(fr || arl || eps->max_len <= kMaxLen,
                 "max_len=%d > %d needs the frontier kernel (hidden 16 or 32) or the adversary path", eps->max_len,
                 kMaxLen);
    SGMM_REQUIRE(!fr || eps->max_len <= kFrontierMaxLen, "max_len=%d > %lld ticks per episode",
                 eps->max_len, (long long)kFrontierMaxLen);
    if (rj_in && rj_in->order) {
        // a walk-order job rides along in this launch's state-parallel table when it takes
        // that path and its workspace use ends below the job's slot counts; otherwise it
        // runs first, before this launch can touch the workspace
        const int nch = (eps->max_len + kChunk - 1) / kChunk;
        const bool fold = !fr && !arl && eps->max_len > 0 && (hidden == 16 || hidden == 32) && !table_valu() &&
                          table_sp(nch, eps->n) &&
                          reinterpret_cast<const char*>(rj_in->wslots) >= w + rollout_ws_bytes(eps->n, eps->total_steps, nsi, arl);
        if (fold) {
            rj_fold = rj_in;
        } else {
            SGMM_LAUNCH(k_walk_reorder, dim3(1), dim3(kScanThreads), 0, s, *rj_in);
            SGMM_LAUNCHED();
            rj_done = true;
        }
    }
    const uint32_t spill = fr ? spill_budget(eps, plan) : 0u;
    const bool fused = fr && eps->max_len > 0 && fused_scan_plan(plan, spill, step, vt);
    if (fr && eps->max_len > 0) {
        FrontierArgs fa{*ticks, ep, params, src, eps->inv_min, nsi, cmaps, reinterpret_cast<uint32_t*>(ctr),
                        kinfo, rew, wslots, wspill, spill};
        if (fused) {
            fa.fitness = fitness;
            fa.trades = trades;
            fa.hstate = arrive;
            fa.handoff = reinterpret_cast<FusedHandoff*>(reinterpret_cast<char*>(arrive) + align256((size_t)eps->n * sizeof(uint32_t)));
            fa.n_eps = eps->n;
            fa.step = step;
            // the arrival words start at zero (the wave that ends an episode's chain
            // resets its word; a workspace is not zeroed before its first use).  A kernel,
            // not hipMemsetAsync: replayed after other launches, a captured memset
            // node left stale values here (tools/diag_fused2.py, round 6)
            if (plan.gmax > 1)
                SGMM_LAUNCH(k_zero_u32, dim3((eps->n + 1023) / 1024), dim3(1024), 0, s, arrive, eps->n);
        }
        ProfScope prof(vt ? "val_policy_frontier" : "policy_frontier", s);
        if (int rc = launch_policy_frontier(hidden, nsi, (unsigned)plan.waves, plan.ls, s, fa)) return rc;
        if (fa.spill_budget) {
            ProfScope prof2(vt ? "val_frontier_spill" : "frontier_spill", s);
            if (int rc = launch_frontier_spill(hidden, nsi, (unsigned)plan.waves, plan.ls, s, fa)) return rc;
        }
    } else if (eps->max_len > 0) {
        dim3 grid((eps->max_len + kChunk - 1) / kChunk, eps->n);
        ProfScope prof(vt ? "val_policy_table" : "policy_table", s);
        const bool valu = table_valu();
        if (rj_fold) {  // the walk-order job rides along in the state-parallel table
            if (hidden == 16)
                launch_table_mfma<16>(arl, nsi, eps->max_len, eps->n, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew, rj_fold, &rj_done);
            else
                launch_table_mfma<32>(arl, nsi, eps->max_len, eps->n, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew, rj_fold, &rj_done);
        } else switch (hidden) {
            case 8: launch_table<8>(arl, nsi, grid, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew); break;
            case 16:
                if (valu) launch_table<16>(arl, nsi, grid, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew);
                else launch_table_mfma<16>(arl, nsi, eps->max_len, eps->n, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew);
                break;
            case 32:
                if (valu) launch_table<32>(arl, nsi, grid, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew);
                else launch_table_mfma<32>(arl, nsi, eps->max_len, eps->n, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew);
                break;
            default:
                if (valu) launch_table<64>(arl, nsi, grid, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew);
                else launch_table_mfma<64>(arl, nsi, eps->max_len, eps->n, s, *ticks, ep, params, src, eps->inv_min, ctr, cmaps, fills, rew);
                break;
        }
        SGMM_LAUNCHED();
    }
    if (fused) {
        // the frontier launch summed every episode and ran the tail
    } else if (ProfScope prof(vt ? "val_path_scan" : "path_scan", s); arl) {
        // 16-wave workgroups while one per CU fits (a 4096-tick segment is one
        // exact-sum window), 4-wave ones beyond
        const int nt = eps->n <= kScanArlAt1024 ? kScanThreads : kScanBlock;
        ep.seq_sum = scan_seq_sum(nt, true, vt) ? 1 : 0;
        size_t lds = arl_scan_lds(ns);
        if (step.st) lds = std::max(lds, step_lds_bytes(nt, step));
        if (nt == kScanThreads)
            SGMM_LAUNCH(k_path_scan_arl<kScanThreads>, dim3(eps->n), dim3(nt), lds, s, ep, params, eps->inv_min,
                        nsi, fills, rew, fitness, trades, step);
        else
            SGMM_LAUNCH(k_path_scan_arl<kScanBlock>, dim3(eps->n), dim3(nt), lds, s, ep, params, eps->inv_min,
                        nsi, fills, rew, fitness, trades, step);
    } else {
        // the workgroup shrinks as episodes grow: few episodes get a 16-wave
        // workgroup each (4096-tick windows, the phases spread over the CU);
        // many get 8- or 4-wave ones (2048- / 1024-tick windows), several
        // resident per CU, so the serial walks of different episodes overlap
        // instead of idling the CU (A/B on MI355X: P=64 / 256 / 1024 / 4096)
        const int nt = scan_threads(eps->n);
        ep.seq_sum = scan_seq_sum(nt, false, vt) ? 1 : 0;
        if (fr && lanes_scan(nt, ep.seq_sum != 0, step, src.pop_eps)) {
            const int lw = lanes_w(eps->n, step);
            const size_t lds = lanes_scan_lds(ep.ngrp, lw);
            const dim3 grid((eps->n + lw - 1) / lw), block(kWave * lw);
#define SGMM_LANES_LAUNCH(N_, W_)                                                                                 \
    SGMM_LAUNCH((k_path_scan_lanes<N_, W_>), grid, block, lds, s, ep, params, eps->inv_min, cmaps,                \
                reinterpret_cast<const uint32_t*>(ctr), kinfo, rew, fitness, trades, step, eps->n)
            if (nsi <= 5) {
                if (lw == 2) SGMM_LANES_LAUNCH(5, 2);
                else SGMM_LANES_LAUNCH(5, 4);
            } else {
                if (lw == 2) SGMM_LANES_LAUNCH(8, 2);
                else SGMM_LANES_LAUNCH(8, 4);
            }
#undef SGMM_LANES_LAUNCH
        } else if (size_t lds = (size_t)(nt == kWave ? 4 * kWave : nt) * kSumTpt * sizeof(double) +  // the window
                                (fr ? (size_t)5 * kFrontierLanes * ep.ngrp : 0);  // chunk start states + merge info
                   fr) {
            if (step.st) lds = std::max(lds, step_lds_bytes(nt, step));
            if (nsi <= 5)
                launch_path_scan<5, true>(nt, eps->n, lds, s, ep, params, eps->inv_min, cmaps, ctr, kinfo, rew,
                                          fitness, trades, step);
            else
                launch_path_scan<8, true>(nt, eps->n, lds, s, ep, params, eps->inv_min, cmaps, ctr, kinfo, rew,
                                          fitness, trades, step);
        } else if (nsi <= 5) {
            if (step.st) lds = std::max(lds, step_lds_bytes(nt, step));
            launch_path_scan<5, false>(nt, eps->n, lds, s, ep, params, eps->inv_min, cmaps, ctr, kinfo, rew,
                                       fitness, trades, step);
        } else {
            if (step.st) lds = std::max(lds, step_lds_bytes(nt, step));
            launch_path_scan<8, false>(nt, eps->n, lds, s, ep, params, eps->inv_min, cmaps, ctr, kinfo, rew,
                                       fitness, trades, step);
        }
    }
    SGMM_LAUNCHED();
    if (fr && step.st && step.mode == 3 && walk_reorder(eps, plan, src, walk_order)) {
        ReorderJob job{wslots, walk_order, eps->n, plan.whole, plan.gtail, src.pop_eps};
        job.len = eps->max_len;  // equal-length episodes (walk_reorder)
        if (const int w = plan_value(SGMM_PLAN_REORDER_WEIGHTS); w > 0 && (w >> 8) > 0 && (w & 255) > 0) {
            job.w_whole = (uint32_t)(w >> 8) & 63u;
            job.w_split = (uint32_t)w & 63u;
        }
        if (rj_out) {
            *rj_out = job;
        } else {
            SGMM_LAUNCH(k_walk_reorder, dim3(1), dim3(kScanThreads), 0, s, job);
            SGMM_LAUNCHED();
        }
    }
    if (rj_in && rj_in->order && !rj_done) {  // (not reached: a job that cannot ride along ran first)
        set_error("walk-order job neither folded nor launched");
        return SGMM_ERR_ARG;
    }
    return SGMM_OK;
}

extern "C" int sgmm_rollout_fitness(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                                    const sgmm_env_params* params, const float* mm_genomes,
                                    int64_t mm_stride, int32_t hidden, const float* adv_genomes,
                                    int64_t adv_stride, double* fitness, int32_t* trades,
                                    void* workspace, size_t workspace_bytes, void* stream) {
    clear_error();
    if (int rc = check_episodes(ticks, eps, params, mm_genomes, hidden)) return rc;
    SGMM_REQUIRE(mm_stride >= (int64_t)hidden * hidden + 7 * hidden + 2, "mm_stride too small");
    const bool arl = adv_genomes != nullptr;
    SGMM_REQUIRE(!arl || adv_stride >= kAdvParams, "adv_stride < 74");
    const GenomeSrc src{mm_genomes, mm_stride, adv_genomes, adv_stride, nullptr, nullptr, nullptr, 0, 0};
    return rollout_impl(ticks, eps, params, src, arl, hidden, fitness, trades, workspace,
                        workspace_bytes, StepArgs{}, as_stream(stream));
}

extern "C" int sgmm_rollout_fitness_asked(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                                          const sgmm_env_params* params,
                                          const sgmm_asked_population* pop, int32_t hidden,
                                          double* fitness, int32_t* trades, void* workspace,
                                          size_t workspace_bytes, void* stream) {
    clear_error();
    SGMM_REQUIRE(pop && pop->state && pop->master_mm, "null asked population");
    if (int rc = check_episodes(ticks, eps, params, pop->master_mm, hidden)) return rc;
    SGMM_REQUIRE(pop->i0 >= 0, "negative i0");
    const bool arl = pop->master_adv != nullptr;
    const GenomeSrc src{nullptr, 0, nullptr, 0, pop->state, pop->master_mm, pop->master_adv, pop->seed, pop->i0};
    return rollout_impl(ticks, eps, params, src, arl, hidden, fitness, trades, workspace,
                        workspace_bytes, StepArgs{}, as_stream(stream));
}

extern "C" int sgmm_generation(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                               const sgmm_env_params* params, sgmm_ga_state* state, float* master_mm,
                               float* master_adv, float* best_master, int32_t hidden, uint64_t seed,
                               int32_t P, double* fitness, int32_t* trades, sgmm_ga_history* history,
                               int32_t history_cap, void* workspace, size_t workspace_bytes,
                               void* stream) {
    clear_error();
    SGMM_REQUIRE(state && master_mm, "null state / master");
    if (int rc = check_episodes(ticks, eps, params, master_mm, hidden)) return rc;
    SGMM_REQUIRE(P > 0 && eps->n == 2 * P, "episodes must be P training + P validation episodes");
    const int64_t n_mm = (int64_t)hidden * hidden + 7 * hidden + 2;
    SGMM_REQUIRE(n_mm <= kMaxStepParams, "genome too large for the fused GA step");
    const bool arl = master_adv != nullptr;
    const GenomeSrc src{nullptr, 0, nullptr, 0, state, master_mm, master_adv, seed, 0};
    StepArgs step{state, master_mm, master_adv, best_master, n_mm, arl ? 1250 : 0, seed, history,
                  history_cap, P};
    return rollout_impl(ticks, eps, params, src, arl, hidden, fitness, trades, workspace,
                        workspace_bytes, step, as_stream(stream));
}

static int check_pops(const sgmm_populations* pops) {
    SGMM_REQUIRE(pops, "null populations");
    SGMM_REQUIRE(pops->n_pop > 0 && pops->P > 0, "n_pop=%d P=%d must be > 0", pops->n_pop, pops->P);
    SGMM_REQUIRE(supported_hidden(pops->hidden), "hidden=%d unsupported (8,16,32,64)", pops->hidden);
    SGMM_REQUIRE(pops->states && pops->masters_mm && pops->seeds, "null states / masters / seeds");
    SGMM_REQUIRE(pops->history_cap >= 0 && (pops->history || pops->history_cap == 0), "history");
    return SGMM_OK;
}

extern "C" int sgmm_generation_multi(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                                     const sgmm_env_params* params, const sgmm_populations* pops,
                                     double* fitness, int32_t* trades, void* workspace,
                                     size_t workspace_bytes, void* stream) {
    clear_error();
    if (int rc = check_pops(pops)) return rc;
    const int32_t H = pops->hidden, K = pops->n_pop, P = pops->P;
    if (int rc = check_episodes(ticks, eps, params, pops->masters_mm, H)) return rc;
    SGMM_REQUIRE((int64_t)eps->n == 2LL * K * P,
                 "episodes must be n_pop x (P training + P validation) = %lld, got %d",
                 2LL * K * P, eps->n);
    const int64_t n_mm = (int64_t)H * H + 7 * H + 2;
    SGMM_REQUIRE(n_mm <= kMaxStepParams, "genome too large for the fused GA step");
    const bool arl = pops->masters_adv != nullptr;
    const int64_t n_adv = arl ? kAdvGenome : 0;
    GenomeSrc src{nullptr, 0, nullptr, 0, pops->states, pops->masters_mm, pops->masters_adv, 0, 0};
    src.pop_eps = 2 * P;
    src.seeds = pops->seeds;
    src.mm_pstride = n_mm;
    src.adv_pstride = n_adv;
    StepArgs step{pops->states, pops->masters_mm, pops->masters_adv, pops->best_masters, n_mm, n_adv, 0,
                  pops->history, pops->history_cap, P, 2 * P, pops->seeds};
    return rollout_impl(ticks, eps, params, src, arl, H, fitness, trades, workspace, workspace_bytes, step,
                        as_stream(stream));
}

// Validation of every population's post-tell master (drl_engine.py:129-160):
// val_eps episode k runs masters_mm row val_eps->genome[k] (= k) with no
// adversary; the scan's workgroup k then runs population k's validation
// bookkeeping (validation_tail).  The policy kernel is the table (K episodes).
// deferred: the training launch's tail ran the tell's argmax only (StepArgs
// mode 3); episode k rolls out population k's best individual from the
// pre-tell master and the scan's workgroup k writes the new master (mode 4)
static int validate_impl(const sgmm_ticks* ticks, const sgmm_episodes* val_eps, const sgmm_env_params* params,
                         const sgmm_populations* pops, double* val_fitness, int32_t* val_trades, void* workspace,
                         size_t workspace_bytes, hipStream_t s, bool deferred = false,
                         const ReorderJob* rj = nullptr) {
    const int32_t H = pops->hidden, K = pops->n_pop;
    if (int rc = check_episodes(ticks, val_eps, params, pops->masters_mm, H)) return rc;
    SGMM_REQUIRE(val_eps->n == K, "validation episodes must be one per population (%d), got %d", K, val_eps->n);
    const int64_t n_mm = (int64_t)H * H + 7 * H + 2;
    const bool arl = pops->masters_adv != nullptr;
    GenomeSrc src{pops->masters_mm, n_mm, nullptr, 0, nullptr, nullptr, nullptr, 0, 0};
    if (deferred) {
        src = GenomeSrc{nullptr, 0, nullptr, 0, pops->states, pops->masters_mm, nullptr, 0, 0};
        src.pop_eps = 1;
        src.seeds = pops->seeds;
        src.mm_pstride = n_mm;
        src.use_best = 1;
    }
    StepArgs step{pops->states, pops->masters_mm, (deferred && arl) ? pops->masters_adv : nullptr, pops->best_masters,
                  n_mm, (deferred && arl) ? (int64_t)kAdvGenome : 0, 0, pops->history, pops->history_cap, 1, 1,
                  pops->seeds, deferred ? 4 : 2};
    return rollout_impl(ticks, val_eps, params, src, false, H, val_fitness, val_trades, workspace, workspace_bytes,
                        step, s, nullptr, rj);
}

extern "C" int sgmm_validate_multi(const sgmm_ticks* ticks, const sgmm_episodes* val_eps,
                                   const sgmm_env_params* params, const sgmm_populations* pops,
                                   double* val_fitness, int32_t* val_trades, void* workspace,
                                   size_t workspace_bytes, void* stream) {
    clear_error();
    if (int rc = check_pops(pops)) return rc;
    return validate_impl(ticks, val_eps, params, pops, val_fitness, val_trades, workspace, workspace_bytes,
                         as_stream(stream));
}

extern "C" int sgmm_generation_multi_best(const sgmm_ticks* ticks, const sgmm_episodes* train_eps,
                                          const sgmm_episodes* val_eps, const sgmm_env_params* params,
                                          const sgmm_populations* pops, double* fitness, int32_t* trades,
                                          double* val_fitness, int32_t* val_trades, void* workspace,
                                          size_t workspace_bytes, void* stream) {
    clear_error();
    if (int rc = check_pops(pops)) return rc;
    const int32_t H = pops->hidden, K = pops->n_pop, P = pops->P;
    if (int rc = check_episodes(ticks, train_eps, params, pops->masters_mm, H)) return rc;
    SGMM_REQUIRE((int64_t)train_eps->n == (int64_t)K * P, "training episodes must be n_pop x P = %lld, got %d",
                 (int64_t)K * P, train_eps->n);
    SGMM_REQUIRE(val_eps && val_eps->n == K, "validation episodes must be one per population");
    SGMM_REQUIRE(val_fitness && val_trades, "null validation outputs");
    const int64_t n_mm = (int64_t)H * H + 7 * H + 2;
    SGMM_REQUIRE(n_mm <= kMaxStepParams, "genome too large for the fused GA step");
    const bool arl = pops->masters_adv != nullptr;
    const int64_t n_adv = arl ? kAdvGenome : 0;
    GenomeSrc src{nullptr, 0, nullptr, 0, pops->states, pops->masters_mm, pops->masters_adv, 0, 0};
    src.pop_eps = P;
    src.seeds = pops->seeds;
    src.mm_pstride = n_mm;
    src.adv_pstride = n_adv;
    StepArgs step{pops->states, pops->masters_mm, pops->masters_adv, pops->best_masters, n_mm, n_adv, 0,
                  pops->history, pops->history_cap, P, P, pops->seeds, 3};
    // the validation batch is checked before anything is enqueued
    if (int rc = check_episodes(ticks, val_eps, params, pops->masters_mm, H)) return rc;
    {
        const int32_t vnsi = val_eps->inv_max - val_eps->inv_min + 1;
        const size_t vneed = rollout_ws_bytes(val_eps->n, val_eps->total_steps, vnsi, false);
        if (val_eps->n > 0 && (!workspace || workspace_bytes < vneed)) {
            set_error("workspace %zu bytes < required %zu (validation batch)", workspace_bytes, vneed);
            return SGMM_ERR_WORKSPACE;
        }
    }
    hipStream_t s = as_stream(stream);
    ReorderJob job{nullptr, nullptr, 0, 0, 0, 1};
    // the training launch walks the caller's writable walk order when given
    // (the feedback rewrites it); train_eps itself is only read
    sgmm_episodes tr = *train_eps;
    if (pops->walk_order) tr.order = pops->walk_order;
    if (int rc = rollout_impl(ticks, &tr, params, src, arl, H, fitness, trades, workspace, workspace_bytes,
                              step, s, &job, nullptr, pops->walk_order))
        return rc;
    return validate_impl(ticks, val_eps, params, pops, val_fitness, val_trades, workspace, workspace_bytes, s, true,
                         &job);
}

extern "C" int sgmm_rollout_fitness_asked_multi(const sgmm_ticks* ticks, const sgmm_episodes* eps,
                                                const sgmm_env_params* params,
                                                const sgmm_populations* pops, int32_t i0,
                                                int32_t n_eps_pop, double* fitness, int32_t* trades,
                                                void* workspace, size_t workspace_bytes,
                                                void* stream) {
    clear_error();
    if (int rc = check_pops(pops)) return rc;
    const int32_t H = pops->hidden, K = pops->n_pop;
    if (int rc = check_episodes(ticks, eps, params, pops->masters_mm, H)) return rc;
    SGMM_REQUIRE(i0 >= 0 && n_eps_pop > 0 && (int64_t)eps->n == (int64_t)K * n_eps_pop,
                 "episodes must be n_pop x n_eps_pop (i0=%d, n_eps_pop=%d, n=%d)", i0, n_eps_pop, eps->n);
    const bool arl = pops->masters_adv != nullptr;
    GenomeSrc src{nullptr, 0, nullptr, 0, pops->states, pops->masters_mm, pops->masters_adv, 0, i0};
    src.pop_eps = n_eps_pop;
    src.seeds = pops->seeds;
    src.mm_pstride = (int64_t)H * H + 7 * H + 2;
    src.adv_pstride = arl ? kAdvGenome : 0;
    return rollout_impl(ticks, eps, params, src, arl, H, fitness, trades, workspace, workspace_bytes,
                        StepArgs{}, as_stream(stream));
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
    ProfScope prof("rollout_direct", s);
    switch (hidden) {
        case 8: SGMM_LAUNCH(k_rollout_direct<8>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
        case 16: SGMM_LAUNCH(k_rollout_direct<16>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
        case 32: SGMM_LAUNCH(k_rollout_direct<32>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
        default: SGMM_LAUNCH(k_rollout_direct<64>, dim3(eps->n), dim3(kWave), 0, s, *ticks, ep, params, mm_genomes, mm_stride, adv_genomes, adv_stride, eps->inv_min, nsi, o); break;
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
    ProfScope prof("policy_forward", s);
    switch (hidden) {
        case 8: SGMM_LAUNCH(k_policy_forward<8>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
        case 16: SGMM_LAUNCH(k_policy_forward<16>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
        case 32: SGMM_LAUNCH(k_policy_forward<32>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
        default: SGMM_LAUNCH(k_policy_forward<64>, grid, blk, 0, s, genomes, genome_stride, genome_idx, states, out, n); break;
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
    ProfScope prof("adversary_forward", as_stream(stream));
    SGMM_LAUNCH(k_adversary_forward, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
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
    ProfScope prof("env_step", as_stream(stream));
    SGMM_LAUNCH(k_env_step, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), params, param_idx, inventory, cash, action, adv_action,
                       mid_next, best_ask, best_bid, buy_max, sell_min, reward, pnl_reward,
                       inventory_reward, fee_paid, fill_buy, fill_sell, n);
    SGMM_LAUNCHED();
    return SGMM_OK;
}
