// sgmm_frontier.hip -- the frontier kernel (policy walk over occupied states).
//
// Reference semantics: evaluate_individual (Env/drl_engine.py:9-67) over a GA
// population -- per tick the TradingPolicy forward (models/model.py:5-26) and
// FTPEnv.step (Env/market_env.py:22-67) -- for the inventory states a chunk's
// paths occupy; the path scan (sgmm_rollout.hip) sums the rewards.
#include <cstddef>
#include <cstdlib>
#include <cstring>

#include "sgmm_rollout.h"

namespace sgmm {

#ifdef SGMM_STAMPS
// diagnostic build only: per-wave timeline / phase stamps of the frontier kernel
constexpr int kStampWaves = 1 << 16;
__device__ unsigned long long g_tstamps[kStampWaves][8];
__device__ unsigned int g_thwid[kStampWaves][2];  // HW_ID, XCC_ID of each wave
#endif

// ------------------------------------------------------------------ fused path scan
// k_policy_frontier<..., FS = true>: the walks sum their own episode while the
// launch's longer walks still run -- the path scan's frontier path (sgmm_rollout.hip,
// scan_episode<..., FR = true>) for one wave and one chunk group at a time: the
// group's chunk start states from its composed chunk maps and the state the
// episode's path enters it in, the trades along that path, then the rewards of the
// path added in windows of kFusedWin ticks as the plain sequential float64 chain
// (the reference's order, drl_engine.py:53-54), carried over from the previous
// group.  An episode walked whole is summed by its walk.  Of an episode walked in
// two groups (the launch plan's halves), group 0 sums its own chunks at once (its
// path enters at inventory 0) and hands the chain on -- sum, state, trades, 16
// bytes -- and group 1 continues over its own chunks: each wave reads only what it
// wrote itself.  Only when group 1 finishes before group 0 has handed the chain on
// does it hand its records and plane rows over instead (re-stored write-through), for
// group 0 to continue with.  The
// chain's last wave adds the idle penalty (drl_engine.py:64-65), stores the record,
// and the last record of a population runs the generation tail (tell_wave, the
// argmax of StepArgs mode 3; mode 1's master regeneration would take the walk
// loop's registers).
struct FusedChain {
    double S;     // the running sum
    uint32_t st;  // the state the path enters the next chunk in (0 .. nsi - 1)
    int32_t tr;   // trades so far
};
// global loads of handed-over bytes: write-through (sc1) both ways
// (MI355X_MICROARCH.md, inter-workgroup visibility, row 1)
// (a wave's own bytes too: its stores drained first, one code path for both)
template <class T>
__device__ __forceinline__ T fused_ld(const T* p) {
    typedef __attribute__((address_space(1))) const T gT;
    return __hip_atomic_load((gT*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void fused_st(T* p, T v) {
    typedef __attribute__((address_space(1))) T gT;
    __hip_atomic_store((gT*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the chain over chunk group g of episode e (CL ticks per chunk, nch chunks);
// win / kin / start: LDS (a 512-tick window, the group's 64 merge infos and start states)
__device__ __forceinline__ FusedChain fused_group(const FrontierArgs& args, int e, int g, int CL, int nch,
                                                  FusedChain cs, double* win, uint32_t* kin, uint8_t* start) {
    const EpArrays& ep = args.ep;
    const int lane = (int)threadIdx.x;
    const int32_t T = ep.len[e];
    const int c0 = g * kFrontierLanes, c1 = min(nch, c0 + kFrontierLanes);
    const int64_t cb = frontier_rec(e, ep.ngrp, 0);
    {
        const int c = c0 + lane;
        const uint64_t m = c < c1 ? fused_ld(args.cmaps + cb + c) : kIdentityMap;
        const uint64_t inc = wave_map_scan(m);
        uint64_t excl = shfl_up_u64(inc, 1);
        if (lane == 0) excl = kIdentityMap;
        const uint32_t st = map_get(excl, cs.st);
        int tr = 0;
        if (c < c1) {
            start[lane] = (uint8_t)st;
            kin[lane] = fused_ld(args.kinfo + cb + c);
            tr = (int)fused_ld(args.ctr32 + (cb + c) * 8 + st);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tr += __shfl_xor(tr, o, kWave);
        cs.tr += tr;
        cs.st = map_get(readlane64(inc, kWave - 1), cs.st);
    }
    __syncthreads();  // start / kin before the gathers read them
    const double* __restrict__ rew = args.rew;
    const int64_t rs = ep.rs;
    const int64_t base = frontier_base(ep.step_off[e], e, ep.ngrp) + (int64_t)g * CL * kFrontierLanes;
    const int t0 = c0 * CL, t1 = min(T, c1 * CL);
    // a window: each lane's two groups of 4 ticks (one chunk each, CL % 4 == 0),
    // from the plane of the chunk's start state before its paths merge and plane p0
    // after; the next window's loads are in flight during this window's sum
    constexpr int kG = kFusedWin / (4 * kWave);
    double r[kG][4];
    auto gather = [&](int w0) {
        const int n = min(kFusedWin, t1 - w0);
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int i0 = (q * kWave + lane) * 4;
            if (i0 < n) {
                const int cl = (w0 - t0 + i0) / CL, u = w0 - t0 + i0 - cl * CL;  // chunk within the group
                const uint32_t ki = kin[cl];
                const int kc = (int)(ki & kKinfoTick);
                const int64_t pst = start[cl], pp0 = ki >> 29;
                const int64_t rb = base + frontier_row(u, cl);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int jj = min(j, n - 1 - i0);
                    r[q][j] = fused_ld(rew + (u + jj >= kc ? pp0 : pst) * rs + rb + (int64_t)jj * kFrontierLanes);
                }
            }
        }
    };
    double S = cs.S;
    if (t0 < t1) gather(t0);
    for (int w0 = t0; w0 < t1; w0 += kFusedWin) {
        const int n = min(kFusedWin, t1 - w0);
#pragma unroll
        for (int q = 0; q < kG; ++q) {
            const int i0 = (q * kWave + lane) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (i0 + j < n) win[i0 + j] = r[q][j];
        }
        __syncthreads();
        if (w0 + kFusedWin < t1) gather(w0 + kFusedWin);
        // lane 0 adds the window in order from LDS, 32 values per round trip
        // (exact_sum_window's sequential chain; on one lane rather than all 64 the
        // walks sharing the SIMD lose less of the vector pipe: config 5's launch
        // 1 270-1 285 -> 1 250-1 256 us, profiles/r06_fused/NOTES.md)
        if (lane == 0) {
        const double2* p = reinterpret_cast<const double2*>(win);
        int i = 0;
        const int nc = n & ~31;
        for (; i < nc; i += 32) {
            double2 v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = p[i / 2 + j];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                S += v[j].x;
                S += v[j].y;
            }
        }
        for (; i < n; ++i) S += win[i];
        }
        S = __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(S), 0));
        __syncthreads();  // the window is read before the next one is written
    }
    cs.S = S;
    return cs;
}

// group 1 finishing before group 0: its records and plane rows re-stored
// write-through, for group 0 to read with sc1 loads (the rows it wrote: every
// tracked start's plane before the chunk's merge tick, plane p0 from it)
__device__ __forceinline__ void fused_ship(const FrontierArgs& args, int e, int CL, int nch) {
    const EpArrays& ep = args.ep;
    const int lane = (int)threadIdx.x;
    const int32_t T = ep.len[e];
    const int c = kFrontierLanes + lane;  // group 1's chunk of this lane
    if (c >= nch) return;
    const int64_t ci = frontier_rec(e, ep.ngrp, c);
    fused_st(args.cmaps + ci, args.cmaps[ci]);
    const uint32_t ki = args.kinfo[ci];
    fused_st(args.kinfo + ci, ki);
#pragma unroll
    for (int s = 0; s < 8; ++s) fused_st(args.ctr32 + ci * 8 + s, args.ctr32[ci * 8 + s]);
    const int kc = min((int)(ki & kKinfoTick), CL);
    const uint32_t p0 = ki >> 29;
    const int ntl = min(CL, T - c * CL);
    double* rb = args.rew + frontier_base(ep.step_off[e], e, ep.ngrp) + (int64_t)CL * kFrontierLanes;
    const int64_t rs = ep.rs;
    // (group 1's chunks track every start state)
    for (int u = 0; u < ntl; ++u) {
        double* row = rb + frontier_row(u, lane);
        if (u < kc) {
            for (int s = 0; s < args.nsi; ++s) fused_st(row + s * rs, row[s * rs]);
        } else {
            fused_st(row + p0 * rs, row[p0 * rs]);
        }
    }
}

// the episode's record and the generation tail (sgmm_rollout.hip generation_tail /
// tail_run, mode 3)
__device__ __forceinline__ void fused_finish(const FrontierArgs& args, int e, FusedChain cs) {
    const EpArrays& ep = args.ep;
    const int lane = (int)threadIdx.x;
    double total = cs.S;
    if (lane == 0) {
        if (cs.tr == 0) total -= args.params[ep.param[e]].idle_penalty;  // drl_engine.py:64-65
        store_record(args.fitness, args.trades, e, total, cs.tr);
    }
    const StepArgs& sa = args.step;
    if (!sa.st) return;
    const int n_eps = sa.pop_eps > 0 ? sa.pop_eps : args.n_eps;
    const int k = sa.pop_eps > 0 ? e / sa.pop_eps : 0;
    int last = 0;
    if (lane == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(&sa.st[k].arrivals, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_eps - 1;
    }
    if (!__shfl(last, 0, kWave)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: loads after the ticket
    sgmm_ga_state* st = sa.st + k;
    float* mm = sa.master_mm + (int64_t)k * sa.n_mm;
    float* ma = sa.master_adv ? sa.master_adv + (int64_t)k * sa.n_adv : nullptr;
    sgmm_ga_history* hist = sa.history ? sa.history + (int64_t)k * sa.hist_cap : nullptr;
    const uint64_t seed = sa.seeds ? sa.seeds[k] : sa.seed;
    const double* fit = args.fitness + (int64_t)k * n_eps;
    const int32_t* trd = args.trades + (int64_t)k * n_eps;
    tell_wave<true, false>(st, fit, trd, sa.P, mm, ma, sa.n_mm, sa.n_adv, seed, hist, sa.hist_cap);
    if (lane == 0) st->arrivals = 0;
}

// after the walk of group cg (ng groups with chunks, at most 2): sum what this wave
// can, hand the chain on or take it over (FrontierArgs::handoff / hstate)
// (CL, nch: the walk's chunk length and the episode's chunks -- not read from group
// 0's first record, which group 1 may reach before group 0 has written it)
__device__ __forceinline__ void fused_scan(const FrontierArgs& args, int e, int cg, int CL, int nch, double* win,
                                           uint32_t* kin, uint8_t* start) {
    const int32_t T = args.ep.len[e];
    FusedChain cs{0.0, (uint32_t)(-args.inv_min), 0};  // inventory 0
    if (T <= 0) {
        fused_finish(args, e, cs);
        return;
    }
    const int ng = (nch + kFrontierLanes - 1) / kFrontierLanes;
    FusedHandoff* ho = args.handoff + e;
    uint32_t* hs = args.hstate + e;
    int g = 0, go = 0;
    if (ng > 1 && cg == 1) {  // group 1: continue group 0's chain, or hand its own bytes over
        if (threadIdx.x == 0) go = __hip_atomic_load(hs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u;
        if (!__shfl(go, 0, kWave)) {
            fused_ship(args, e, CL, nch);
            if (threadIdx.x == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                go = __hip_atomic_fetch_add(hs, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u;
            }
            if (!__shfl(go, 0, kWave)) return;  // group 0 continues
        }
        const double S0 = fused_ld(&ho->S);
        const uint32_t w = fused_ld(&ho->st_tr);
        cs = FusedChain{S0, w & 0xFFu, (int32_t)(w >> 8)};
        g = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's records and rows, before its sc1 loads
    for (;;) {  // group g, then (group 0 of two, group 1 handed over) group 1
        cs = fused_group(args, e, g, CL, nch, cs, win, kin, start);
        if (g + 1 >= ng) break;
        // group 0 of two: hand the chain on; continue only if group 1 has handed its bytes over
        go = 0;
        if (threadIdx.x == 0) {
            fused_st(&ho->S, cs.S);
            fused_st(&ho->st_tr, cs.st | ((uint32_t)cs.tr << 8));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            go = __hip_atomic_fetch_add(hs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2u;
        }
        if (!__shfl(go, 0, kWave)) return;  // group 1 continues
        g = 1;
    }
    if (ng > 1 && threadIdx.x == 0) fused_st(hs, 0u);  // zero for the next launch
    fused_finish(args, e, cs);
}

// ------------------------------------------------------------------ frontier kernel
// The table evaluates the policy for every inventory state of every tick,
// because a chunk's start state is unknown until the scan.  But the paths
// from the different start states merge within a few ticks (fills move the
// inventory by +-1 against the caps): on the bench data a chunk's paths are at
// 1.2 distinct states per tick on average, not 5.  So here one wave walks a
// whole episode, lane = one chunk of CL = frontier_len(T) consecutive ticks
// (at most 64 chunks), and at each tick evaluates only the states its paths
// are currently in (the "frontier"):
//   per tick: slot k = the k-th frontier state of every lane; the layer-2
//   MFMAs run per 16-lane tile only while one of its lanes has a k-th state
//   (samples = the 64 lanes' chunks at the same tick offset); layer 3, the
//   FPT step and the frontier update run per lane.
// Per chunk it writes what the scan needs: the chunk map (byte s = end state of
// the path from start state s), the trade count along each path (u32), the
// path rewards (plane s, row = tick) -- and once every tracked path has merged
// (tick offset kc) only plane p0 (the lowest start state), so the planes cost
// ~1.3 rows per tick instead of one per state.  Chunk 0 starts at inventory 0;
// the other chunks track every state in [inv_min, inv_max].  Arithmetic per
// (tick, state) is the table's (same MFMA chains, same fp64 step), so every
// output bit is the table's.
//
// Wave b walks a chunk group of the episode at an order position (longest
// episodes first; frontier_wave maps b by the launch plan).  (Round 3's walks
// with tick hand-offs and the launch with the path scans fused in measured no
// faster: tools/experiments/round3_opt_in_paths.patch; round 5's helper waves
// and tile offers neither: tools/experiments/round5_tile_offers.patch.  Round 4's
// kernel, three waves per SIMD, is in the round-4 commits.)
//
// Each slot's MLP is laid out for the SIMD's pipes
// (tools/mb/mb_xwave3.hip: one wave's vector ops do not overlap its own MFMAs,
// but another wave's float ops run beside them at full rate):
//   - layer 1 on the matrix core: per 16-column tile q and neuron half hf one
//     v_mfma_f32_16x16x4_f32 with A = W1 rows in the order that makes D's
//     registers layer 2's B operand (D row 4g + r = neuron 16 hf + 4r + g, the
//     B operand of k-step 4 hf + r), B = the column's inputs (s1, s2, inv/2, 0)
//     read from a per-column LDS row, C = b1: the MFMA's k-ordered fused chain
//     b1 + w0 s1 + w1 s2 + w2 x2 is the canonical one (the trailing + 0 * 0
//     only turns -0 into +0, which relu maps to +0 either way) -- this replaces
//     the 3 fmas per (neuron, column) of the vector layer 1;
//   - layer 2 as one block of MFMAs (no vector work interleaved);
//   - relu and the transpose through LDS one 16-neuron half at a time (5 KB
//     instead of 9 KB), layer 3 as the two canonical output chains;
//   - a lane whose paths have merged keeps one trade count and stores its
//     slot-0 reward straight from the register.
// <= 128 VGPRs and <= 10 KB of LDS (H = 32, 5 states): four walks per SIMD.
// LS: waves per 64-chunk group (lane split).  With LS > 1 each wave walks
// 64 / LS of the group's chunks (lanes past them idle): the same chunks, the
// same chunk starts, LS times the waves -- for launches with fewer walks than
// the SIMDs hold.
// SP: the spill variant (FrontierArgs::wspill / spill_budget); without it the
// walk loop compiles exactly as before (its registers sit at the 128-VGPR edge)
template <int H, int NSI, int LS, bool SP, bool FS = false>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4))) void k_policy_frontier(FrontierArgs args) {
    static_assert(!FS || (LS == 1 && !SP), "the fused scan: one wave per walk, no spill");
    static_assert(H % 16 == 0 && H <= 32, "frontier kernel: H = 16 or 32");
    using L = GenomeLayout<H>;
    constexpr int NT = H / 16, KS = H / 4;
    constexpr int HP = 20;  // LDS row pitch (floats) of one transposed 16-neuron half
    constexpr int kHb = kWave * HP * 4;
    // `big`: the staged genome, then the transpose rows (also the columns'
    // layer-1 inputs)
    constexpr int kBig = L::N * 4 > kHb ? L::N * 4 : kHb;
    __shared__ __attribute__((aligned(16))) unsigned char big[kBig];
    __shared__ __attribute__((aligned(16))) float w3i[2 * H + 2];  // (W3[0][j], W3[1][j]) pairs, then b3
    __shared__ __attribute__((aligned(16))) float c1s[NT][4][4];   // layer-1 C: [hf][g][r] = b1[16 hf + 4r + g]
    __shared__ __attribute__((aligned(16))) float b2s[H];
    __shared__ __attribute__((aligned(8))) float sig[kWave][2];    // the tick's signals of each chunk
    __shared__ double px[5][kWave];  // the tick's prices of each chunk (for the extra slots' FPT steps)
    // the tick's extra (chunk, state) pairs: lane << 3 | state, then the
    // successor (bits 9-11) and the fill (bit 12) written back by the column
    __shared__ uint16_t pl[kWave * (NSI - 1)];
    __shared__ uint32_t nslot_s;  // MLP slots run (FrontierArgs::wslots; in LDS: the walk loop has no register to spare)
    // spill bookkeeping in LDS (no register is spare in the walk loop): this wave's
    // id, the first tick offset it may stop at, its slot budget
    __shared__ uint32_t wid_s, tmin_s, t0_s, spk_s;
    // FS: the kernarg pointer, for the scan after the walk (no SGPR is spare through
    // the walk loop to keep it, nor the scan's arguments, live)
    // FS: the scan's arguments (FrontierArgs from ep to src and from inv_min on),
    // copied from the kernarg segment at the start -- the kernarg memory is not
    // read again at the end of the walk
    constexpr int kFa0 = (int)(offsetof(FrontierArgs, ep) / 4), kFa1 = (int)(offsetof(FrontierArgs, src) / 4);
    constexpr int kFa2 = (int)(offsetof(FrontierArgs, inv_min) / 4), kFa3 = (int)(sizeof(FrontierArgs) / 4);
    constexpr int kFaWords = (kFa1 - kFa0) + (kFa3 - kFa2);
    static_assert(offsetof(FrontierArgs, src) % 4 == 0 && offsetof(FrontierArgs, inv_min) % 4 == 0 &&
                  sizeof(FrontierArgs) % 4 == 0, "whole words");
    __shared__ uint32_t fa_s[FS ? kFaWords : 1];
    __shared__ uint32_t ep_s, cl_s, nch_s, cg_s;  // FS: the episode, its chunk length and chunks, this walk's group
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (FS) {
        typedef __attribute__((address_space(4))) const uint32_t ka_u32;
        const ka_u32* ka = (const ka_u32*)__builtin_amdgcn_kernarg_segment_ptr();
        for (int i = (int)threadIdx.x; i < kFaWords; i += kWave)
            fa_s[i] = ka[i < kFa1 - kFa0 ? kFa0 + i : kFa2 + i - (kFa1 - kFa0)];
    }
#endif
    if (SP && threadIdx.x == 0) {  // every wave of the launch writes its spill entry, spilled or not
        wid_s = blockIdx.x;
        spk_s = 0;
        t0_s = (uint32_t)wall_clock64();  // 100 MHz
        args.wspill[blockIdx.x] = 0u;
    }

    const sgmm_ticks& tk = args.tk;
    const EpArrays& ep = args.ep;
    const sgmm_env_params* __restrict__ params = args.params;
    const GenomeSrc& src = args.src;
    const int32_t inv_min = args.inv_min, nsi = args.nsi;
    uint64_t* __restrict__ cmaps = args.cmaps;
    uint32_t* __restrict__ ctr32 = args.ctr32;
    uint32_t* __restrict__ kinfo = args.kinfo;
    double* __restrict__ rew = args.rew;
    static_assert(LS == 1 || LS == 2 || LS == 4, "lane split 1, 2 or 4");
    constexpr int NL = kFrontierLanes / LS;  // chunks (lanes) this wave walks
    int pos, cg, nw;  // order position, chunk group, the episode's groups
    frontier_wave(ep, (int)blockIdx.x / LS, pos, cg, nw);
    const int off = ((int)blockIdx.x % LS) * NL;  // this wave's first chunk within the group
    const int e = ep.order ? ep.order[pos] : pos;
    const int32_t T = ep.len[e];
    if (T <= 0) {  // block-uniform; FS: group 0 stores the empty episode's record after the walk below
        if (!FS || cg != 0) return;
        if (threadIdx.x == 0) {
            ep_s = (uint32_t)e;
            cl_s = 4u;
            nch_s = 0u;
            cg_s = 0u;
        }
    }
    if (T > 0) {  // the walk
        const int CL = frontier_len(T, nw);
        const int nch = (T + CL - 1) / CL;
        if (cg * kFrontierLanes + off >= nch) return;  // a group (part) past the episode's last chunk (no arrival)
        if (FS && threadIdx.x == 0) {  // for the scan after the walk (kept in LDS, as kap_s)
            ep_s = (uint32_t)e;
            cl_s = (uint32_t)CL;
            nch_s = (uint32_t)nch;
            cg_s = (uint32_t)cg;
        }
        const int lane = (int)threadIdx.x, grp = lane >> 4, col = lane & 15;
        const bool lane_ok = LS == 1 || lane < NL;
        const int c = cg * kFrontierLanes + off + lane;    // this lane's chunk
        const int64_t tb = ep.tick_off[e], so = ep.step_off[e];
        const int64_t rbase = frontier_base(so, e, ep.ngrp) + (int64_t)cg * CL * kFrontierLanes;  // the group's rows
        const int t0 = c * CL;
        const int ntl = lane_ok ? max(0, min(T, t0 + CL) - t0) : 0;  // its ticks (0 past the last chunk)

        float* gsm = reinterpret_cast<float*>(big);
        stage_genomes(src, e, ep.genome[e], -1, L::N, gsm, nullptr);
        __syncthreads();
        if (lane < 2 * H) w3i[lane] = gsm[L::W3 + (lane & 1) * H + (lane >> 1)];
        if (lane < 2) w3i[2 * H + lane] = gsm[L::B3 + lane];
        if (lane < H) {
            b2s[lane] = gsm[L::B2 + lane];
            c1s[lane >> 4][lane & 3][(lane >> 2) & 3] = gsm[L::B1 + lane];  // neuron lane = 16 hf + 4 r + g
        }
        // A of layer 1, lane (g, col): W1[16 hf + 4 (col % 4) + col / 4][g], 0 at g = 3
        float a1[NT];
#pragma unroll
        for (int hf = 0; hf < NT; ++hf)
            a1[hf] = grp < 3 ? gsm[L::W1 + 3 * (16 * hf + 4 * (col & 3) + (col >> 2)) + grp] : 0.0f;
        float w2f[NT][KS];  // A of layer 2: neuron 16 rt + col, k = 4 i + grp
#pragma unroll
        for (int rt = 0; rt < NT; ++rt)
#pragma unroll
            for (int i = 0; i < KS; ++i) w2f[rt][i] = gsm[L::W2 + (16 * rt + col) * H + 4 * i + grp];
        __syncthreads();  // gsm is dead from here
        float* hb = reinterpret_cast<float*>(big);  // [64][HP]; rows [64][4]: the columns' inputs
        const sgmm_env_params p = params[ep.param[e]];

        // per-lane path bookkeeping: byte s of cur = the state of the path that
        // started the chunk in state s (tracked starts: bits of sset)
        const uint32_t all = (1u << nsi) - 1u;
        const uint32_t sset = (!lane_ok || c >= nch) ? 0u : (c == 0 ? 1u << (uint32_t)(-inv_min) : all);
        const uint32_t p0 = sset ? (uint32_t)__builtin_ctz(sset) : 0u;
        uint64_t cur = kIdentityMap;
        // trade count along the path from each tracked start until the paths
        // merge (16 bits per start, two per word: a chunk has < 2^16 ticks), then
        // one count for the merged path
        uint32_t cnt[(NSI + 1) / 2];
#pragma unroll
        for (int s = 0; s < (NSI + 1) / 2; ++s) cnt[s] = 0;
        uint32_t mcnt = 0;
        bool merged = __builtin_popcount(sset) <= 1;
        int kc = merged ? 0 : CL;  // merge offset (CL: never)
        // (a split wave's idle lanes read the episode's first tick)
        auto tick_of = [&](int tt) { return tb + (LS == 1 || ntl > 0 ? t0 : 0) + min(tt, max(ntl - 1, 0)); };
#ifdef SGMM_STAMPS
        unsigned long long lite_t0, lite_sl = 0, lite_ts = 0, lite_s8 = 0, lite_s16 = 0;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(lite_t0)::"memory");
#endif
#ifdef SGMM_STAMPS_PHASE
        // per wave: 0 cycles, 1 layers 1-2 (MFMA issue), 2 layer-2 drain + transpose
        // + layer 3, 4 FPT step + plane stores, 5 per-tick head, 6 tick tail,
        // 3 slots run, 7 wall time (10 ns ticks)
        unsigned long long fs_t0, fs_a, fs_b, fs_c[7] = {0, 0, 0, 0, 0, 0, 0}, fs_r0;
#define SGMM_FT(var) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory")
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(fs_r0)::"memory");
        SGMM_FT(fs_t0);
#define SGMM_PH(k)                    \
        do {                              \
            unsigned long long t_;        \
            SGMM_FT(t_);                  \
            fs_c[k] += t_ - fs_b;         \
            fs_b = t_;                    \
        } while (0)
#else
#define SGMM_PH(k) \
        do {           \
        } while (0)
#endif
        int64_t ti = tick_of(0);
        float ns1 = tk.s1n[ti], ns2 = tk.s2n[ti];  // the signals one tick ahead
        int fr_extra = 0;
        if ((SP || LS == 1) && lane == 0) {
            nslot_s = 0;
            if (SP) tmin_s = (uint32_t)max(4, CL - kSpillTicks);
        }

        // layers 1-3 for the columns of this slot (their inputs in the rows of
        // hb as (s1, s2, inv/2, 0)); tiles >= NQ are skipped; o0 / o1 = the
        // outputs of this lane's column
        auto mlp = [&](auto nq, float& o0, float& o1, auto&& after_layer2) {
            constexpr int NQ = decltype(nq)::value;
            float xb[NQ];  // B of layer 1, lane (grp, col): input grp of column 16 q + col
#pragma unroll
            for (int q = 0; q < NQ; ++q) xb[q] = hb[(16 * q + col) * 4 + grp];
            f32x4 acc[NQ][NT];
            // two column tiles at a time: their layer-1 MFMAs, relu, then their
            // layer-2 MFMAs as one block (h1 of two tiles live, not four)
#pragma unroll
            for (int q0 = 0; q0 < NQ; q0 += 2) {
                constexpr int Q2 = NQ < 2 ? NQ : 2;
                f32x4 h1[Q2][NT];
#pragma unroll
                for (int hf = 0; hf < NT; ++hf) {
                    const f32x4 cc = *reinterpret_cast<const f32x4*>(&c1s[hf][grp][0]);
#pragma unroll
                    for (int q = 0; q < Q2; ++q)
                        h1[q][hf] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[hf], xb[q0 + q], cc, 0, 0, 0);
                }
#pragma unroll
                for (int q = 0; q < Q2; ++q)
#pragma unroll
                    for (int hf = 0; hf < NT; ++hf)
#pragma unroll
                        for (int r = 0; r < 4; ++r) h1[q][hf][r] = relu(h1[q][hf][r]);
#pragma unroll
                for (int rt = 0; rt < NT; ++rt) {
                    const f32x4 bb = *reinterpret_cast<const f32x4*>(&b2s[16 * rt + 4 * grp]);
#pragma unroll
                    for (int q = 0; q < Q2; ++q) acc[q0 + q][rt] = bb;
                }
#pragma unroll
                for (int i = 0; i < KS; ++i)
#pragma unroll
                    for (int q = 0; q < Q2; ++q)
#pragma unroll
                        for (int rt = 0; rt < NT; ++rt)
                            acc[q0 + q][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[rt][i], h1[q][i >> 2][i & 3],
                                                                                  acc[q0 + q][rt], 0, 0, 0);
            }
            SGMM_PH(1);
            after_layer2();
            asm volatile("" ::: "memory");  // the input rows are read before the transpose overwrites them
            o0 = w3i[2 * H];
            o1 = w3i[2 * H + 1];
#pragma unroll
            for (int rt = 0; rt < NT; ++rt) {
                // relu'd neurons 16 rt + 4 grp + r of column 16 q + col -> row 16 q + col
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = relu(acc[q][rt][r]);
                    *reinterpret_cast<f32x4*>(&hb[(16 * q + col) * HP + 4 * grp]) = v;
                }
                // layer 3 of this lane's column over neurons 16 rt .. 16 rt + 15, in
                // order; the weight pairs are read where they are used (an opaque
                // base: hoisted, the 64 floats would take 64 registers)
#pragma unroll 1
                for (int j4 = 0; j4 < 4; ++j4) {
                    lds_cf* w3p = (lds_cf*)(&w3i[2 * (16 * rt + 4 * j4)]);
                    asm volatile("" : "+v"(w3p));
                    const f32x4 h = *reinterpret_cast<const f32x4*>(&hb[lane * HP + 4 * j4]);
#pragma unroll
                    for (int r2 = 0; r2 < 2; ++r2) {
                        const f32x4 w = *reinterpret_cast<lds_cf4*>(w3p + 4 * r2);
                        o0 = __builtin_fmaf(w[0], h[2 * r2], o0);
                        o1 = __builtin_fmaf(w[1], h[2 * r2], o1);
                        o0 = __builtin_fmaf(w[2], h[2 * r2 + 1], o0);
                        o1 = __builtin_fmaf(w[3], h[2 * r2 + 1], o1);
                    }
                }
                asm volatile("" ::: "memory");  // this half's rows are read before the next half is written
            }
#ifdef SGMM_STAMPS_PHASE
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
            SGMM_PH(2);
        };

#pragma unroll 1
        for (int tt = 0; tt < CL; ++tt) {
#ifdef SGMM_STAMPS_PHASE
            SGMM_FT(fs_b);
#endif
            // spill: a walk still running at the launch's deadline (spill_budget, in
            // 10 ns since the wave started) stops here once its chunks have at most
            // kSpillTicks ticks left; k_frontier_spill finishes them tick-parallel from
            // the records written below (checked every 4 ticks)
            if constexpr (SP) {
                if ((tt & 3) == 0 && (uint32_t)tt >= (uint32_t)__builtin_amdgcn_readfirstlane((int)tmin_s) &&
                    (uint32_t)wall_clock64() - (uint32_t)__builtin_amdgcn_readfirstlane((int)t0_s) > args.spill_budget) {
                    if (lane == 0) spk_s = (uint32_t)tt;
                    break;
                }
            }
            const bool act = tt < ntl;
            const float s1 = ns1, s2 = ns2;
            const int64_t tcur = ti;
            ti = tick_of(tt + 1);
            ns1 = tk.s1n[ti];
            ns2 = tk.s2n[ti];
            // frontier: the distinct current states of the tracked paths
            uint32_t fmask = 0;
            if (merged) {
                fmask = 1u << map_get(cur, p0);
            } else {
#pragma unroll
                for (int s = 0; s < NSI; ++s)
                    if ((sset >> s) & 1u) fmask |= 1u << map_get(cur, (uint32_t)s);
            }
            if (!act) fmask = 0;
            // Slot 0: each lane's first frontier state in its own column (most
            // ticks need nothing more).  Slots 1..: the remaining (chunk, state)
            // pairs packed densely into the 64 columns, each with its own inputs.
            const uint32_t ext = fmask & (fmask - 1u);  // frontier states after the first
            int epfx = 0, etot = 0;
            if (__ballot(ext != 0u)) {
                *reinterpret_cast<f32x2*>(&sig[lane][0]) = f32x2{s1, s2};
                const uint32_t nex = (uint32_t)__builtin_popcount(ext);
                const uint64_t eb0 = __ballot(nex & 1u), eb1 = __ballot(nex & 2u), eb2 = __ballot(nex & 4u);
                epfx = mbcnt64(eb0) + 2 * mbcnt64(eb1) + 4 * mbcnt64(eb2);  // first pair of this lane
                etot = __popcll(eb0) + 2 * __popcll(eb1) + 4 * __popcll(eb2);  // extra pairs (uniform)
                uint32_t r = ext;
                int pp = epfx;
#pragma unroll
                for (int m = 0; m < NSI - 1; ++m)
                    if (r) {
                        pl[pp++] = (uint16_t)((lane << 3) | __builtin_ctz(r));
                        r &= r - 1u;
                    }
            }
            const bool any0 = __ballot(fmask != 0u) != 0ull;
            const int nx = (etot + kWave - 1) / kWave;
            // a walk whose ticks have needed extra slots for a while (its paths stay
            // apart: a heavy walk, the launch's tail) takes the SIMD's issue
            // priority over the light walks beside it (round 4, profiles/r04_ab)
            fr_extra = fr_extra - (fr_extra >> 3) + (nx << 5);  // decaying average of extra slots per tick, x 256
            if ((SP || LS == 1) && lane == 0)
                __hip_atomic_fetch_add(&nslot_s, (uint32_t)((any0 ? 1 : 0) + nx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            if ((tt & 7) == 7) {
                if (fr_extra > kFrPrioExtra) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(0);
            }
#ifdef SGMM_STAMPS
            lite_sl += (any0 ? 1 : 0) + nx;
            if (tt == 7) lite_s8 = lite_sl;
            if (tt == 15) lite_s16 = lite_sl;
            lite_ts += (any0 ? 4 : 0) + (etot + 15) / 16;
#endif
            // the tick's plane rows (tick-offset-major: row u of an episode's block
            // holds the 64 chunks' rewards at offset u, so a merged wave's store is
            // one coalesced 512-byte row); a uniform base, the plane stride opaque
            // per tick so the compiler keeps one address, not one per plane
            int64_t prs = ep.rs;
            asm volatile("" : "+s"(prs));
            const uint64_t pa = reinterpret_cast<uint64_t>(rew + rbase);
            uint64_t pu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pa >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pa);
            asm volatile("" : "+s"(pu));
            double* const prow = reinterpret_cast<double*>(pu) + frontier_row(tt, off);
            uint64_t stepmap = kIdentityMap;  // byte f = successor of frontier state f
            uint32_t trm = 0;                 // bit f: a fill from frontier state f
#ifdef SGMM_STAMPS_PHASE
            fs_c[3] += (any0 ? 1 : 0) + nx;
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
            SGMM_PH(5);
            if (any0) {
                const bool has = fmask != 0u;
                const uint32_t f = has ? (uint32_t)__builtin_ctz(fmask) : 0u;
                *reinterpret_cast<f32x4*>(&hb[lane * 4]) = f32x4{s1, s2, (float)(inv_min + (int)f) * 0.5f, 0.0f};
                float o0, o1;
                double tmid, task, tbid, tbmax, tsmin;
                // this tick's prices, requested after layer 2 (out of the register
                // peak), their latency hidden by layer 3
                mlp(IntC<NL / 16>{}, o0, o1, [&] {
                    tmid = tk.mid_next[tcur];
                    task = tk.best_ask[tcur];
                    tbid = tk.best_bid[tcur];
                    tbmax = tk.buy_max[tcur];
                    tsmin = tk.sell_min[tcur];
                });
                if (etot) {
                    px[0][lane] = tmid;
                    px[1][lane] = task;
                    px[2][lane] = tbid;
                    px[3][lane] = tbmax;
                    px[4][lane] = tsmin;
                }
                const int32_t oa = act_to_int(rintf(o0 * p.act_scale));  // drl_engine.py:38-39
                const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
                const StepOut so1 = ftp_step(p, inv_min + (int)f, oa, ob, tmid, task, tbid, tbmax, tsmin);
                if (has) {
                    const uint64_t to = (uint64_t)(f + so1.fill_buy - so1.fill_sell);
                    stepmap = (stepmap & ~(0xFFull << (8 * f))) | (to << (8 * f));
                    trm |= (uint32_t)(so1.fill_buy | so1.fill_sell) << f;
                    // the reward goes to the plane of every tracked start whose path
                    // is at f; after the merge only plane p0 is read
                    if (merged) {
                        prow[p0 * prs + lane] = so1.reward;
                    } else {
#pragma unroll
                        for (int s = 0; s < NSI; ++s)
                            if (((sset >> s) & 1u) && map_get(cur, (uint32_t)s) == f) prow[s * prs + lane] = so1.reward;
                    }
                }
#ifdef SGMM_STAMPS_PHASE
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
                SGMM_PH(4);
            }
#pragma unroll 1
            for (int x = 0; x < nx; ++x) {
                // column lane = pair 64 x + lane: (chunk src, state f)
                const int pidx = kWave * x + lane;
                const bool has = pidx < etot;
                const uint32_t v = has ? (uint32_t)pl[pidx] : 0u;
                const int src = (int)(v >> 3);
                const uint32_t f = v & 7u;
                const f32x2 sg = *reinterpret_cast<const f32x2*>(&sig[src][0]);
                *reinterpret_cast<f32x4*>(&hb[lane * 4]) = f32x4{sg[0], sg[1], (float)(inv_min + (int)f) * 0.5f, 0.0f};
                const int ntile = min(4, (etot - kWave * x + 15) >> 4);
                float o0, o1;
                if (ntile == 1)
                    mlp(IntC<1>{}, o0, o1, [] {});
                else if (ntile == 2)
                    mlp(IntC<2>{}, o0, o1, [] {});
                else
                    mlp(IntC<4>{}, o0, o1, [] {});
                // the FPT step with the pair's chunk's prices
                const double smid = px[0][src], sask = px[1][src], sbid = px[2][src], sbmax = px[3][src];
                const double ssmin = px[4][src];
                const int32_t oa = act_to_int(rintf(o0 * p.act_scale));  // drl_engine.py:38-39
                const int32_t ob = act_to_int(rintf(o1 * p.act_scale));
                const StepOut so1 = ftp_step(p, inv_min + (int)f, oa, ob, smid, sask, sbid, sbmax, ssmin);
                const uint64_t scur = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(cur >> 32), src, kWave) << 32) |
                                      (uint32_t)__shfl((int)(uint32_t)cur, src, kWave);
                if (has) {
                    // the pair's chunk is unmerged (a merged chunk has one state): every
                    // tracked start of chunk src whose path is at f
                    const uint32_t ss = cg * kFrontierLanes + off + src == 0 ? 1u << (uint32_t)(-inv_min) : all;
#pragma unroll
                    for (int s = 0; s < NSI; ++s)
                        if (((ss >> s) & 1u) && map_get(scur, (uint32_t)s) == f) prow[s * prs + src] = so1.reward;
                    const uint32_t to = f + (uint32_t)so1.fill_buy - (uint32_t)so1.fill_sell;
                    pl[pidx] = (uint16_t)(v | (to << 9) | ((uint32_t)(so1.fill_buy | so1.fill_sell) << 12));
                }
#ifdef SGMM_STAMPS_PHASE
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
                SGMM_PH(4);
            }
            if (etot) {
                // the owner lane collects its extra states' successors and fills
                uint32_t r = ext;
                int pp = epfx;
#pragma unroll
                for (int m = 0; m < NSI - 1; ++m)
                    if (r) {
                        const uint32_t f = (uint32_t)__builtin_ctz(r);
                        r &= r - 1u;
                        const uint32_t w = pl[pp++];
                        stepmap = (stepmap & ~(0xFFull << (8 * f))) | ((uint64_t)((w >> 9) & 7u) << (8 * f));
                        trm |= ((w >> 12) & 1u) << f;
                    }
            }
            // the trade counts along the tracked paths, the paths' new states
            if (act) {
                if (merged) {
                    mcnt += trm != 0u;
                } else {
#pragma unroll
                    for (int s = 0; s < NSI; ++s)
                        if ((sset >> s) & 1u) cnt[s >> 1] += ((trm >> map_get(cur, (uint32_t)s)) & 1u) << (16 * (s & 1));
                }
                cur = map_then(cur, stepmap);
                if (!merged) {
                    uint32_t fm = 0;
#pragma unroll
                    for (int s = 0; s < NSI; ++s)
                        if ((sset >> s) & 1u) fm |= 1u << map_get(cur, (uint32_t)s);
                    if (__builtin_popcount(fm) <= 1) {
                        merged = true;
                        kc = tt + 1;
                    }
                }
            }
#ifdef SGMM_STAMPS_PHASE
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
            SGMM_PH(6);
        }
#ifdef SGMM_STAMPS_PHASE
        {
            unsigned long long t_, r1;
            SGMM_FT(t_);
            fs_c[0] = t_ - fs_t0;
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
            if (lane == 0 && e < kStampWaves) {
                for (int k = 0; k < 7; ++k) g_tstamps[e][k] = fs_c[k];
                g_tstamps[e][7] = r1 - fs_r0;
            }
        }
#undef SGMM_FT
#endif
#undef SGMM_PH
#if defined(SGMM_STAMPS) && !defined(SGMM_STAMPS_PHASE)
        {
            unsigned long long t1;
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
            unsigned h_, x_;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)" : "=s"(h_), "=s"(x_));
            const int srow = e + cg * 16384;
            if (lane == 0 && srow < 32768) {
                g_tstamps[srow][0] = lite_t0;
                g_tstamps[srow][1] = t1;
                g_tstamps[srow][2] = lite_sl;
                g_tstamps[srow][3] = lite_ts;
                g_tstamps[srow][6] = lite_s8;
                g_tstamps[srow][7] = lite_s16;
                g_thwid[srow][0] = h_;
                g_thwid[srow][1] = x_;
            }
        }
#endif
        if (SP && lane == 0) {
            const uint32_t k = spk_s;
            if (k) {  // spilled: the entry for k_frontier_spill, and the walk-order feedback's
                      // slot count extrapolated to the whole walk
                args.wspill[wid_s] = k;
                nslot_s = __hip_atomic_load(&nslot_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) * (uint32_t)CL / k;
            }
        }
        if (lane_ok && c < nch) {
            // untracked start states keep the identity byte (never on the episode's path)
            uint64_t cm = kIdentityMap;
#pragma unroll
            for (int s = 0; s < NSI; ++s)
                if ((sset >> s) & 1u) cm = (cm & ~(0xFFull << (8 * s))) | ((uint64_t)map_get(cur, (uint32_t)s) << (8 * s));
            const int64_t ci = frontier_rec(e, ep.ngrp, c);
            cmaps[ci] = cm;
#pragma unroll
            for (int s = 0; s < NSI; ++s) ctr32[ci * 8 + s] = ((cnt[s >> 1] >> (16 * (s & 1))) & 0xFFFFu) + (((sset >> s) & 1u) ? mcnt : 0u);
            kinfo[ci] = (uint32_t)kc | ((uint32_t)nw << 20) | (p0 << 29);
            // the walk's slot count at (its first record) / 64 = e * ngrp + cg: indexed from
            // the live record index (a block index kept to here costs spills)
            if (LS == 1 && lane == 0 && args.wslots)
                args.wslots[ci / NL] = __hip_atomic_load(&nslot_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
    }  // the walk
    if constexpr (FS) {
        // the scan's arguments and the walk's episode come from LDS (fa_s, ep_s, ...):
        // nothing the scan needs is kept live through the walk loop
        FrontierArgs a{};
        uint32_t* aw = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
        for (int i = 0; i < kFaWords; ++i)
            aw[i < kFa1 - kFa0 ? kFa0 + i : kFa2 + i - (kFa1 - kFa0)] =
                (uint32_t)__builtin_amdgcn_readfirstlane((int)fa_s[i]);
        asm volatile("" ::: "memory");
        const int ef = __builtin_amdgcn_readfirstlane((int)ep_s);
        const int clf = __builtin_amdgcn_readfirstlane((int)cl_s);
        const int nchf = __builtin_amdgcn_readfirstlane((int)nch_s);
        const int cgf = __builtin_amdgcn_readfirstlane((int)cg_s);
        __syncthreads();  // the walk's LDS is dead: the scan's window and chunk tables
        fused_scan(a, ef, cgf, clf, nchf, reinterpret_cast<double*>(big), reinterpret_cast<uint32_t*>(&px[0][0]),
                   reinterpret_cast<uint8_t*>(&px[0][0]) + 4 * kFrontierLanes);
    }
}

// ------------------------------------------------------------------ spill: the rest of the heavy walks
// The frontier launch ends with its heaviest walks: policies whose paths rarely
// merge run up to five MLP slots per tick, serially, while the SIMDs around them
// have run dry (config 3: the last SIMD ends ~570 us into the launch, the median
// one at ~400 us, profiles/r05_timeline/tlo_g15_default.txt).  A walk that passes
// the launch's slot budget therefore stops at a tick offset K (a multiple of 4,
// once its chunks have at most kSpillTicks ticks left), leaving its records as
// they stand -- per chunk the map of the tracked start states to their states at
// K, the trade counts so far, the merge tick -- and K in wspill[its wave id].
// This kernel, stream-ordered after the walk launch, runs the remaining ticks of
// every spilled chunk tick-parallel: all inventory states of each tick, one wave
// per state (the state-parallel table's arithmetic, k_policy_table_sp), lanes =
// (chunk, tick) in segments of 16 / 32 / 64 ticks, then a segmented map scan
// composes each chunk's path from its state at K, and the kernel writes the plane
// rows of ticks K.. (every tracked start's plane, or p0's after the merge), the
// final map and the completed trade counts in the frontier layout -- exactly what
// the walk would have written, so the path scan reads them unchanged.
// Fixed grid (graph-capturable): every workgroup reads the launch's entries, ranks
// the spilled waves identically, and takes a contiguous range of the work items
// (spilled wave, 4 of its chunks); with nothing spilled it exits after one load.
constexpr int kSpillBlocks = 512;  // two workgroups per CU (54-83 KB of LDS each)
// wave_map_scan_seg for a runtime segment width (wave-uniform: every lane takes the same steps)
__device__ __forceinline__ uint64_t m_scan_seg(uint64_t m, int seg) {
    if (seg >= 64) return wave_map_scan_seg<64>(m);
    if (seg >= 32) return wave_map_scan_seg<32>(m);
    return wave_map_scan_seg<16>(m);
}
template <int H, int NSI>
__global__ __launch_bounds__(kWave * NSI) void k_frontier_spill(FrontierArgs args, int32_t n_waves, int32_t ls) {
    static_assert(H % 16 == 0 && H <= 32, "spill: H = 16 or 32");
    using L = GenomeLayout<H>;
    constexpr int NT = H / 16, KS = H / 4, HP = H + 4;
    constexpr int kPer = 16;   // entries per thread and segment
    constexpr int kCap = 512;  // spilled waves per window
    const EpArrays& ep = args.ep;
    const int tid = (int)threadIdx.x, nt = (int)blockDim.x, wv = tid >> 6, lane = tid & (kWave - 1);
    const int grp = lane >> 4, col = lane & 15;
    const int nwv = nt >> 6;
    const int NL = kFrontierLanes / ls;
    const int ipw = NL / 4;  // work items per spilled wave: 4 chunks each
    const int32_t inv_min = args.inv_min, nsi = args.nsi;
    __shared__ uint32_t list_s[kCap];
    __shared__ uint32_t wcnt_s[kPer][NSI];
    __shared__ __attribute__((aligned(16))) float gsm[L::N];
    __shared__ __attribute__((aligned(16))) float w3i[2 * H];
    __shared__ __attribute__((aligned(16))) float hb_s[NSI][kWave * HP];
    __shared__ __attribute__((aligned(16))) double rl_s[NSI][kWave];
    __shared__ uint8_t to_s[NSI][kWave];  // successor state | traded << 7
    int staged = -1;                      // the episode whose genome is in gsm
    float w2f[NT][KS];
    f32x4 b2c[NT];
    for (int seg0 = 0; seg0 < n_waves; seg0 += kPer * nt) {
        // this segment's entries in registers, ranked by (k, thread): the same
        // order in every workgroup
        uint32_t ent[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int b = seg0 + k * nt + tid;
            ent[k] = b < n_waves ? args.wspill[b] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint64_t m = __ballot(ent[k] != 0u);
            if (lane == 0) wcnt_s[k][wv] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        uint32_t total = 0, rank[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            uint32_t before = 0;
            for (int w = 0; w < nwv; ++w) {
                if (w == wv) before = total;
                total += wcnt_s[k][w];
            }
            rank[k] = before + (uint32_t)mbcnt64(__ballot(ent[k] != 0u));
        }
        __syncthreads();  // wcnt_s is rewritten by the next segment
        for (uint32_t r0 = 0; r0 < total; r0 += kCap) {
#pragma unroll
            for (int k = 0; k < kPer; ++k)
                if (ent[k] && rank[k] >= r0 && rank[k] < r0 + kCap) list_s[rank[k] - r0] = (uint32_t)(seg0 + k * nt + tid);
            __syncthreads();
            const int m = (int)min(total - r0, (uint32_t)kCap);
            const int items = m * ipw;
            const int per = (items + (int)gridDim.x - 1) / (int)gridDim.x;
            const int i0 = (int)blockIdx.x * per, i1 = min(items, i0 + per);
            for (int it = i0; it < i1; ++it) {
                const int b = (int)list_s[it / ipw], q = it % ipw;
                int pos, cg, nw;
                frontier_wave(ep, b / ls, pos, cg, nw);
                const int off = (b % ls) * NL;
                const int e = __builtin_amdgcn_readfirstlane(ep.order ? ep.order[pos] : pos);
                const int32_t T = ep.len[e];
                const int CL = frontier_len(T, nw);
                const int nch = (T + CL - 1) / CL;
                const int K = __builtin_amdgcn_readfirstlane((int)args.wspill[b]);
                const int R = CL - K;  // remaining ticks of a full chunk (1..kSpillTicks)
                const int SEG = __builtin_amdgcn_readfirstlane(R <= 16 ? 16 : (R <= 32 ? 32 : 64));
                const int shs = SEG == 16 ? 4 : (SEG == 32 ? 5 : 6);
                const int cpp = kWave / SEG;  // chunks per pass
                const int64_t tb = ep.tick_off[e], so = ep.step_off[e];
                const int64_t rbase = frontier_base(so, e, ep.ngrp) + (int64_t)cg * CL * kFrontierLanes;
                if (e != staged) {  // block-uniform
                    __syncthreads();
                    stage_genomes(args.src, e, ep.genome[e], -1, L::N, gsm, nullptr);
                    __syncthreads();
                    if (tid < 2 * H) w3i[tid] = gsm[L::W3 + (tid & 1) * H + (tid >> 1)];
#pragma unroll
                    for (int rt = 0; rt < NT; ++rt) {
#pragma unroll
                        for (int i = 0; i < KS; ++i) w2f[rt][i] = gsm[L::W2 + (16 * rt + col) * H + 4 * i + grp];
#pragma unroll
                        for (int r = 0; r < 4; ++r) b2c[rt][r] = gsm[L::B2 + 16 * rt + 4 * grp + r];
                    }
                    staged = e;
                    __syncthreads();
                }
                const sgmm_env_params p = args.params[ep.param[e]];
                for (int pass = 0; pass < 4 / cpp; ++pass) {
                    // sample s = lane: chunk (within the wave's NL) q*4 + pass*cpp + s/SEG, tick offset K + s%SEG
                    auto tick_of = [&](int smp, bool& ok, int& lg) {
                        const int ch = 4 * q + pass * cpp + (smp >> shs);
                        lg = off + ch;
                        const int c = cg * kFrontierLanes + lg, tt = K + (smp & (SEG - 1));
                        ok = c < nch && c * CL + tt < T && tt < CL;
                        return tb + min((int64_t)c * CL + tt, (int64_t)T - 1);
                    };
                    const int si = wv;
                    float xs0[4], xs1[4];
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq) {
                        bool ok;
                        int lg;
                        const int64_t ti = tick_of(16 * qq + col, ok, lg);
                        xs0[qq] = args.tk.s1n[ti];
                        xs1[qq] = args.tk.s2n[ti];
                    }
                    bool valid;
                    int lg;
                    const int64_t tix = tick_of(lane, valid, lg);
                    const double tmid = args.tk.mid_next[tix], task = args.tk.best_ask[tix], tbid = args.tk.best_bid[tix];
                    const double tbmax = args.tk.buy_max[tix], tsmin = args.tk.sell_min[tix];
                    const float x2 = (float)((double)(inv_min + si) / 2.0);
                    float h1[KS][4];
#pragma unroll
                    for (int i = 0; i < KS; ++i) {
                        const int k = 4 * i + grp;
                        const float a0 = gsm[L::W1 + 3 * k], a1 = gsm[L::W1 + 3 * k + 1], bb = gsm[L::B1 + k];
                        const float w1s = gsm[L::W1 + 3 * k + 2];
#pragma unroll
                        for (int qq = 0; qq < 4; ++qq)
                            h1[i][qq] = relu(__builtin_fmaf(w1s, x2, __builtin_fmaf(a1, xs1[qq], __builtin_fmaf(a0, xs0[qq], bb))));
                    }
                    f32x4 acc[4][NT];
#pragma unroll
                    for (int i = 0; i < KS; ++i)
#pragma unroll
                        for (int qq = 0; qq < 4; ++qq)
#pragma unroll
                            for (int rt = 0; rt < NT; ++rt)
                                acc[qq][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2f[rt][i], h1[i][qq],
                                                                                   i == 0 ? b2c[rt] : acc[qq][rt], 0, 0, 0);
                    float* hb = hb_s[si];
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
                        for (int rt = 0; rt < NT; ++rt) {
                            f32x4 v;
#pragma unroll
                            for (int r = 0; r < 4; ++r) v[r] = relu(acc[qq][rt][r]);
                            *reinterpret_cast<f32x4*>(&hb[(16 * qq + col) * HP + 16 * rt + 4 * grp]) = v;
                        }
                    float o0 = gsm[L::B3], o1 = gsm[L::B3 + 1];
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
                    const StepOut so1 = ftp_step(p, inv_min + si, oa, ob, tmid, task, tbid, tbmax, tsmin);
                    to_s[si][lane] = (uint8_t)((si + so1.fill_buy - so1.fill_sell) | ((so1.fill_buy | so1.fill_sell) << 7));
                    rl_s[si][lane] = so1.reward;
                    __syncthreads();
                    if (wv == 0) {
                        // the chunk's steps from K on: segmented map scan, then each tracked
                        // start's path from its state at K
                        uint64_t map = kIdentityMap;
                        uint32_t traded = 0;
                        if (valid) {
                            for (int st = 0; st < nsi; ++st) {
                                const uint32_t b8 = to_s[st][lane];
                                map = (map & ~(0xFFull << (8 * st))) | ((uint64_t)(b8 & 0x7Fu) << (8 * st));
                                traded |= (b8 >> 7) << st;
                            }
                        }
                        uint64_t inc = m_scan_seg(map, SEG);
                        uint64_t excl = shfl_up_u64(inc, 1);
                        const int u = lane & (SEG - 1);
                        if (u == 0) excl = kIdentityMap;
                        const int c = cg * kFrontierLanes + lg;
                        const bool has = c < nch;
                        const int64_t ci = frontier_rec(e, ep.ngrp, has ? c : 0);
                        const uint64_t cur = args.cmaps[ci];
                        const uint32_t ki = args.kinfo[ci];
                        const bool merged = (int)(ki & kKinfoTick) < CL;
                        const uint32_t p0 = ki >> 29;
                        const uint32_t all = (1u << nsi) - 1u;
                        const uint32_t sset = c == 0 ? 1u << (uint32_t)(-inv_min) : all;
                        const int sh = (lane >> shs) << shs;
                        const uint64_t segm = SEG == 64 ? ~0ull : (((1ull << SEG) - 1ull) << sh);
                        // the last valid tick of the chunk: R_c - 1 (<= SEG - 1)
                        const int ntl = has ? min(T, (c + 1) * CL) - c * CL : 0;
                        const bool last = valid && u == ntl - K - 1;
                        uint64_t cm = cur;
#pragma unroll
                        for (int st = 0; st < NSI; ++st) {
                            const bool tr = st < nsi && ((sset >> st) & 1u);
                            const uint32_t x = map_get(cur, (uint32_t)st);
                            const uint32_t y = map_get(excl, x & 7u);
                            if (valid && tr && (!merged || (uint32_t)st == p0))
                                args.rew[(int64_t)st * ep.rs + rbase + frontier_row(K + u, lg)] = rl_s[y & 7u][lane];
                            const uint32_t cnt = (uint32_t)__popcll(__ballot(valid && tr && ((traded >> (y & 7u)) & 1u)) & segm);
                            if (last && tr) {
                                args.ctr32[ci * 8 + st] += cnt;
                                cm = (cm & ~(0xFFull << (8 * st))) | ((uint64_t)map_get(inc, x & 7u) << (8 * st));
                            }
                        }
                        if (last) args.cmaps[ci] = cm;
                    }
                    __syncthreads();  // to_s / rl_s / hb_s are rewritten by the next pass
                }
            }
            __syncthreads();  // list_s is rewritten by the next window
        }
    }
}

int launch_frontier_spill(int hidden, int nsi, unsigned n_waves, int ls, hipStream_t s, const FrontierArgs& fa) {
    if (!fa.spill_budget || !fa.wspill || n_waves == 0) return SGMM_OK;
    const int total = (int)(n_waves * (unsigned)ls);
    const dim3 grid(kSpillBlocks), block(kWave * nsi);
    if (hidden == 16) {
        if (nsi <= 5) SGMM_LAUNCH((k_frontier_spill<16, 5>), grid, block, 0, s, fa, total, ls);
        else SGMM_LAUNCH((k_frontier_spill<16, 8>), grid, block, 0, s, fa, total, ls);
    } else {
        if (nsi <= 5) SGMM_LAUNCH((k_frontier_spill<32, 5>), grid, block, 0, s, fa, total, ls);
        else SGMM_LAUNCH((k_frontier_spill<32, 8>), grid, block, 0, s, fa, total, ls);
    }
    SGMM_LAUNCHED();
    return SGMM_OK;
}

int launch_policy_frontier(int hidden, int nsi, unsigned n_waves, int ls, hipStream_t s, const FrontierArgs& fa) {
    const dim3 grid(n_waves), block(kWave);
    if (fa.fitness && (ls != 1 || fa.ep.ngrp > kFusedMaxGroups || fa.spill_budget || !fa.handoff || !fa.hstate)) {
        set_error("fused path scan: one wave per walk, <= %d groups, no spill, hand-off arrays", kFusedMaxGroups);
        return SGMM_ERR_ARG;
    }
    {
        const dim3 gs(n_waves * (unsigned)ls);
#define SGMM_FR_LAUNCH2(H_, N_, SP_)                                                             \
    do {                                                                                         \
        if (ls == 4) SGMM_LAUNCH((k_policy_frontier<H_, N_, 4, SP_>), gs, block, 0, s, fa);      \
        else if (ls == 2) SGMM_LAUNCH((k_policy_frontier<H_, N_, 2, SP_>), gs, block, 0, s, fa); \
        else SGMM_LAUNCH((k_policy_frontier<H_, N_, 1, SP_>), grid, block, 0, s, fa);            \
    } while (0)
#define SGMM_FR_LAUNCH(H_, N_)                                                                  \
    do {                                                                                        \
        if (fa.fitness) SGMM_LAUNCH((k_policy_frontier<H_, N_, 1, false, true>), grid, block, 0, s, fa); \
        else if (fa.spill_budget && fa.wspill) SGMM_FR_LAUNCH2(H_, N_, true);                   \
        else SGMM_FR_LAUNCH2(H_, N_, false);                                                    \
    } while (0)
        if (hidden == 16) {
            if (nsi <= 5) SGMM_FR_LAUNCH(16, 5);
            else SGMM_FR_LAUNCH(16, 8);
        } else {
            if (nsi <= 5) SGMM_FR_LAUNCH(32, 5);
            else SGMM_FR_LAUNCH(32, 8);
        }
#undef SGMM_FR_LAUNCH
#undef SGMM_FR_LAUNCH2
    }
    SGMM_LAUNCHED();
    return SGMM_OK;
}

}  // namespace sgmm

#ifdef SGMM_STAMPS
extern "C" int sgmm_debug_frontier_tstamps(unsigned long long* host, int n_waves) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(sgmm::g_tstamps), sizeof(unsigned long long) * 8 * n_waves);
}
extern "C" int sgmm_debug_frontier_thwid(unsigned int* host, int n_waves) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(sgmm::g_thwid), sizeof(unsigned int) * 2 * n_waves);
}
#endif
