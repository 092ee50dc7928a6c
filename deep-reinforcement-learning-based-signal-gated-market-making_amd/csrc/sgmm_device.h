// sgmm_device.h -- device-side building blocks shared by the gfx950 kernels.
//
// Everything here is written for CDNA4 (wave64, gfx950) directly.  The
// numerics contract (see include/sgmm.h) is implemented once, here:
//   * ftp_fill / ftp_step: FTPEnv.step (Env/market_env.py:22-67) in float64,
//     reference operation order; the library is compiled with
//     -ffp-contract=off so `a + b * c` never becomes v_fma_f64.
//   * mlp_*: TradingPolicy / AdversaryPolicy forward (models/model.py:5-57),
//     every dot product the k-ordered fused chain from the bias (v_fma_f32).
//   * philox / normal4: counter-based N(0,1) stream for NeuroEvolution.ask.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sgmm.h"

namespace sgmm {

constexpr int kWave = 64;

// ReLU as one v_med3_f32(a, 0, +inf) on the float pipe.  +inf goes through an
// empty asm (opaque to the optimizer, hoisted once per kernel): a visible
// med3(a, 0, inf) is folded into max(a, 0), and max of an MFMA result gets an
// extra canonicalising v_max per value.  Not the integer max on the bit
// pattern: while another wave of the SIMD streams MFMAs, integer VALU ops
// issue at half rate and float ops at full rate (tools/mb/mb_mfma_xwave2.hip).
// Equals torch's relu for every non-NaN input (-0.0 -> +0.0 up to the sign of
// an exact zero, which no action depends on); NaN pre-activations (NaN state
// inputs only) are outside the parity domain (oracle/sgmm_oracle.c relu32).
__device__ __forceinline__ float relu(float a) {
#ifdef SGMM_RELU_INT  // A/B builds only: round 1's integer max on the bit pattern
    return __int_as_float(max(__float_as_int(a), 0));
#else
    float pinf = __builtin_inff();
    asm("" : "+s"(pinf));
    return __builtin_amdgcn_fmed3f(a, 0.0f, pinf);
#endif
}

// float -> int action: saturating, NaN -> INT32_MIN (the x86 cvtt value numpy's
// astype(int) produces).  Values are already integral (rint) when called.
// Branch-free: fmaxf maps NaN to the lower clamp, so NaN and -inf both land
// on -2^31; the upper clamp is the largest float below 2^31.
__device__ __forceinline__ int32_t act_to_int(float r) {
    const int32_t v = (int32_t)fminf(fmaxf(r, -2147483648.0f), 2147483520.0f);
    return r >= 2147483520.0f ? INT32_MAX : v;
}

// ---------------------------------------------------------------- FTPEnv.step
struct StepOut {
    double reward, pnl, fee_paid;
    int32_t inv;
    int fill_buy, fill_sell;
    double cash_delta_buy, cash_delta_sell;  // applied to cash in reference order
};

// One FTPEnv.step from inventory `inv` with final offsets (adversary already
// added, market_env.py:25-28).  Pure function of its inputs.
__device__ __forceinline__ StepOut ftp_step(const sgmm_env_params& p, int32_t inv,
                                            int32_t off_a, int32_t off_b, double mid_next,
                                            double best_ask, double best_bid, double buy_max,
                                            double sell_min) {
    StepOut o;
    const double qa = best_ask + (double)off_a * p.tick;   // market_env.py:30
    const double qb = best_bid - (double)off_b * p.tick;   // market_env.py:31
    o.fill_buy = (inv < p.i_max) && (qb >= sell_min);      // :34,:37 (NaN -> no fill)
    o.fill_sell = (inv > p.i_min) && (qa <= buy_max);      // :35,:38
    // both sides computed, then selected: the same operations in the same
    // order as the reference's conditional updates (no branches on the GPU)
    const double fb = qb * p.fee, fs = qa * p.fee;         // :44-55
    const double pnl_b = o.fill_buy ? 0.0 + ((mid_next - qb) - fb) : 0.0;
    const double pnl = o.fill_sell ? pnl_b + ((qa - mid_next) - fs) : pnl_b;
    const double fee_b = o.fill_buy ? 0.0 + fb : 0.0;
    const double fees = o.fill_sell ? fee_b + fs : fee_b;
    o.cash_delta_buy = o.fill_buy ? qb + fb : 0.0;
    o.cash_delta_sell = o.fill_sell ? qa - fs : 0.0;
    const int32_t q = inv + o.fill_buy - o.fill_sell;
    o.inv = q;
    o.pnl = pnl;
    o.fee_paid = fees;
    o.reward = pnl - p.phi * (double)(q < 0 ? -q : q);     // :57-58
    return o;
}

// cash update with the reference's two separate in-place ops (:47, :53)
__device__ __forceinline__ double apply_cash(double cash, const StepOut& o) {
    if (o.fill_buy) cash -= o.cash_delta_buy;
    if (o.fill_sell) cash += o.cash_delta_sell;
    return cash;
}

// ---------------------------------------------------------------- policy MLP
// Genome layout (parameters() order, model.py:8-15): W1[H,3] b1[H] W2[H,H]
// b2[H] W3[2,H] b3[2].
template <int H>
struct GenomeLayout {
    static constexpr int W1 = 0, B1 = 3 * H, W2 = 4 * H, B2 = 4 * H + H * H;
    static constexpr int W3 = 5 * H + H * H, B3 = 7 * H + H * H, N = 7 * H + H * H + 2;
};

// Full forward for one state; `g` may be a per-lane or a uniform pointer.
template <int H>
__device__ __forceinline__ void mlp_forward(const float* __restrict__ g, float x0, float x1,
                                            float x2, float& out0, float& out1) {
    using L = GenomeLayout<H>;
    float h1[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        float a = g[L::B1 + j];
        a = __builtin_fmaf(g[L::W1 + 3 * j + 0], x0, a);
        a = __builtin_fmaf(g[L::W1 + 3 * j + 1], x1, a);
        a = __builtin_fmaf(g[L::W1 + 3 * j + 2], x2, a);
        h1[j] = relu(a);
    }
    float o0 = g[L::B3 + 0], o1 = g[L::B3 + 1];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        float a = g[L::B2 + j];
#pragma unroll
        for (int k = 0; k < H; ++k) a = __builtin_fmaf(g[L::W2 + j * H + k], h1[k], a);
        const float h2 = relu(a);
        // layer 3 accumulates in j order: the same chain as
        // out_o = b3[o]; for j: out_o = fma(W3[o,j], h2[j], out_o)
        o0 = __builtin_fmaf(g[L::W3 + j], h2, o0);
        o1 = __builtin_fmaf(g[L::W3 + H + j], h2, o1);
    }
    out0 = o0;
    out1 = o1;
}

// AdversaryPolicy (model.py:38-57): 3 -> 12 (ReLU) -> 2 (tanh), weights = the
// first 74 floats of the genome row.
__device__ __forceinline__ void adv_forward(const float* __restrict__ g, float x0, float x1,
                                            float x2, float& out0, float& out1) {
    float h[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        float a = g[36 + j];
        a = __builtin_fmaf(g[3 * j + 0], x0, a);
        a = __builtin_fmaf(g[3 * j + 1], x1, a);
        a = __builtin_fmaf(g[3 * j + 2], x2, a);
        h[j] = relu(a);
    }
    float o0 = g[72], o1 = g[73];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        o0 = __builtin_fmaf(g[48 + j], h[j], o0);
        o1 = __builtin_fmaf(g[60 + j], h[j], o1);
    }
    out0 = tanhf(o0);
    out1 = tanhf(o1);
}

// Adversary delta for state (inventory, sell flag, buy flag): drl_engine.py:43-48
// (round(tanh * scale)) and market_env.py:26 (round again: idempotent).
__device__ __forceinline__ void adv_delta(const float* __restrict__ g, const sgmm_env_params& p,
                                          int32_t inv, int fill_sell_prev, int fill_buy_prev,
                                          int32_t& da, int32_t& db) {
    float r0, r1;
    adv_forward(g, (float)((double)inv / 2.0), fill_sell_prev ? 1.0f : 0.0f,
                fill_buy_prev ? 1.0f : 0.0f, r0, r1);
    da = act_to_int(rintf(r0 * p.adv_scale));
    db = act_to_int(rintf(r1 * p.adv_scale));
}

// ---------------------------------------------------------------- cross-lane (DPP)
// Data-parallel-primitive moves: a VALU operand modifier, no LDS round trip.
// Lanes whose source is outside the row (or whose row is masked off) get
// `old`.  Integer / float32 data only: DPP moves fed directly by float64
// arithmetic measured wrong-but-plausible values on gfx950 (the exact sum
// stayed exact -- its verification caught every misprediction -- but ran 4x
// slower), so float64 partial sums are never exchanged this way.  GFX9 controls: row_shr:n = 0x110 + n, row_bcast:15 = 0x142,
// row_bcast:31 = 0x143.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp32(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint64_t dpp64(uint64_t old, uint64_t v) {
    const uint32_t lo = dpp32<CTRL, ROW_MASK>((uint32_t)old, (uint32_t)v);
    const uint32_t hi = dpp32<CTRL, ROW_MASK>((uint32_t)(old >> 32), (uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
// inclusive prefix sums within rows of 16 lanes / over the wave
__device__ __forceinline__ uint64_t row_scan_add(uint64_t v) {
    v += dpp64<0x111>(0, v);
    v += dpp64<0x112>(0, v);
    v += dpp64<0x114>(0, v);
    v += dpp64<0x118>(0, v);
    return v;
}
__device__ __forceinline__ uint64_t wave_scan_add(uint64_t v) {
    v = row_scan_add(v);
    v += dpp64<0x142, 0xA>(0, v);
    v += dpp64<0x143, 0xC>(0, v);
    return v;
}
// inclusive min / max scans within rows of 16 lanes (signed 64-bit)
__device__ __forceinline__ int64_t row_scan_min(int64_t v) {
    v = min(v, (int64_t)dpp64<0x111>((uint64_t)INT64_MAX, (uint64_t)v));
    v = min(v, (int64_t)dpp64<0x112>((uint64_t)INT64_MAX, (uint64_t)v));
    v = min(v, (int64_t)dpp64<0x114>((uint64_t)INT64_MAX, (uint64_t)v));
    v = min(v, (int64_t)dpp64<0x118>((uint64_t)INT64_MAX, (uint64_t)v));
    return v;
}
__device__ __forceinline__ int64_t row_scan_max(int64_t v) {
    v = max(v, (int64_t)dpp64<0x111>((uint64_t)INT64_MIN, (uint64_t)v));
    v = max(v, (int64_t)dpp64<0x112>((uint64_t)INT64_MIN, (uint64_t)v));
    v = max(v, (int64_t)dpp64<0x114>((uint64_t)INT64_MIN, (uint64_t)v));
    v = max(v, (int64_t)dpp64<0x118>((uint64_t)INT64_MIN, (uint64_t)v));
    return v;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------- Philox4x32-10
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Four N(0,1) floats for counter (block, individual, gen, stream) via
// Box-Muller on two uniform pairs in (0,1].
__device__ __forceinline__ void normal4(uint64_t seed, uint32_t stream_id, uint32_t gen,
                                        uint32_t indiv, uint32_t block, float z[4]) {
    const U4 r = philox4x32_10(U4{block, indiv, gen, stream_id}, (uint32_t)seed,
                               (uint32_t)(seed >> 32));
    const float inv32 = 2.3283064365386963e-10f;  // 2^-32
    const float u0 = ((float)r.x + 1.0f) * inv32;  // (0, 1]
    const float u1 = (float)r.y * inv32;           // [0, 1)
    const float u2 = ((float)r.z + 1.0f) * inv32;
    const float u3 = (float)r.w * inv32;
    const float m0 = sqrtf(-2.0f * logf(u0 > 1.0f ? 1.0f : u0));
    const float m1 = sqrtf(-2.0f * logf(u2 > 1.0f ? 1.0f : u2));
    float s0, c0, s1, c1;
    sincospif(2.0f * u1, &s0, &c0);
    sincospif(2.0f * u3, &s1, &c1);
    z[0] = m0 * c0;
    z[1] = m0 * s0;
    z[2] = m1 * c1;
    z[3] = m1 * s1;
}

// ask() of one individual, 4 consecutive parameters (models/model.py:65-71).
// out = master + (z * (float)sigma): the reference's randn_like * sigma in
// float32, then the float32 add (model.py:69-70).
__device__ __forceinline__ void ask_row4(const float* __restrict__ master, int64_t n_params,
                                         float sig, uint64_t seed, uint32_t sid, uint32_t gen,
                                         uint32_t indiv, int64_t k4, float* dst) {
    float z[4];
    normal4(seed, sid, gen, indiv, (uint32_t)k4, z);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t k = 4 * k4 + q;
        if (k < n_params) {
            const float noise = z[q] * sig;
            dst[q] = master[k] + noise;
        }
    }
}

// first index of the maximum, NaN counting as the maximum (np.argmax)
__device__ __forceinline__ bool better(double a, int ia, double b, int ib) {
    // branch-free (selects, no divergent control flow inside shuffle reductions)
    const bool na = a != a, nb = b != b;
    const bool tie = na || a == b;
    const bool ord = tie ? (ia < ib) : (a > b);
    return na == nb ? ord : na;
}

// Population results gathered shard by shard: individual i's value lives in
// shard i / n at byte offset (i / n) * stride, element i % n (n <= 0: one
// contiguous array).  This is the layout of an all-gather of per-rank records.
struct ShardView {
    int32_t n;
    int64_t stride;
};

template <class T>
__device__ __forceinline__ T shard_at(const T* __restrict__ base, ShardView v, int i) {
    if (v.n <= 0) return base[i];
    const char* p = reinterpret_cast<const char*>(base) + (int64_t)(i / v.n) * v.stride;
    return reinterpret_cast<const T*>(p)[i % v.n];
}

constexpr int kMaxStepParams = 4096;  // largest genome a one-workgroup GA step stages in LDS

}  // namespace sgmm
