// sgmm_sgu2.hip -- SGU2 inference on gfx950: the LSTM
// signal unit that turns every SGU2 window into the s2 signal of the bundle.
//
// Reference semantics (restated and pinned in oracle/sgu2_oracle.py):
//   utils/scaler.py:14-18        StandardScaler3D.transform, float32
//                                (X - mean) / std (fit on float32 windows)
//   models/GateUnits.py:42-54    SGU2Model.forward, eval mode: nn.LSTM(1, H)
//                                over the window (gate rows i, f, g, o),
//                                the last hidden state -> Dropout (identity)
//                                -> Linear(H, 1)
//   models/GateUnits.py:116-120  SGU2.predict: float32 in, float32 out
//
// One thread per window, the whole recurrence in registers.  The weights are
// wave-uniform: they are read with scalar loads (s_load, scalar cache) and
// used as SGPR operands of the FMAs, so there is no LDS traffic at all.  Per
// window and step: 4H*H multiply-adds as 2H*H packed FMAs (v_pk_fma_f32: two
// columns of a gate row per instruction), 3H sigmoids + 2H tanh on the
// transcendental unit (v_exp_f32 + v_rcp_f32: 1/(1+2^(-x log2 e)) and
// 1 - 2/(1+2^(2x log2 e)), saturating correctly at +-inf); the input is 4T
// bytes per window -- VALU-bound, not HBM-bound.  Float32 throughout; the
// summation order and the hardware exp2/rcp differ from the reference's CPU
// LSTM within the tolerance tests/test_sgu2.py states.
#include <cmath>

#include "sgmm_device.h"
#include "sgmm_internal.h"

namespace sgmm {

constexpr int kSgu2Block = 256;

typedef float f32x2 __attribute__((ext_vector_type(2)));
// constant address space: wave-uniform loads through it become s_load
typedef const __attribute__((address_space(4))) float* CFloatPtr;
constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ float sigmoid_fast(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * kLog2e));
}

__device__ __forceinline__ float tanh_fast(float x) {
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(2.0f * kLog2e * x)), 1.0f);
}

template <int H>
__global__ __launch_bounds__(kSgu2Block) void k_sgu2(const float* __restrict__ w, const float* __restrict__ X,
                                                     int64_t n, int T, const float* __restrict__ mean,
                                                     const float* __restrict__ std_, float* __restrict__ out) {
    constexpr int G = 4 * H;
    const int64_t i = (int64_t)blockIdx.x * kSgu2Block + threadIdx.x;
    if (i >= n) return;
    const bool scaled = mean != nullptr;
    const float mu = scaled ? mean[0] : 0.0f, sd = scaled ? std_[0] : 1.0f;
    float h[H], c[H];
#pragma unroll
    for (int j = 0; j < H; ++j) h[j] = c[j] = 0.0f;
    const float* x = X + i * T;
    for (int t = 0; t < T; ++t) {
        // re-derive the weight pointer every step: the 4H(H+3) weights are
        // re-read from the scalar cache per step instead of being hoisted into
        // (and spilled out of) SGPRs for the whole loop
        uint64_t wa = reinterpret_cast<uint64_t>(w);
        asm volatile("" : "+s"(wa));
        const CFloatPtr w_ih = reinterpret_cast<CFloatPtr>(wa);  // [4H, 1]
        const CFloatPtr w_hh = w_ih + G;                         // [4H, H]
        const CFloatPtr b_ih = w_hh + G * H;                     // [4H]
        const CFloatPtr b_hh = b_ih + G;                         // [4H]
        const float xt = scaled ? (x[t] - mu) / sd : x[t];
        float g[G];
#pragma unroll
        for (int r = 0; r < G; ++r) {
            // input part (W_ih x + b_ih) and hidden part (W_hh h + b_hh), then summed;
            // the hidden part as two interleaved partial sums (even / odd columns)
            f32x2 acc = {0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k + 1 < H; k += 2)
                acc = __builtin_elementwise_fma(f32x2{w_hh[r * H + k], w_hh[r * H + k + 1]}, f32x2{h[k], h[k + 1]}, acc);
            float hh = acc.x + acc.y;
            if (H & 1) hh = fmaf(w_hh[r * H + H - 1], h[H - 1], hh);
            g[r] = fmaf(w_ih[r], xt, b_ih[r]) + (hh + b_hh[r]);
        }
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float ig = sigmoid_fast(g[j]), fg = sigmoid_fast(g[H + j]);
            const float gg = tanh_fast(g[2 * H + j]), og = sigmoid_fast(g[3 * H + j]);
            c[j] = fmaf(fg, c[j], ig * gg);
            h[j] = og * tanh_fast(c[j]);
        }
    }
    const float* fc_w = w + 3 * G + G * H;     // [1, H] after w_ih, w_hh, b_ih, b_hh
    const float* fc_b = fc_w + H;              // [1]
    float y = 0.0f;
#pragma unroll
    for (int k = 0; k < H; ++k) y = fmaf(fc_w[k], h[k], y);
    out[i] = y + fc_b[0];
}

}  // namespace sgmm

using namespace sgmm;

extern "C" int sgmm_sgu2_forward(const float* weights, int32_t hidden, const float* X, int64_t n,
                                 int32_t time_steps, const float* mean, const float* std_, float* out,
                                 void* stream) {
    clear_error();
    SGMM_REQUIRE(weights, "null weights");
    SGMM_REQUIRE((mean == nullptr) == (std_ == nullptr), "mean and std must both be given or both NULL");
    SGMM_REQUIRE(n >= 0 && time_steps >= 0, "negative size");
    SGMM_REQUIRE(hidden == 10 || hidden == 16 || hidden == 32, "hidden %d not in {10, 16, 32}", hidden);
    if (n == 0) return SGMM_OK;  // empty windows may come with NULL buffers
    SGMM_REQUIRE(X && out, "null windows / output");
    const dim3 grid((unsigned)((n + kSgu2Block - 1) / kSgu2Block)), block(kSgu2Block);
    ProfScope prof("sgu2", as_stream(stream));
    switch (hidden) {
        case 10: hipLaunchKernelGGL(k_sgu2<10>, grid, block, 0, as_stream(stream), weights, X, n, time_steps, mean, std_, out); break;
        case 16: hipLaunchKernelGGL(k_sgu2<16>, grid, block, 0, as_stream(stream), weights, X, n, time_steps, mean, std_, out); break;
        default: hipLaunchKernelGGL(k_sgu2<32>, grid, block, 0, as_stream(stream), weights, X, n, time_steps, mean, std_, out); break;
    }
    SGMM_LAUNCHED();
    return SGMM_OK;
}
