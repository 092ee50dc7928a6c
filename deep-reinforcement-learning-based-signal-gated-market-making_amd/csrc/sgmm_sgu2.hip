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
// window and step: 4H(H+1) FMAs + 3H sigmoids + 2H tanh; the input is 4T
// bytes per window -- VALU-bound, not HBM-bound.
#include <cmath>

#include "sgmm_device.h"
#include "sgmm_internal.h"

namespace sgmm {

constexpr int kSgu2Block = 256;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

template <int H>
__global__ __launch_bounds__(kSgu2Block) void k_sgu2(const float* __restrict__ w, const float* __restrict__ X,
                                                     int64_t n, int T, const float* __restrict__ mean,
                                                     const float* __restrict__ std_, float* __restrict__ out) {
    constexpr int G = 4 * H;
    const float* w_ih = w;                 // [4H, 1]
    const float* w_hh = w_ih + G;          // [4H, H]
    const float* b_ih = w_hh + G * H;      // [4H]
    const float* b_hh = b_ih + G;          // [4H]
    const float* fc_w = b_hh + G;          // [1, H]
    const float* fc_b = fc_w + H;          // [1]
    const int64_t i = (int64_t)blockIdx.x * kSgu2Block + threadIdx.x;
    if (i >= n) return;
    const bool scaled = mean != nullptr;
    const float mu = scaled ? mean[0] : 0.0f, sd = scaled ? std_[0] : 1.0f;
    float h[H], c[H];
#pragma unroll
    for (int j = 0; j < H; ++j) h[j] = c[j] = 0.0f;
    const float* x = X + i * T;
    for (int t = 0; t < T; ++t) {
        const float xt = scaled ? (x[t] - mu) / sd : x[t];
        float g[G];
#pragma unroll
        for (int r = 0; r < G; ++r) {
            // input part (W_ih x + b_ih) and hidden part (W_hh h + b_hh), then summed
            float hh = 0.0f;
#pragma unroll
            for (int k = 0; k < H; ++k) hh = fmaf(w_hh[r * H + k], h[k], hh);
            g[r] = (w_ih[r] * xt + b_ih[r]) + (hh + b_hh[r]);
        }
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const float ig = sigmoidf_(g[j]), fg = sigmoidf_(g[H + j]);
            const float gg = tanhf(g[2 * H + j]), og = sigmoidf_(g[3 * H + j]);
            c[j] = fg * c[j] + ig * gg;
            h[j] = og * tanhf(c[j]);
        }
    }
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
