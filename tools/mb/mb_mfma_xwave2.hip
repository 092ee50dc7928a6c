// Microbenchmark: how much vector issue does ANOTHER wave's f32 MFMA stream
// take from a wave on the same SIMD (gfx950)?  One workgroup of 8 waves:
// waves 0-3 (one per SIMD) stream independent MFMAs, waves 4-7 (the same
// SIMDs) a throughput-bound vector loop of one instruction class (8
// independent accumulators, each reused 8 instructions later).  Each wave
// records its own clock span.  Mode 0: both, 1: MFMA waves only, 2: vector
// waves only.  MFMA kind: 0 = 16x16x4 f32 (32 cycles), 1 = 32x32x2 f32 (64).
// Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int KIND, int MK>
__global__ void k_xwave2(float* out, int iters, int mode, long long* cyc) {
    const int w = threadIdx.x >> 6;
    const bool mf = w < 4;
    long long t0 = clock64(), t1 = t0;
    float s = 0.f;
    if (mf && mode != 2) {
        const float a = threadIdx.x * 1e-3f, b = 1.0f - a;
        if (MK == 0) {
            f32x4 acc[8];
            for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            t0 = clock64();
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m], 0, 0, 0);
            }
            t1 = clock64();
            for (int i = 0; i < 8; ++i) s += acc[i][0];
        } else {
            f32x16 acc[4];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
            t0 = clock64();
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int m = 0; m < 4; ++m) acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m], 0, 0, 0);
            }
            t1 = clock64();
            for (int i = 0; i < 4; ++i) s += acc[i][0];
        }
    } else if (!mf && mode != 1) {
        float v[8];
        int iv[8];
        double d[8];
        f32x2 p[8];
        const float wv = out[1000];
        const double dw = out[1001];
        const int sh = (int)out[1002];
        for (int i = 0; i < 8; ++i) {
            v[i] = threadIdx.x * (i + 1) * 1e-3f;
            iv[i] = threadIdx.x - i;
            d[i] = v[i];
            p[i] = f32x2{v[i], -v[i]};
        }
        t0 = clock64();
        // 64 instructions per iteration (32 for the f64 class)
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 64; ++k) {
                if (KIND == 0) v[k & 7] = v[k & 7] + wv;                            // v_add_f32
                if (KIND == 1) iv[k & 7] = max(iv[k & 7], iv[(k + 3) & 7]);         // v_max_i32
                if (KIND == 2) v[k & 7] = __builtin_fmaxf(v[k & 7], v[(k + 3) & 7]);  // v_max_f32
                if (KIND == 3) p[k & 7] = __builtin_elementwise_fma(p[k & 7], f32x2{wv, wv}, p[(k + 1) & 7]);  // v_pk_fma_f32
                if (KIND == 4 && k < 32) d[k & 7] = __builtin_fma(d[k & 7], dw, dw);  // v_fma_f64
                if (KIND == 5) iv[k & 7] = __builtin_amdgcn_perm(iv[k & 7], iv[(k + 3) & 7], 0x05040100u + k);  // v_perm_b32
                if (KIND == 6) iv[k & 7] = iv[k & 7] ^ iv[(k + 3) & 7];              // v_xor_b32
                if (KIND == 7) v[k & 7] = __builtin_fmaf(v[k & 7], wv, 0.5f);        // v_fma_f32
            }
        }
        t1 = clock64();
        for (int i = 0; i < 8; ++i) s += v[i] + (float)iv[i] + (float)d[i] + p[i][0] + p[i][1];
    }
    out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

template <int KIND, int MK>
void run(const char* name, float* out, long long* cyc) {
    const int iters = 4096;
    long long c[8];
    double mf[3] = {0, 0, 0}, vv[3] = {0, 0, 0};
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL((k_xwave2<KIND, MK>), dim3(1), dim3(512), 0, 0, out, iters, mode, cyc);
        hipLaunchKernelGGL((k_xwave2<KIND, MK>), dim3(1), dim3(512), 0, 0, out, iters, mode, cyc);
        hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        for (int w = 0; w < 4; ++w) mf[mode] += (double)c[w] / iters / 4;
        for (int w = 4; w < 8; ++w) vv[mode] += (double)c[w] / iters / 4;
    }
    const int nins = KIND == 4 ? 32 : 64;
    printf("%-14s mfma%s | vector alone %6.1f cyc/iter (%5.2f per instr) | with MFMA waves %6.1f (%5.2f per instr)"
           " | MFMA waves alone %6.1f, with vector %6.1f cyc/iter\n",
           name, MK ? "32x32x2" : "16x16x4", vv[2], vv[2] / nins, vv[0], vv[0] / nins, mf[1], mf[0]);
}

template <int MK>
void all(float* out, long long* cyc) {
    run<0, MK>("v_add_f32", out, cyc);
    run<1, MK>("v_max_i32", out, cyc);
    run<2, MK>("v_max_f32", out, cyc);
    run<3, MK>("v_pk_fma_f32", out, cyc);
    run<4, MK>("v_fma_f64", out, cyc);
    run<5, MK>("v_perm_b32", out, cyc);
    run<6, MK>("v_xor_b32", out, cyc);
    run<7, MK>("v_fma_f32", out, cyc);
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 1 << 20);
    hipMemset(out, 0, 1 << 20);
    hipMalloc(&cyc, 64);
    all<0>(out, cyc);
    all<1>(out, cyc);
    return 0;
}
