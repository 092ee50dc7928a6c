// Microbenchmark (round 5): which vector / LDS instruction classes of one wave
// overlap ANOTHER wave's f32 MFMA stream on the same SIMD (gfx950)?  Extends
// mb_mfma_xwave2.hip with the classes the frontier kernel's register transpose
// and packed layer 1 would use: v_permlane32_swap, v_permlane16_swap,
// v_pk_fma_f32, v_med3_f32, ds_read_b128, ds_bpermute.  One workgroup of 8
// waves: waves 0-3 stream independent 16x16x4 f32 MFMAs, waves 4-7 a
// throughput-bound loop of one class (8 independent registers, each reused 8
// instructions later).  Mode 0: both, 1: MFMA waves only, 2: vector waves only.
// Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void k_xwave3(float* out, int iters, int mode, long long* cyc) {
    __shared__ f32x4 lds[512];
    const int w = threadIdx.x >> 6;
    const bool mf = w < 4;
    for (int i = threadIdx.x; i < 512; i += blockDim.x) lds[i] = f32x4{(float)i, 1.f, 2.f, 3.f};
    __syncthreads();
    long long t0 = clock64(), t1 = t0;
    float s = 0.f;
    if (mf && mode != 2) {
        const float a = threadIdx.x * 1e-3f, b = 1.0f - a;
        f32x4 acc[8];
        for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        t0 = clock64();
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m], 0, 0, 0);
        }
        t1 = clock64();
        for (int i = 0; i < 8; ++i) s += acc[i][0];
    } else if (!mf && mode != 1) {
        float v[8];
        unsigned u[8];
        int iv[8];
        double d[8];
        f32x2 p[8];
        f32x4 q[8];
        const float wv = out[1000];
        const double dw = out[1001];
        const int lane = threadIdx.x & 63;
        for (int i = 0; i < 8; ++i) {
            v[i] = threadIdx.x * (i + 1) * 1e-3f;
            u[i] = threadIdx.x * 7u + i;
            iv[i] = threadIdx.x - i;
            d[i] = v[i];
            p[i] = f32x2{v[i], -v[i]};
            q[i] = f32x4{v[i], 0.f, 0.f, 0.f};
        }
        t0 = clock64();
        // 64 instructions per iteration (32 for f64, 16 LDS ops)
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 64; ++k) {
                if (KIND == 0) v[k & 7] = __builtin_fmaf(v[k & 7], wv, 0.5f);  // v_fma_f32
                if (KIND == 1) p[k & 7] = __builtin_elementwise_fma(p[k & 7], f32x2{wv, wv}, p[(k + 1) & 7]);  // v_pk_fma_f32
                if (KIND == 2) v[k & 7] = __builtin_amdgcn_fmed3f(v[k & 7], 0.f, __builtin_inff());  // v_med3_f32
                if (KIND == 3 && (k & 1) == 0) {  // v_permlane32_swap (32 per iteration, 2 registers each)
                    auto r = __builtin_amdgcn_permlane32_swap(u[k & 7], u[(k + 1) & 7], false, false);
                    u[k & 7] = r[0];
                    u[(k + 1) & 7] = r[1];
                }
                if (KIND == 4 && (k & 1) == 0) {  // v_permlane16_swap
                    auto r = __builtin_amdgcn_permlane16_swap(u[k & 7], u[(k + 1) & 7], false, false);
                    u[k & 7] = r[0];
                    u[(k + 1) & 7] = r[1];
                }
                if (KIND == 5 && k < 32) d[k & 7] = __builtin_fma(d[k & 7], dw, dw);  // v_fma_f64
                if (KIND == 6) iv[k & 7] = iv[k & 7] + iv[(k + 3) & 7];                // v_add_u32
                if (KIND == 7 && k < 16) q[k & 7] += lds[(lane * 8 + k + it) & 511];   // ds_read_b128 (+4 v_add)
                if (KIND == 8 && k < 16)
                    u[k & 7] = __builtin_amdgcn_ds_bpermute((int)((lane ^ (k + 1)) << 2), (int)u[k & 7]);  // ds_bpermute
                if (KIND == 9) v[k & 7] = __builtin_fmaf(v[k & 7], wv, v[(k + 7) & 7]);  // dependent f32 fma chain-ish
            }
        }
        t1 = clock64();
        for (int i = 0; i < 8; ++i) s += v[i] + (float)u[i] + (float)iv[i] + (float)d[i] + p[i][0] + p[i][1] + q[i][0];
    }
    out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[w] = t1 - t0;
}

template <int KIND>
void run(const char* name, int nins, float* out, long long* cyc) {
    const int iters = 4096;
    long long c[8];
    double mf[3] = {0, 0, 0}, vv[3] = {0, 0, 0};
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL((k_xwave3<KIND>), dim3(1), dim3(512), 0, 0, out, iters, mode, cyc);
        hipLaunchKernelGGL((k_xwave3<KIND>), dim3(1), dim3(512), 0, 0, out, iters, mode, cyc);
        hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        for (int w = 0; w < 4; ++w) mf[mode] += (double)c[w] / iters / 4;
        for (int w = 4; w < 8; ++w) vv[mode] += (double)c[w] / iters / 4;
    }
    printf("%-18s | alone %6.1f cyc/iter (%5.2f per instr) | beside MFMA %6.1f (%5.2f per instr)"
           " | MFMA alone %6.1f (%5.2f per mfma), beside it %6.1f\n",
           name, vv[2], vv[2] / nins, vv[0], vv[0] / nins, mf[1], mf[1] / 8, mf[0]);
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 1 << 20);
    hipMemset(out, 0, 1 << 20);
    hipMalloc(&cyc, 64);
    run<0>("v_fma_f32", 64, out, cyc);
    run<1>("v_pk_fma_f32", 64, out, cyc);
    run<2>("v_med3_f32", 64, out, cyc);
    run<3>("v_permlane32_swap", 32, out, cyc);
    run<4>("v_permlane16_swap", 32, out, cyc);
    run<5>("v_fma_f64", 32, out, cyc);
    run<6>("v_add_u32", 64, out, cyc);
    run<7>("ds_read_b128+4add", 16, out, cyc);
    run<8>("ds_bpermute", 16, out, cyc);
    run<9>("v_fma_f32 dep8", 64, out, cyc);
    return 0;
}
