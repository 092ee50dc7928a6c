// Microbenchmark: does vector f32 work overlap v_mfma_f32_16x16x4_f32 on gfx950?
// One wave alone (1 block of 64 threads) and 2/4 waves on one CU; cycles per
// loop iteration of  NM MFMAs (8 independent accumulators) + NV vector ops,
// interleaved one MFMA then NV/NM vector ops (sched_group_barrier).
// Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NM, int NV, int KIND>
__global__ void k_mix(float* out, int iters, long long* cyc) {
    f32x4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float a = threadIdx.x * 1e-3f, b = 1.0f - a;
    float v[8];
    double d[8];
    int iv[8];
    for (int i = 0; i < 8; ++i) { v[i] = a * (i + 1); d[i] = b * (i + 2); iv[i] = threadIdx.x * (i + 3) - 100; }
    const float w = out[64];
    const double dw = (double)out[65];
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < NM; ++m) acc[m & 7] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 7], 0, 0, 0);
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            if (KIND == 0) v[k & 7] = __builtin_fmaf(v[k & 7], w, a);
            if (KIND == 1) iv[k & 7] = max(iv[k & 7] ^ (int)it, 0);
            if (KIND == 2) d[k & 7] = d[k & 7] * dw + dw;
        }
        if constexpr (NM > 0 && NV > 0) {
            constexpr int PER = NV / (NM > 0 ? NM : 1);
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x2, PER, 0);
            }
        }
    }
    long long t1 = clock64();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3] + v[i] + (float)d[i] + (float)iv[i];
    out[threadIdx.x + blockIdx.x * blockDim.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int NM, int NV, int KIND>
void run(const char* name, float* out, long long* cyc, int threads) {
    const int iters = 4096;
    hipLaunchKernelGGL((k_mix<NM, NV, KIND>), dim3(1), dim3(threads), 0, 0, out, iters, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((k_mix<NM, NV, KIND>), dim3(1), dim3(threads), 0, 0, out, iters, cyc);
    long long c;
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-34s waves/CU=%d  %8.1f cyc/iter  (%5.2f per MFMA, %5.2f per vector op)\n", name, threads / 64,
           (double)c / iters, NM ? (double)c / iters / NM : 0.0, NV ? (double)c / iters / NV : 0.0);
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 1 << 20);
    hipMemset(out, 0, 1 << 20);
    hipMalloc(&cyc, 8);
    for (int th : {64, 256, 512}) {
        run<8, 0, 0>("8 mfma", out, cyc, th);
        run<0, 48, 0>("48 v_fma_f32", out, cyc, th);
        run<8, 16, 0>("8 mfma + 16 v_fma_f32", out, cyc, th);
        run<8, 32, 0>("8 mfma + 32 v_fma_f32", out, cyc, th);
        run<8, 48, 0>("8 mfma + 48 v_fma_f32", out, cyc, th);
        run<0, 48, 1>("48 xor+max_i32", out, cyc, th);
        run<8, 48, 1>("8 mfma + 48 xor+max_i32", out, cyc, th);
        run<0, 16, 2>("16 f64 mul+add", out, cyc, th);
        run<8, 16, 2>("8 mfma + 16 f64 mul+add", out, cyc, th);
    }
    return 0;
}
