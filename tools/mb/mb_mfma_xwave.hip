// Microbenchmark: do f32 MFMAs of one wave overlap vector f32 work of ANOTHER
// wave on the same SIMD (gfx950)?  One workgroup of 8 waves: waves 0-3 (one
// per SIMD) run an MFMA-only loop, waves 4-7 (the same SIMDs, cyclic wave ->
// SIMD order) a vector-only loop; each wave records its own s_memtime span
// and its SIMD id.  Modes: 0 both loops, 1 MFMA waves only, 2 vector waves only.
// Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ void k_xwave(float* out, int iters, int mode, long long* cyc, unsigned* hw) {
    const int w = threadIdx.x >> 6;
    const bool mf = w < 4;
    unsigned hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    long long t0 = clock64(), t1 = t0;
    float s = 0.f;
    if (mf && mode != 2) {
        f32x4 acc[8];
        for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float a = threadIdx.x * 1e-3f, b = 1.0f - a;
        t0 = clock64();
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int m = 0; m < 8; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m], 0, 0, 0);
        }
        t1 = clock64();
        for (int i = 0; i < 8; ++i) s += acc[i][0];
    } else if (!mf && mode != 1) {
        float v[8];
        int iv[8];
        double d[8];
        const float wv = out[1000];
        const double dw = out[1001];
        for (int i = 0; i < 8; ++i) { v[i] = threadIdx.x * (i + 1) * 1e-3f; iv[i] = threadIdx.x - i; d[i] = v[i]; }
        t0 = clock64();
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 48; ++k) {
                if (KIND == 0) v[k & 7] = __builtin_fmaf(v[k & 7], wv, 0.5f);
                if (KIND == 1) iv[k & 7] = max(iv[k & 7] ^ it, 0);
                if (KIND == 2 && k < 16) d[k & 7] = d[k & 7] * dw + dw;
                if (KIND == 3) v[k & 7] = __builtin_fmaxf(v[k & 7] * wv, 0.0f);
                if (KIND == 4) iv[k & 7] = iv[k & 7] + (it | k);
                if (KIND == 5) iv[k & 7] = max(iv[k & 7] - it, 0);
                if (KIND == 6) iv[k & 7] = (v[k & 7] > wv) ? iv[k & 7] + 1 : iv[(k + 1) & 7];
                if (KIND == 7) v[k & 7] = __builtin_fmaf(v[k & 7], wv, 0.5f) + v[(k + 3) & 7];
            }
        }
        t1 = clock64();
        for (int i = 0; i < 8; ++i) s += v[i] + (float)iv[i] + (float)d[i];
    }
    out[threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        cyc[w] = t1 - t0;
        hw[w] = hwid;
    }
}

template <int KIND>
void run(const char* name, float* out, long long* cyc, unsigned* hw) {
    const int iters = 8192;
    long long c[8];
    unsigned h[8];
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL((k_xwave<KIND>), dim3(1), dim3(512), 0, 0, out, iters, mode, cyc, hw);
        hipLaunchKernelGGL((k_xwave<KIND>), dim3(1), dim3(512), 0, 0, out, iters, mode, cyc, hw);
        hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        hipMemcpy(h, hw, sizeof(h), hipMemcpyDeviceToHost);
        printf("%-22s mode %d  mfma waves (cyc/iter of 8 MFMA):", name, mode);
        for (int w = 0; w < 4; ++w) printf(" %6.1f[simd%u]", (double)c[w] / iters, (h[w] >> 4) & 3);
        printf("   vector waves (cyc/iter):");
        for (int w = 4; w < 8; ++w) printf(" %6.1f[simd%u]", (double)c[w] / iters, (h[w] >> 4) & 3);
        printf("\n");
    }
}

int main() {
    float* out;
    long long* cyc;
    unsigned* hw;
    hipMalloc(&out, 1 << 20);
    hipMemset(out, 0, 1 << 20);
    hipMalloc(&cyc, 64);
    hipMalloc(&hw, 64);
    run<0>("48 v_fma_f32", out, cyc, hw);
    run<1>("48 xor+max_i32", out, cyc, hw);
    run<2>("16 f64 mul+add", out, cyc, hw);
    run<3>("48 mul_f32+max_f32", out, cyc, hw);
    run<4>("48 add_u32 (+or)", out, cyc, hw);
    run<5>("48 sub+max_i32", out, cyc, hw);
    run<6>("48 cmp+cndmask", out, cyc, hw);
    run<7>("48 fma+add f32", out, cyc, hw);
    return 0;
}
