// Microbenchmark: dependent-chain latency of float64 add on gfx950, and the
// cost of feeding a sequential float64 sum from LDS.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void chain_reg(double* out, double a, double b, int n, long long* cyc) {
    double s = a;
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        s += b; s += a; s += b; s += a; s += b; s += a; s += b; s += a;
    }
    long long t1 = clock64();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void chain_fma(double* out, double a, double b, int n, long long* cyc) {
    double s = a;
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
        s = __builtin_fma(1.0, s, b); s = __builtin_fma(1.0, s, a); s = __builtin_fma(1.0, s, b); s = __builtin_fma(1.0, s, a);
        s = __builtin_fma(1.0, s, b); s = __builtin_fma(1.0, s, a); s = __builtin_fma(1.0, s, b); s = __builtin_fma(1.0, s, a);
    }
    long long t1 = clock64();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

// one lane sums an LDS array of n doubles in order
__global__ void chain_lds(const double* in, double* out, int n, long long* cyc) {
    __shared__ double buf[4096];
    for (int i = threadIdx.x; i < n; i += blockDim.x) buf[i] = in[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        long long t0 = clock64();
        for (int i = 0; i < n; i += 8) {
            const double2 x0 = *reinterpret_cast<const double2*>(buf + i);
            const double2 x1 = *reinterpret_cast<const double2*>(buf + i + 2);
            const double2 x2 = *reinterpret_cast<const double2*>(buf + i + 4);
            const double2 x3 = *reinterpret_cast<const double2*>(buf + i + 6);
            s += x0.x; s += x0.y; s += x1.x; s += x1.y; s += x2.x; s += x2.y; s += x3.x; s += x3.y;
        }
        long long t1 = clock64();
        out[0] = s;
        *cyc = t1 - t0;
    }
}

int main() {
    double* out; long long* cyc; double* in;
    hipMalloc(&out, 1024 * sizeof(double)); hipMalloc(&cyc, sizeof(long long)); hipMalloc(&in, 4096 * sizeof(double));
    std::vector<double> h(4096); for (int i = 0; i < 4096; ++i) h[i] = 1e-4 * ((i * 7919) % 101 - 50);
    hipMemcpy(in, h.data(), 4096 * sizeof(double), hipMemcpyHostToDevice);
    long long c; hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms;
    const int n = 4096;  // x8 adds
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0); hipLaunchKernelGGL(chain_reg, 1, 64, 0, 0, out, 1.0000001, -0.9999999, n, cyc); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("v_add_f64 chain: %.2f clock64-ticks/add, %.3f ns/add (event)\n", (double)c / (8.0 * n), ms * 1e6 / (8.0 * n));
        hipEventRecord(e0); hipLaunchKernelGGL(chain_fma, 1, 64, 0, 0, out, 1.0000001, -0.9999999, n, cyc); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("v_fma_f64 chain: %.2f ticks/op, %.3f ns/op\n", (double)c / (8.0 * n), ms * 1e6 / (8.0 * n));
        hipEventRecord(e0); hipLaunchKernelGGL(chain_lds, 1, 256, 0, 0, in, out, 4096, cyc); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1); hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("LDS-fed sum: %.2f ticks/element (kernel %.2f us for 4096)\n", (double)c / 4096.0, ms * 1e3);
    }
    return 0;
}
