// Do kernels on different HIP streams overlap?  A one-workgroup kernel that
// spins ~N us, launched on S streams (eager, then as S captured graphs).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void spin(long long cycles, int* out) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}
int main() {
    int* d;
    hipMalloc(&d, 4096);
    hipStream_t st[8];
    for (int i = 0; i < 8; ++i) hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
    const long long cyc = 100LL * 1000 * 100;  // ~100 ms at 100 MHz? clock64 = shader clock
    for (int S : {1, 2, 4, 8}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < S; ++i) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st[i], cyc, d);
            hipDeviceSynchronize();
            double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            printf("eager S=%d: %.2f ms\n", S, ms);
        }
        hipGraphExec_t ge[8];
        for (int i = 0; i < S; ++i) {
            hipGraph_t g;
            hipStreamBeginCapture(st[i], hipStreamCaptureModeThreadLocal);
            for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, st[i], cyc / 4, d);
            hipStreamEndCapture(st[i], &g);
            hipGraphInstantiate(&ge[i], g, nullptr, nullptr, 0);
        }
        for (int rep = 0; rep < 2; ++rep) {
            hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < S; ++i) hipGraphLaunch(ge[i], st[i]);
            hipDeviceSynchronize();
            double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            printf("graph S=%d: %.2f ms\n", S, ms);
        }
    }
    return 0;
}
