// Microbenchmark: what a small dependent kernel costs on MI355X.
//   empty kernel (1 block), kernel with N dependent global loads (1 lane),
//   1-block Philox+Box-Muller work; back-to-back launches timed by events.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) { if (threadIdx.x == 1023) p[0] = 1; }

__global__ void k_chase(const int* __restrict__ next, int* out, int n) {
    if (threadIdx.x) return;
    int i = 0;
    for (int k = 0; k < n; ++k) i = next[i];
    out[0] = i;
}

__global__ void k_math(float* out, int iters) {
    float s = threadIdx.x * 1e-3f;
    for (int k = 0; k < iters; ++k) {
        float a, b;
        sincospif(s, &a, &b);
        s = sqrtf(-2.0f * logf(fabsf(a) + 1e-3f)) * b + 1e-3f;
    }
    out[threadIdx.x] = s;
}

int main() {
    int* buf; hipMalloc(&buf, 64 << 20);
    int* next; hipMalloc(&next, 64 << 20);
    // pointer chase through 16 MB with a large stride
    const int N = 4 << 20;
    int* h = new int[N];
    for (int i = 0; i < N; ++i) h[i] = (int)(((long long)i * 7919 + 1234567) % N);
    hipMemcpy(next, h, N * 4, hipMemcpyHostToDevice);
    float* fo; hipMalloc(&fo, 4096 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b); float ms;
    for (int rep = 0; rep < 2; ++rep) {
        const int L = 200;
        hipEventRecord(a);
        for (int i = 0; i < L; ++i) hipLaunchKernelGGL(k_empty, 1, 1024, 0, 0, buf);
        hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
        printf("empty 1x1024 kernel back-to-back: %.2f us each\n", ms * 1e3 / L);
        for (int n : {1, 8, 64}) {
            hipEventRecord(a);
            for (int i = 0; i < L; ++i) hipLaunchKernelGGL(k_chase, 1, 64, 0, 0, next, buf, n);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("chase %2d dependent loads: %.2f us per kernel\n", n, ms * 1e3 / L);
        }
        for (int it : {1, 6, 24}) {
            hipEventRecord(a);
            for (int i = 0; i < L; ++i) hipLaunchKernelGGL(k_math, 1, 1024, 0, 0, fo, it);
            hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
            printf("1 block x1024 math iters %2d: %.2f us per kernel\n", it, ms * 1e3 / L);
        }
    }
    return 0;
}
