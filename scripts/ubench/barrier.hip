// microbenchmark: cost of s_barrier in a 1024/512/256/64-thread workgroup, and the shader clock
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void kb(unsigned long long* out, int n, double* sink) {
    __shared__ double s[1024];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    unsigned long long w0 = wall_clock64(), c0 = clock64();
    double acc = 0;
    for (int i = 0; i < n; ++i) {
        acc += s[(threadIdx.x + i) & 1023];
        __syncthreads();
    }
    unsigned long long w1 = wall_clock64(), c1 = clock64();
    if (threadIdx.x == 0) { out[0] = w1 - w0; out[1] = c1 - c0; }
    if (acc == 12345.0) sink[threadIdx.x] = acc;
}
__global__ void kfma(unsigned long long* out, int n, double* sink) {
    // dependent f64 fma chain: 27 per iteration
    double a = threadIdx.x * 1e-3, b = 1.0000001;
    unsigned long long w0 = wall_clock64(), c0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int q = 0; q < 27; ++q) a = fma(a, b, 1e-9);
    }
    unsigned long long w1 = wall_clock64(), c1 = clock64();
    if (threadIdx.x == 0) { out[0] = w1 - w0; out[1] = c1 - c0; }
    if (a == 12345.0) sink[threadIdx.x] = a;
}
int main() {
    unsigned long long *d, h[2];
    double* sink;
    hipMalloc(&d, 16);
    hipMalloc(&sink, 8192);
    int rate = 0;
    hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);  // kHz
    const int n = 10000;
    for (int nt : {1024, 512, 256, 64}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kb, dim3(1), dim3(nt), 0, 0, d, n, sink);
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        }
        double us = h[0] * 1e3 / rate;
        printf("barrier nt=%4d: %.3f us per iteration, %.1f clock64 ticks per iteration, clock %.2f GHz\n", nt,
               us / n, (double)h[1] / n, h[1] / (us * 1e3));
    }
    for (int nt : {1024, 64}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(kfma, dim3(1), dim3(nt), 0, 0, d, n, sink);
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        }
        double us = h[0] * 1e3 / rate;
        printf("fma chain nt=%4d: %.3f us per 27 dependent fma, %.1f ticks, %.2f ticks per fma\n", nt, us / n,
               (double)h[1] / n, (double)h[1] / n / 27);
    }
    return 0;
}
