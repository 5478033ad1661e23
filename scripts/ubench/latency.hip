// Latency microbenchmark (one workgroup): cycles per link of a dependent chain, measured with the
// shader clock (s_memtime) inside the kernel.
//   fma_f64 chain (1, 2, 4 interleaved chains), add_f64 chain, ds_read_b64 pointer chase,
//   __syncthreads() round trip at 64 / 256 / 1024 threads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N 2048

template <int CH>
__global__ void k_fma(double* out, double a, double b, unsigned long long* cyc) {
    double d[CH];
    for (int c = 0; c < CH; ++c) d[c] = threadIdx.x * 1e-9 + c;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N; ++it)
#pragma unroll
        for (int c = 0; c < CH; ++c) d[c] = __builtin_fma(d[c], a, b);
    asm volatile("" ::"v"(d[0]));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int c = 0; c < CH; ++c) s += d[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_add(double* out, double a, unsigned long long* cyc) {
    double d = threadIdx.x * 1e-9;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N; ++it) d = d + a;
    asm volatile("" ::"v"(d));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = d;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_lds(double* out, unsigned long long* cyc) {
    __shared__ int nxt[1024];
    for (int q = threadIdx.x; q < 1024; q += blockDim.x) nxt[q] = (q + 65) & 1023;
    __syncthreads();
    int p = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N; ++it) p = nxt[p];
    asm volatile("" ::"v"(p));
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = p;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_bar(double* out, unsigned long long* cyc) {
    __shared__ double v[1024];
    v[threadIdx.x] = threadIdx.x;
    __syncthreads();
    double s = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N; ++it) {
        s += v[(threadIdx.x + it) & (blockDim.x - 1)];
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double* out;
    unsigned long long* cyc;
    hipMalloc(&out, 4096 * 8);
    hipMalloc(&cyc, 8);
    unsigned long long h;
    auto rep = [&](const char* what, int links) {
        hipDeviceSynchronize();
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-36s %8.2f cycles per link\n", what, (double)h / links);
    };
    for (int r = 0; r < 2; ++r) {
        k_fma<1><<<1, 64>>>(out, 1.0000001, 1e-9, cyc); rep("fma_f64 1 chain, 1 wave", N);
        k_fma<2><<<1, 64>>>(out, 1.0000001, 1e-9, cyc); rep("fma_f64 2 chains, 1 wave", N);
        k_fma<4><<<1, 64>>>(out, 1.0000001, 1e-9, cyc); rep("fma_f64 4 chains, 1 wave", N);
        k_fma<1><<<1, 256>>>(out, 1.0000001, 1e-9, cyc); rep("fma_f64 1 chain, 4 waves", N);
        k_fma<1><<<1, 1024>>>(out, 1.0000001, 1e-9, cyc); rep("fma_f64 1 chain, 16 waves", N);
        k_add<<<1, 64>>>(out, 1e-9, cyc); rep("add_f64 1 chain, 1 wave", N);
        k_lds<<<1, 64>>>(out, cyc); rep("ds_read_b32 chase, 1 wave", N);
        k_lds<<<1, 1024>>>(out, cyc); rep("ds_read_b32 chase, 16 waves", N);
        k_bar<<<1, 64>>>(out, cyc); rep("lds read + syncthreads, 64 thr", N);
        k_bar<<<1, 256>>>(out, cyc); rep("lds read + syncthreads, 256 thr", N);
        k_bar<<<1, 1024>>>(out, cyc); rep("lds read + syncthreads, 1024 thr", N);
    }
    return 0;
}
