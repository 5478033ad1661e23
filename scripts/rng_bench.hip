// Throughput of the noise building blocks on gfx950 (tuning experiment, not product code).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "philox_normal.h"
using namespace mgmc;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
// Threefry-4x32 (Random123 rotation constants)
template <int ROUNDS>
__device__ __forceinline__ Philox4 threefry4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    const uint32_t k2 = 0, k3 = 0, k4 = 0x1BD11BDA ^ k0 ^ k1 ^ k2 ^ k3;
    const uint32_t ks[5] = {k0, k1, k2, k3, k4};
    const int R0[8] = {10, 11, 13, 23, 6, 17, 25, 18}, R1[8] = {26, 21, 27, 5, 20, 11, 10, 20};
    uint32_t x0 = c0 + k0, x1 = c1 + k1, x2 = c2 + k2, x3 = c3 + k3;
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
        if (r & 1) { x0 += x3; x3 = rotl(x3, R0[r & 7]); x3 ^= x0; x2 += x1; x1 = rotl(x1, R1[r & 7]); x1 ^= x2; }
        else { x0 += x1; x1 = rotl(x1, R0[r & 7]); x1 ^= x0; x2 += x3; x3 = rotl(x3, R1[r & 7]); x3 ^= x2; }
        if ((r & 3) == 3) { const int s = (r + 1) / 4; x0 += ks[s % 5]; x1 += ks[(s + 1) % 5]; x2 += ks[(s + 2) % 5]; x3 += ks[(s + 3) % 5] + s; }
    }
    Philox4 o; o.v[0] = x0; o.v[1] = x1; o.v[2] = x2; o.v[3] = x3; return o;
}

template <int KIND>
__global__ void k(double* out, int iters, uint32_t key) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0.0;
    uint32_t h = 0;
    for (int it = 0; it < iters; ++it) {
        Philox4 r;
        if (KIND == 0 || KIND == 3) r = philox4x32_10(t, it, 7, 0, key, key * 3);
        else if (KIND == 1) r = threefry4x32<20>(t, it, 7, 0, key, key * 3);
        else if (KIND == 2) r = threefry4x32<13>(t, it, 7, 0, key, key * 3);
        else { r.v[0] = t * 0x9E3779B9u + it; r.v[1] = r.v[0] ^ key; r.v[2] = r.v[0] + 12345u; r.v[3] = r.v[1] * 3u; }
        if (KIND == 3) { h ^= r.v[0] ^ r.v[1] ^ r.v[2] ^ r.v[3]; continue; }
        double z0, z1;
        normal_pair(r, &z0, &z1);
        acc += z0 + z1;
    }
    out[t] = acc + (double)h;
}

int main() {
    const int nb = 256 * 32, nt = 256, iters = 200;
    double* d;
    hipMalloc(&d, sizeof(double) * nb * nt);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[5] = {"philox10+BM", "threefry20+BM", "threefry13+BM", "philox10 only", "BM only (cheap hash)"};
    for (int kind = 0; kind < 5; ++kind) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            switch (kind) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(nb), dim3(nt), 0, 0, d, iters, 99u); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(nb), dim3(nt), 0, 0, d, iters, 99u); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(nb), dim3(nt), 0, 0, d, iters, 99u); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(nb), dim3(nt), 0, 0, d, iters, 99u); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(nb), dim3(nt), 0, 0, d, iters, 99u); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double calls = (double)nb * nt * iters;
            if (rep) printf("%-22s %8.3f ms  %7.2f G calls/s  -> %.3f ms per 66.7M calls (one 512^3 sweep)\n", names[kind], ms,
                            calls / ms / 1e6, 66.7e6 / (calls / ms));
        }
    }
    return 0;
}
