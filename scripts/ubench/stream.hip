// Achievable-bandwidth reference for the fine sweep's traffic pattern: y = x + c*f over three 1.1 GB
// FP64 arrays (2 reads + 1 write, 16 B per lane), plus read-only and write-only streams.
// Reports GB/s of algorithmic bytes for several launch shapes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void __launch_bounds__(256) k_triad(const double2* __restrict__ x, const double2* __restrict__ f,
                                               double2* __restrict__ y, long long n2, int per_thread) {
    long long i = ((long long)blockIdx.x * 256 + threadIdx.x);
    const long long stride = (long long)gridDim.x * 256;
    for (; i < n2; i += stride) {
        const double2 a = x[i], b = f[i];
        y[i] = make_double2(a.x + 0.5 * b.x, a.y + 0.5 * b.y);
    }
}
__global__ void __launch_bounds__(256) k_triad_nt(const double2* __restrict__ x, const double2* __restrict__ f,
                                                  double2* __restrict__ y, long long n2, int per_thread) {
    long long i = ((long long)blockIdx.x * 256 + threadIdx.x);
    const long long stride = (long long)gridDim.x * 256;
    for (; i < n2; i += stride) {
        const double2 a = x[i], b = f[i];
        double2 r = make_double2(a.x + 0.5 * b.x, a.y + 0.5 * b.y);
        __builtin_nontemporal_store(r.x, &y[i].x);
        __builtin_nontemporal_store(r.y, &y[i].y);
    }
}
__global__ void __launch_bounds__(256) k_read(const double2* __restrict__ x, const double2* __restrict__ f,
                                              double2* __restrict__ y, long long n2, int) {
    long long i = ((long long)blockIdx.x * 256 + threadIdx.x);
    const long long stride = (long long)gridDim.x * 256;
    double s = 0;
    for (; i < n2; i += stride) {
        const double2 a = x[i], b = f[i];
        s += a.x + b.y;
    }
    if (s == 1.2345) y[0].x = s;
}
__global__ void __launch_bounds__(256) k_write(const double2* __restrict__ x, const double2* __restrict__ f,
                                               double2* __restrict__ y, long long n2, int) {
    long long i = ((long long)blockIdx.x * 256 + threadIdx.x);
    const long long stride = (long long)gridDim.x * 256;
    for (; i < n2; i += stride) y[i] = make_double2(1.0, 2.0);
}
typedef void (*K)(const double2*, const double2*, double2*, long long, int);
int main() {
    const long long n = 136853824LL;  // padded 512^3 level vector (doubles)
    const long long n2 = n / 2;
    double2 *x, *f, *y;
    if (hipMalloc(&x, n * 8) || hipMalloc(&f, n * 8) || hipMalloc(&y, n * 8)) { printf("alloc failed\n"); return 1; }
    hipMemset(x, 0, n * 8); hipMemset(f, 0, n * 8); hipMemset(y, 0, n * 8);
    struct { const char* name; K k; double bytes; } ks[] = {
        {"triad 2R+1W", k_triad, 24.0 * n}, {"triad nt-store", k_triad_nt, 24.0 * n},
        {"read 2R", k_read, 16.0 * n}, {"write 1W", k_write, 8.0 * n}};
    int grids[] = {1024, 2048, 4096, 8192, 32768, (int)((n2 + 255) / 256)};
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (auto& kk : ks) {
        for (int g : grids) {
            hipLaunchKernelGGL(kk.k, dim3(g), dim3(256), 0, 0, x, f, y, n2, 0);
            hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kk.k, dim3(g), dim3(256), 0, 0, x, f, y, n2, 0);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
            printf("%-16s grid %7d  %8.3f ms  %7.1f GB/s\n", kk.name, g, ms, kk.bytes / ms / 1e6);
        }
    }
    return 0;
}
