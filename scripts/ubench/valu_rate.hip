// VALU issue-rate microbenchmark: N independent chains of one instruction class per lane, full
// occupancy; reports wave-instruction issue cost in cycles per SIMD (clock from s_memrealtime is
// the 100 MHz constant clock -> we use wall time and the reported shader clock instead).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 4096
#define CH 8
template <int K>
__global__ void __launch_bounds__(256) kern(double* out, uint32_t seed) {
    uint32_t a[CH];
    double d[CH];
    uint64_t q[CH];
    for (int c = 0; c < CH; ++c) { a[c] = seed + threadIdx.x * 7 + c; d[c] = 1.0 + a[c] * 1e-9; q[c] = a[c]; }
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if (K == 0) d[c] = __builtin_fma(d[c], 1.0000001, 1e-9);                         // v_fma_f64
            if (K == 1) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[c]) : "v"(a[c]), "v"(0xD2511F53u) : "vcc");
            if (K == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(0xD2511F53u));
            if (K == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(0xD2511F53u));
            if (K == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(seed));
            if (K == 5) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[c]));
            if (K == 6) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[c]) : "v"(d[(c + 1) % CH]));
            if (K == 7) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[c]) : "v"(d[(c + 1) % CH]));
            if (K == 8) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[c]) : "v"(a[c]));
            if (K == 9) asm volatile("v_mov_b64 %0, %1" : "=v"(d[c]) : "v"(d[(c + 1) % CH]));
            if (K == 10) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[c]) : "v"(a[c]));
            if (K == 11) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(seed));
            if (K == 12) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(q[c]) : "v"(q[(c + 1) % CH]));
            if (K == 13) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(seed));
            if (K == 14) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[c]));
            if (K == 15) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[c]));
            if (K == 16) asm volatile("v_fract_f64 %0, %0" : "+v"(d[c]));
            if (K == 17) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q[c]) : "v"(q[(c + 1) % CH]));
        }
    }
    double s = 0;
    for (int c = 0; c < CH; ++c) s += d[c] + (double)a[c] + (double)q[c];
    if (s == 12345.678) out[threadIdx.x] = s;
}
const char* names[] = {"v_fma_f64", "v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_xor_b32", "v_rsq_f64",
                       "v_mul_f64", "v_add_f64", "v_ldexp_f64", "v_mov_b64", "v_cvt_f64_i32", "v_fma_f32",
                       "v_pk_fma_f32", "v_cndmask_b32", "v_sqrt_f64", "v_rcp_f64", "v_fract_f64", "v_lshl_add_u64"};
template <int K>
void run(double* out, int clk_khz, int ncu) {
    const int blocks = ncu * 8;  // 32 waves per CU
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    kern<K><<<blocks, 256>>>(out, 1);
    hipEventRecord(e0);
    kern<K><<<blocks, 256>>>(out, 1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr_per_simd = (double)blocks * 4 * ITER * CH / (ncu * 4.0);
    const double cycles = ms * 1e-3 * clk_khz * 1e3;
    printf("%-16s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (at %d MHz)\n", names[K], ms, cycles / wave_instr_per_simd, clk_khz / 1000);
}
int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    double* out; hipMalloc(&out, 4096 * 8);
    int clk = p.clockRate;  // kHz
    printf("CUs %d clock %d MHz\n", p.multiProcessorCount, clk / 1000);
    run<0>(out, clk, p.multiProcessorCount); run<1>(out, clk, p.multiProcessorCount); run<2>(out, clk, p.multiProcessorCount);
    run<3>(out, clk, p.multiProcessorCount); run<4>(out, clk, p.multiProcessorCount); run<5>(out, clk, p.multiProcessorCount);
    run<6>(out, clk, p.multiProcessorCount); run<7>(out, clk, p.multiProcessorCount); run<8>(out, clk, p.multiProcessorCount);
    run<9>(out, clk, p.multiProcessorCount); run<10>(out, clk, p.multiProcessorCount); run<11>(out, clk, p.multiProcessorCount);
    run<12>(out, clk, p.multiProcessorCount); run<13>(out, clk, p.multiProcessorCount); run<14>(out, clk, p.multiProcessorCount);
    run<15>(out, clk, p.multiProcessorCount); run<16>(out, clk, p.multiProcessorCount); run<17>(out, clk, p.multiProcessorCount);
    return 0;
}
