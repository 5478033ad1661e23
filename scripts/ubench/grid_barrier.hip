// microbenchmark: cost of a device-wide barrier between phases of one persistent launch (VERDICT r5
// #3: one occupancy-sized launch for levels 2-4 instead of ~20 launches).  G co-resident workgroups
// (one or two per CU) run N phases; each phase: every thread writes one double (the phase's "work"),
// __syncthreads, one lane releases (agent fence), adds to a counter (agent-scope atomic), polls it until
// all G arrived (bounded: a poll count limit sets an error flag and leaves, so the grid always drains),
// acquires (agent fence), __syncthreads.  Reported: microseconds per phase, against an empty launch in a
// graph of N launches.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) k_phases(unsigned* count, int* err, double* buf, int nphase, int G) {
    const int tid = threadIdx.x;
    for (int p = 0; p < nphase; ++p) {
        buf[((size_t)p % 8) * G * 256 + blockIdx.x * 256 + tid] = p + tid;  // the phase's stores
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(count + (tid & 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)G * (unsigned)(p + 1);
            long polls = 0;
            while (__hip_atomic_load(count + (tid & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++polls > 20000000L) {  // ~seconds: give up, record it, leave
                    atomicOr(err, 1);
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
}

__global__ void __launch_bounds__(256) k_empty(double* buf, int G) {
    buf[blockIdx.x * 256 + threadIdx.x] = threadIdx.x;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned* count;
    int* err;
    double* buf;
    hipMalloc(&count, 64);
    hipMalloc(&err, 4);
    hipMalloc(&buf, (size_t)8 * 2 * ncu * 256 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int N = 2000;
    for (int per : {1, 2}) {
        const int G = per * ncu;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(count, 0, 64);
            hipMemset(err, 0, 4);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_phases, dim3(G), dim3(256), 0, 0, count, err, buf, N, G);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            int h_err = 0;
            hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost);
            printf("grid barrier: %d workgroups (%d per CU), %d phases: %.3f us per phase%s\n", G, per, N,
                   ms * 1e3 / N, h_err ? "  (POLL LIMIT HIT)" : "");
        }
    }
    // the alternative: N dependent launches of a small kernel captured in one graph
    hipStream_t s;
    hipStreamCreate(&s);
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int p = 0; p < 200; ++p) hipLaunchKernelGGL(k_empty, dim3(ncu), dim3(256), 0, s, buf, ncu);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0, s);
        hipGraphLaunch(ge, s);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("graph of 200 small launches (%d workgroups each): %.3f us per launch\n", ncu, ms * 1e3 / 200);
    }
    return 0;
}
