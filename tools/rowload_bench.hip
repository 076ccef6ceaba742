// One wave streams N band rows (P doubles each, row stride lda) from HBM into
// an LDS ring, 32 rows per batch, waiting for each batch (the stage-2 loader
// pattern).  Reports cycles per row for several load forms (developer tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
constexpr int P = 96, RING = 192, BATCH = 32;
typedef __attribute__((address_space(3))) void lds_void;

template <int MODE>
__global__ void __launch_bounds__(64) k(const double *A, long lda, int n, unsigned long long *cyc, double *sink) {
    __shared__ __align__(16) double ring[RING * P];
    const int lane = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r0 = 0; r0 < n; r0 += BATCH) {
        for (int r = r0; r < r0 + BATCH; ++r) {
            double *dst = ring + (r % RING) * P;
            const double *src = A + (long)r * lda + r;
            if constexpr (MODE == 0 || MODE == 1) {          // glds dword (sc1 / default)
#pragma unroll
                for (int k = 0; k < P * 2; k += 64)
                    if (k + lane < P * 2)
                        __builtin_amdgcn_global_load_lds((const void *)((const char *)src + 4 * (k + lane)),
                                                         (lds_void *)((char *)dst + 4 * k), 4, 0, MODE == 0 ? 16 : 0);
            } else if constexpr (MODE == 2 || MODE == 3) {   // glds dwordx4 (16 B per lane)
                if (lane < P / 2)
                    __builtin_amdgcn_global_load_lds((const void *)((const char *)src + 16 * lane),
                                                     (lds_void *)dst, 16, 0, MODE == 2 ? 16 : 0);
            }
        }
        if constexpr (MODE == 4 || MODE == 5) {              // registers, dwordx2 sc1 / default
            double v[BATCH][2];
#pragma unroll
            for (int rr = 0; rr < BATCH; ++rr) {
                const double *src = A + (long)(r0 + rr) * lda + r0 + rr;
                if constexpr (MODE == 4) {
                    v[rr][0] = __hip_atomic_load(src + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    v[rr][1] = lane < P - 64 ? __hip_atomic_load(src + 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
                } else {
                    v[rr][0] = src[lane];
                    v[rr][1] = lane < P - 64 ? src[64 + lane] : 0.0;
                }
            }
#pragma unroll
            for (int rr = 0; rr < BATCH; ++rr) {
                double *dst = ring + ((r0 + rr) % RING) * P;
                dst[lane] = v[rr][0];
                if (lane < P - 64) dst[64 + lane] = v[rr][1];
            }
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    double s = 0;
    for (int i = lane; i < RING * P; i += 64) s += ring[i];
    if (s == 12345.678) sink[0] = s;
}

int main() {
    const int n = 8192; const long lda = n + 64;
    double *A, *sink; unsigned long long *cyc;
    (void)hipMalloc(&A, sizeof(double) * lda * (n + 64)); (void)hipMalloc(&sink, 8); (void)hipMalloc(&cyc, 8 * 64);
    (void)hipMemset(A, 0, sizeof(double) * lda * (n + 64));
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const char *names[] = {"glds dword sc1", "glds dword", "glds x4 sc1", "glds x4", "reg x2 sc1", "reg x2"};
    for (int mode = 0; mode < 6; ++mode)
        for (int it = 0; it < 2; ++it) {
            (void)hipEventRecord(e0);
            switch (mode) {
                case 0: k<0><<<1, 64>>>(A, lda, n, cyc, sink); break;
                case 1: k<1><<<1, 64>>>(A, lda, n, cyc, sink); break;
                case 2: k<2><<<1, 64>>>(A, lda, n, cyc, sink); break;
                case 3: k<3><<<1, 64>>>(A, lda, n, cyc, sink); break;
                case 4: k<4><<<1, 64>>>(A, lda, n, cyc, sink); break;
                case 5: k<5><<<1, 64>>>(A, lda, n, cyc, sink); break;
            }
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%-16s it%d: %.3f ms  %.0f cyc/row  %.1f GB/s (%s)\n", names[mode], it, ms, (double)c / n,
                   n * P * 8.0 / (ms * 1e-3) / 1e9, hipGetErrorString(hipGetLastError()));
        }
    return 0;
}
