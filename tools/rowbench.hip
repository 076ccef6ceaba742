// Band-row read bandwidth probe (developer tool): the stage-2 loader's access
// pattern -- 768-byte rows (the ring slice of a b = 32 fp64 band row) at a
// stride of (lda + 1) * 8 bytes, 16-byte sc1 loads by lanes 0..47, staged into
// LDS.  G workgroups, each with WV loader waves taking rows round-robin; a wave
// keeps D rows in flight (issue D, wait, store them to LDS, repeat).  Prints
// GB/s per workgroup and in total.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int D, bool SC1>
__global__ void k_rows(const double *A, long lda, int rows_per_group, int wv) {
    __shared__ u32x4 lds[4][D][48];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r0 = blockIdx.x * rows_per_group;
    const char *base = (const char *)A;
    const long rstep = (lda + 1) * 8;
    for (int r = r0 + w * D; r < r0 + rows_per_group; r += wv * D) {
        u32x4 v[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const u32x4 *p = (const u32x4 *)(base + (long)(r + i) * rstep) + (lane < 48 ? lane : 0);
            if (SC1) asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[i]) : "v"(p) : "memory");
            else v[i] = *p;
        }
        if (SC1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < D; ++i)
            if (lane < 48) lds[w & 3][i][lane] = v[i];
    }
}

template <int D, bool SC1>
static void run(const double *A, long lda, int G, int rpg, int wv) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int it = 0; it < 4; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_rows<D, SC1>), dim3(G), dim3(64 * wv), 0, 0, A, lda, rpg, wv);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double bytes = (double)G * rpg * 768;
    printf("D=%2d %s waves=%d groups=%3d: %8.1f us  %6.1f GB/s per group  %7.1f GB/s total\n", D,
           SC1 ? "sc1" : "pl ", wv, G, best * 1e3, bytes / G / (best * 1e-3) / 1e9, bytes / (best * 1e-3) / 1e9);
}

int main() {
    const int n = 8192;
    double *A;
    (void)hipMalloc(&A, sizeof(double) * (size_t)n * n);
    (void)hipMemset(A, 0, sizeof(double) * (size_t)n * n);
    const int rpg = 240;
    for (int G : {1, 32}) {
        run<8, false>(A, n, G, rpg, 1);
        run<16, false>(A, n, G, rpg, 1);
        run<24, false>(A, n, G, rpg, 1);
        run<8, false>(A, n, G, rpg, 2);
        run<8, false>(A, n, G, rpg, 3);
        run<16, false>(A, n, G, rpg, 2);
        run<16, true>(A, n, G, rpg, 1);
    }
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
