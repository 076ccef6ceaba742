// Streaming-bandwidth probe for the stage-1 trailing update's access pattern
// (developer tool): an M x N fp64 row-major matrix, 512 x 16 slabs, one
// workgroup (512 threads) per (512-row node, run of slabs); every lane moves the
// k_apply2 register pattern (4 rows x 16 columns per wave instruction) or a
// row-contiguous pattern, X <- X + 1, with DEPTH slabs of loads in flight.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int DEPTH, bool ROWS, int NT>
__global__ void __launch_bounds__(512) k_stream(double *A, long ld, int ncols, int spw) {
    const int grp = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l15 = lane & 15;
    const int nslabs = ncols / 16, s0 = blockIdx.y * spw, s1 = min(nslabs, s0 + spw);
    double *base = A + (long)grp * 512 * ld;
    double x[DEPTH][16];
    auto addr = [&](int slab, int i) -> double * {
        if (ROWS) {   // thread -> (row tid, 16 consecutive columns): 128 B per lane
            return base + (long)tid * ld + slab * 16 + i;
        } else {      // k_apply2: block jb, register s -> row (w + 8 jb) * 16 + q + 4 s, column l15
            const int jb = i >> 2, s = i & 3;
            return base + (long)((w + 8 * jb) * 16 + q + 4 * s) * ld + slab * 16 + l15;
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[d][i] = s0 + d < s1 ? *addr(s0 + d, i) : 0.0;
    for (int slab = s0; slab < s1; slab += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            if (slab + d < s1) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (NT & 1) __builtin_nontemporal_store(x[d][i] + 1.0, addr(slab + d, i));
                    else *addr(slab + d, i) = x[d][i] + 1.0;
                }
            }
            const int nx = slab + d + DEPTH;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                x[d][i] = nx < s1 ? ((NT & 2) ? __builtin_nontemporal_load(addr(nx, i)) : *addr(nx, i)) : 0.0;
        }
    }
}

template <int DEPTH, bool ROWS, int NT = 0>
static void run(double *A, int M, int N, const char *name) {
    const int groups = M / 512, nslabs = N / 16, spw = (groups * nslabs + 255) / 256;
    dim3 grid(groups, (nslabs + spw - 1) / spw);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int it = 0; it < 3; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_stream<DEPTH, ROWS, NT>), grid, dim3(512), 0, 0, A, (long)N, N, spw);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it == 2) printf("%-28s M=%d N=%d: %8.1f us  %7.0f GB/s (read+write)\n", name, M, N, ms * 1e3,
                            2.0 * M * N * 8 / (ms * 1e-3) / 1e9);
    }
}

int main() {
    for (int n : {8192, 4096}) {
        double *A;
        (void)hipMalloc(&A, sizeof(double) * (size_t)n * n);
        (void)hipMemset(A, 0, sizeof(double) * (size_t)n * n);
        run<1, false>(A, n, n, "apply2 pattern, depth 1");
        run<1, false, 1>(A, n, n, "apply2 pattern, nt stores");
        run<1, false, 2>(A, n, n, "apply2 pattern, nt loads");
        run<1, false, 3>(A, n, n, "apply2 pattern, nt both");
        (void)hipFree(A);
    }
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
