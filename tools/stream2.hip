// Flat streaming probe (developer tool): in-place read-modify-write vs
// out-of-place copy vs read-only over an N x N fp64 matrix, 16 B per lane per
// access, each workgroup sweeping one contiguous chunk with UNR accesses in
// flight per lane.  Question answered: is the ~4 TB/s the stage-1 update
// reaches (tools/stream) the in-place ceiling, or would a ping-pong
// (out-of-place) update stream faster?
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int MODE, int UNR>   // 0 in place, 1 copy, 2 read only
__global__ void __launch_bounds__(512) k_flat(const d2 *__restrict__ X, d2 *__restrict__ Y, long n2, double *sink) {
    const long per = (n2 + gridDim.x - 1) / gridDim.x;
    const long beg = blockIdx.x * per, end = beg + per < n2 ? beg + per : n2;
    d2 acc = {0, 0};
    for (long i = beg + threadIdx.x; i < end; i += (long)blockDim.x * UNR) {
        d2 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const long j = i + (long)u * blockDim.x;
            v[u] = j < end ? X[j] : d2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const long j = i + (long)u * blockDim.x;
            if (MODE == 2) acc += v[u];
            else if (j < end) Y[j] = v[u] + 1.0;
        }
    }
    if (MODE == 2 && acc.x == -1.0) sink[0] = acc.y;
}

// The stage-1 apply's assignment (512-row node x run of W-column slabs per
// workgroup), RMW in place, W*8-byte row segments: lanes cover consecutive
// 16-B pieces of a row, 512/(W/2) rows per wave-instruction round.
template <int W>
__global__ void __launch_bounds__(512) k_slab(double *A, long ld, int ncols, int spw) {
    constexpr int LPR = W / 2, RPI = 512 / LPR, ITER = 512 / RPI;   // lanes per row, rows per round
    const int g = blockIdx.x, t = threadIdx.x, r = t / LPR, c = (t % LPR) * 2;
    const int nslabs = ncols / W, s0 = blockIdx.y * spw, s1 = min(nslabs, s0 + spw);
    double *base = A + (long)g * 512 * ld;
    for (int sl = s0; sl < s1; ++sl) {
        d2 v[ITER];
#pragma unroll
        for (int i = 0; i < ITER; ++i) v[i] = *(const d2 *)(base + (long)(r + i * RPI) * ld + sl * W + c);
#pragma unroll
        for (int i = 0; i < ITER; ++i) *(d2 *)(base + (long)(r + i * RPI) * ld + sl * W + c) = v[i] + 1.0;
    }
}

template <int W>
static void run_slab(double *A, int n, int pad = 0) {
    const long ld = n + pad;
    const int groups = n / 512, nslabs = n / W;
    int spw = (groups * nslabs + 255) / 256;
    while (groups * ((nslabs + spw - 1) / spw) > 256) ++spw;
    dim3 grid(groups, (nslabs + spw - 1) / spw);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_slab<W>), grid, dim3(512), 0, 0, A, ld, n, spw);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it > 0 && ms < best) best = ms;
    }
    printf("slab RMW width %3d (%4d-B rows), ld pad %3d, grid %d x %d: %8.1f us  %7.0f GB/s\n", W, W * 8, pad, grid.x, grid.y,
           best * 1e3, 2.0 * n * (double)n * 8 / (best * 1e-3) / 1e9);
}

template <int MODE, int UNR>
static void run(const d2 *X, d2 *Y, long n2, int grid, double *sink, const char *name) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_flat<MODE, UNR>), dim3(grid), dim3(512), 0, 0, X, Y, n2, sink);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it > 0 && ms < best) best = ms;
    }
    const double bytes = (MODE == 2 ? 1.0 : 2.0) * n2 * 16;
    printf("%-24s grid %5d unroll %d: %8.1f us  %7.0f GB/s\n", name, grid, UNR, best * 1e3, bytes / (best * 1e-3) / 1e9);
}

int main() {
    const long n = 8192, n2 = n * n / 2;
    d2 *A, *B;
    double *sink;
    (void)hipMalloc(&A, sizeof(double) * n * n);
    (void)hipMalloc(&B, sizeof(double) * n * n);
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(A, 0, sizeof(double) * n * n);
    (void)hipMemset(B, 0, sizeof(double) * n * n);
    // the slab pattern at n = 8192 with padded leading dimensions (A, B are
    // contiguous 2 x 512 MiB here, so an n x (n + pad) matrix fits in A..B)
    double *P = nullptr;
    (void)hipMalloc(&P, sizeof(double) * n * (n + 256));
    for (int pad : {0, 16, 32, 64, 256}) {
        run_slab<16>(P, (int)n, pad);
        run_slab<32>(P, (int)n, pad);
    }
    run_slab<16>(P, 7680, 0);
    run_slab<16>(P, 4096 + 2048, 0);
    for (int grid : {256}) {
        run<0, 4>(A, A, n2, grid, sink, "in place (RMW)");
        run<1, 4>(A, B, n2, grid, sink, "copy A -> B");
        run<2, 4>(A, B, n2, grid, sink, "read only");
        run<0, 8>(A, A, n2, grid, sink, "in place (RMW)");
        run<1, 8>(A, B, n2, grid, sink, "copy A -> B");
    }
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
