// Dependent-launch cost on one stream (developer tool):
// a chain of N launches of a kernel that does (almost) nothing, per variant:
//   plain      64 threads, no LDS
//   lds138k    256 threads, 138 KB static LDS (the panel-QR kernels' CqrLds)
//   lds64k     512 threads, 64 KB LDS (the read passes' block)
//   wide       grid of 256 workgroups x 256 threads, no LDS
//   dirty<MB>  the predecessor writes <MB> MB (plain stores), then an empty
//              dependent kernel: the boundary's write-back of dirty L2 lines
// Prints us per launch (hipEvent over the chain / N) for each variant.
// Build: hipcc --offload-arch=gfx950 -O3 tools/launch_gap.hip -o tools/launch_gap
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_plain(int *p) { if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1; }
__global__ void __launch_bounds__(256) k_lds138(int *p) {
    __shared__ double s[138 * 1024 / 8];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0 && p[0] == 12345) p[1] = (int)s[5];
}
__global__ void __launch_bounds__(512) k_lds64(int *p) {
    __shared__ double s[8192];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0 && p[0] == 12345) p[1] = (int)s[5];
}
__global__ void k_write(double *d, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) d[i] = (double)i;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 400;
    int *p;
    double *d;
    const long maxmb = 64;
    CK(hipMalloc(&p, 64));
    CK(hipMemset(p, 0, 64));
    CK(hipMalloc(&d, maxmb << 20));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 20; ++i) launch();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        for (int i = 0; i < N; ++i) launch();
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-12s %8.2f us per launch\n", name, ms * 1e3f / N);
    };
    run("plain", [&] { hipLaunchKernelGGL(k_plain, dim3(1), dim3(64), 0, s, p); });
    run("wide", [&] { hipLaunchKernelGGL(k_plain, dim3(256), dim3(256), 0, s, p); });
    run("lds138k", [&] { hipLaunchKernelGGL(k_lds138, dim3(32), dim3(256), 0, s, p); });
    run("lds64k", [&] { hipLaunchKernelGGL(k_lds64, dim3(256), dim3(512), 0, s, p); });
    for (long mb : {1L, 4L, 16L}) {
        // the pair (write mb MB, then an empty dependent kernel) minus the write alone
        char nm[32];
        snprintf(nm, sizeof nm, "write%ldMB", mb);
        const long n = (mb << 20) / 8;
        run(nm, [&] { hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, s, d, n); });
        snprintf(nm, sizeof nm, "+empty", mb);
        run(nm, [&] {
            hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, s, d, n);
            hipLaunchKernelGGL(k_plain, dim3(1), dim3(64), 0, s, p);
        });
    }
    return 0;
}
