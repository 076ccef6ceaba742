// Stage-2 timeline harness (developer tool; needs the STAMPS=1 library build).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdio>
#include <vector>
#include "brd_internal.h"
namespace brd { hipError_t read_s2stamps(unsigned long long *out, size_t n); hipError_t read_s2acc(unsigned long long *out, size_t n); }
static void check_err(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e)); exit(3); }
}
int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 8192, b = 32;
    double *A; (void)hipMalloc(&A, sizeof(double) * (size_t)n * n);
    std::vector<double> h((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) for (int j = i; j <= std::min(n - 1, i + b); ++j) h[(size_t)i * n + j] = 1.0 + ((i * 31 + j * 17) % 97) / 97.0;
    int *flags; (void)hipMalloc(&flags, sizeof(int) * (n + 2));
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int it = 0; it < 2; ++it) {
        (void)hipMemcpy(A, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
        (void)hipEventRecord(e0);
        (void)brd::launch_band2bd<double>(A, n, n, b, false, flags, flags + n + 1, 256, 0);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("stage2 n=%d: %.2f ms\n", n, ms);
        check_err("stage2");
    }
    const int S = 2, nb = std::min(4096, (n - 1 + S - 1) / S);
    std::vector<unsigned long long> st((size_t)nb * 6);
    (void)brd::read_s2stamps(st.data(), st.size());
    printf("beta   lead_t0   lead_done  trail_done  writer  loader   (cycles after the bundle's start)\n");
    for (int beta : {0, 1, 2, 3, 10, 100, 500, 1000, 2000, 3000, 4000}) {
        if (beta >= nb) continue;
        const unsigned long long *s = &st[(size_t)beta * 6];
        printf("%5d %8lld %10lld %10lld %8lld %8lld\n", beta, (long long)(s[1] - s[0]),
               (long long)(s[2] - s[0]), (long long)(s[3] - s[0]), (long long)(s[4] - s[0]), (long long)(s[5] - s[0]));
    }
    std::vector<unsigned long long> ac((size_t)4096 * 32);
    (void)brd::read_s2acc(ac.data(), ac.size());
    printf("per-bundle cycles (2 runs / 2): w0[prev,rows,work] w1[prev,rows,work] loader[issue,landed] writer[wait,write]\n");
    for (int beta : {0, 1, 2, 10, 100, 1000, 2000, 3000}) {
        if (beta >= nb) continue;
        const unsigned long long *a = &ac[(size_t)beta * 32];
        printf("%5d  %9llu %9llu %9llu | %9llu %9llu %9llu | %9llu %9llu | %9llu %9llu\n", beta, a[0] / 2, a[1] / 2, a[2] / 2,
               a[4] / 2, a[5] / 2, a[6] / 2, a[8] / 2, a[9] / 2, a[12] / 2, a[13] / 2);
    }
    return 0;
}
