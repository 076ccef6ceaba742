// Stage-2 timeline harness (developer tool; needs the STAMPS=1 library build).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdio>
#include <vector>
#include "brd_internal.h"
namespace brd { hipError_t read_s2stamps(unsigned long long *out, size_t n); hipError_t read_s2acc(unsigned long long *out, size_t n); hipError_t read_s2ev(unsigned long long *out, size_t n); hipError_t reset_s2tt(); hipError_t read_s2tt(void *tt, void *pub, void *npub); }
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
    (void)hipMemset(flags, 0, sizeof(int) * (n + 2));
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    std::vector<unsigned long long> zero((size_t)4096 * 8, 0ull);
    for (int it = 0; it < 2; ++it) {
        (void)hipMemcpy(A, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
        (void)brd::reset_s2tt();
        (void)hipEventRecord(e0);
        (void)brd::launch_band2bd<double>(A, n, n, b, false, getenv("BRD_SIGMA") != nullptr, flags, flags + n + 1, 256, 0);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("stage2 n=%d: %.2f ms\n", n, ms);
        check_err("stage2");
    }
    const int S = argc > 2 ? atoi(argv[2]) : 3, nb = std::min(4096, (n - 1 + S - 1) / S);   // sweeps per bundle of the run
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
    printf("per-bundle cycles (2 runs / 2): compute waves [prev,rows,work] x4 | loader[issue,landed] writer[wait,write]\n");
    for (int beta : {0, 1, 2, 10, 100, 1000, 2000, 3000}) {
        if (beta >= nb) continue;
        const unsigned long long *a = &ac[(size_t)beta * 32];
        printf("%5d ", beta);
        for (int w = 0; w < 4; ++w) printf(" %8llu %8llu %8llu |", a[4 * w] / 2, a[4 * w + 1] / 2, a[4 * w + 2] / 2);
        printf(" %8llu %8llu | %8llu %8llu [issue %llu drain %llu]\n", a[16] / 2, a[17] / 2, a[20] / 2, a[21] / 2, a[22] / 2, a[23] / 2);
    }
    {
        std::vector<unsigned long long> ev((size_t)4096 * 8);
        (void)brd::read_s2ev(ev.data(), ev.size());
        printf("hand-off of row beta*S+300 (us, from the trail's front passing it): writer-published poller-seen loader-loaded lead-uses  | next bundle's t0 lag\n");
        printf("bundle lag (lead task 0 done, us) and lead us/task, averaged over ranges of beta:\n");
        const int rngs[][2] = {{0, 10}, {10, 100}, {100, 500}, {500, 1000}, {1000, 2000}, {2000, 3000}, {3000, 4000}};
        for (auto &rg : rngs) {
            if (rg[1] >= nb) continue;
            double lag = (double)(ev[(size_t)rg[1] * 8 + 5] - ev[(size_t)rg[0] * 8 + 5]) / 100.0 / (rg[1] - rg[0]);
            double tau = 0; int cnt = 0;
            for (int beta = rg[0]; beta < rg[1]; ++beta) {
                const int i = beta * S;
                const int nt = 2 + 2 * ((n - std::min(i + 65, n)) / 32 + 1);
                tau += (double)(ev[(size_t)beta * 8 + 6] - ev[(size_t)beta * 8 + 5]) / 100.0 / nt; ++cnt;
            }
            printf("  beta %4d..%4d: lag %.2f us/bundle, lead %.3f us/task\n", rg[0], rg[1], lag, tau / cnt);
        }
        for (int beta : {1, 2, 3, 10, 100, 500, 1000, 2000, 3000}) {
            if (beta + 1 >= nb) continue;
            const unsigned long long *e0 = &ev[(size_t)beta * 8], *e1 = &ev[(size_t)(beta + 1) * 8];
            auto us = [&](unsigned long long x) { return x ? (double)((long long)(x - e0[0])) / 100.0 : -1.0; };
            printf("%5d  %8.2f %8.2f %8.2f %8.2f\n", beta, us(e0[1]), us(e1[2]), us(e1[3]), us(e1[4]));
        }
    }
    {
        static unsigned long long tt[2][4][520][3], pub[2][3][2048][2];
        static int npub[2][3];
        (void)brd::read_s2tt(tt, pub, npub);
        FILE *f = fopen("gpurun_out/s2tt.bin", "wb");
        if (f) { fwrite(tt, sizeof(tt), 1, f); fwrite(pub, sizeof(pub), 1, f); fwrite(npub, sizeof(npub), 1, f); fclose(f); }
    }
    return 0;
}
