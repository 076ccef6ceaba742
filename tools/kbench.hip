// Kernel micro-benchmark for the stage-1 trailing update (developer tool).
// Times launch_apply of tree level 0 (the whole N x (N-b) trailing matrix,
// the dominant stage-1 launch shape) for both views and prints the per-phase
// cycle split of workgroup (0,0), wave 0 (stamp build).
// Build: make -C tools kbench ; run: tools/kbench [n=8192] [f64|f32] [target=256] [ncols=n-32] [ld=n]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "brd_internal.h"
namespace brd {
// the stamp build of the library defines this; the plain build gets zeros
__attribute__((weak)) hipError_t read_stamps(unsigned long long *out) {
    memset(out, 0, 64 * sizeof(unsigned long long));
    return hipSuccess;
}
}
using namespace brd;

static void check_err(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e)); exit(3); }
}

template <typename T>
static void run(int n, int target, int ncols, long ld) {
    const int b = 32;
    T *A;
    hipMalloc(&A, sizeof(T) * (size_t)n * ld);
    std::vector<T> h((size_t)n * ld);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (T)((double)((i * 2654435761u) % 1000) / 200.0);
    hipMemcpy(A, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice);
    Tree t = make_tree(n, b);
    void *ws;
    hipMalloc(&ws, tree_ws_bytes(t, sizeof(T)));
    hipMemset(ws, 0, tree_ws_bytes(t, sizeof(T)));
    TreeWs w;
    tree_ws_carve(t, sizeof(T), ws, w);
    launch_factor<T>(false, A, ld, t, 0, w, 0);   // real V / T for level 0
    hipDeviceSynchronize();
    check_err("factor");
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int trans = 0; trans < 2; ++trans)
        for (int lvl = 0; lvl < t.nlevels; ++lvl)
            for (int it = 0; it < 3; ++it) {
                hipEventRecord(e0);
                launch_factor<T>(trans, A, ld, t, lvl, w, 0);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                check_err("factor");
                unsigned long long st[64];
                read_stamps(st);
                printf("%s factor trans=%d level=%d groups=%d: %.1f us | stamps(cyc) init %llu load %llu pub0 %llu "
                       "loop %llu T %llu out %llu | per-column phases vload/dot/upd/pub/bar %llu %llu %llu %llu %llu\n",
                       sizeof(T) == 8 ? "f64" : "f32", trans, lvl, t.lv[lvl].groups, ms * 1e3, st[1] - st[0],
                       st[2] - st[1], st[3] - st[2], st[4] - st[3], st[5] - st[4], st[6] - st[5], st[10], st[11],
                       st[12], st[13], st[14]);
            }
    launch_factor<T>(false, A, ld, t, 0, w, 0);
    hipDeviceSynchronize();
    for (int trans = 0; trans < 2; ++trans) {
        for (int it = 0; it < 4; ++it) {
            hipEventRecord(e0);
            launch_apply<T>(trans, A, ld, t, 0, ncols, w, 0, target, nullptr, 0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            check_err("apply");
            unsigned long long st[64];
            read_stamps(st);
            const double fl = 4.0 * b * n * (double)ncols;
            printf("%s apply ld=%ld trans=%d M=%d ncols=%d target=%d: %.1f us %.1f TF/s %.0f GB/s | phases(cyc) pre %llu "
                   "W %llu red %llu upd %llu store %llu next %llu\n",
                   sizeof(T) == 8 ? "f64" : "f32", ld, trans, n, ncols, target, ms * 1e3, fl / (ms * 1e-3) / 1e12,
                   2.0 * sizeof(T) * n * (double)ncols / (ms * 1e-3) / 1e9, st[20], st[21], st[22], st[23], st[24],
                   st[25]);
            memset(st, 0, sizeof(st));
        }
    }
    hipFree(ws);
    hipFree(A);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 8192;
    const bool f32 = argc > 2 && !strcmp(argv[2], "f32");
    const int target = argc > 3 ? atoi(argv[3]) : 256;
    const int ncols = argc > 4 ? atoi(argv[4]) : n - 32;
    const long ld = argc > 5 ? atol(argv[5]) : n;
    if (f32) run<float>(n, target, ncols, ld);
    else run<double>(n, target, ncols, ld);
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
