// Kernel micro-benchmark for the stage-1 kernels (developer tool).
// Build: make -C svdsolver_amd clean && make -C svdsolver_amd STAMPS=1 && \
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -Isvdsolver_amd/csrc tools/kbench.hip \
//         -Lsvdsolver_amd/lib -lbrd_hip -Wl,-rpath,$PWD/svdsolver_amd/lib -o /tmp/kbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "brd_internal.h"
namespace brd { hipError_t read_stamps(unsigned long long *out); }
using namespace brd;
static void check_err(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e)); exit(3); }
}
int main(int argc, char **argv) {
    int n = argc > 1 ? atoi(argv[1]) : 8192;
    int b = 32;
    double *A; hipMalloc(&A, sizeof(double) * (size_t)n * n);
    std::vector<double> h((size_t)n * n);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 200.0;
    hipMemcpy(A, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
    Tree t = make_tree(n, b);
    void *ws; hipMalloc(&ws, tree_ws_bytes(t, 8));
    TreeWs w; tree_ws_carve(t, 8, ws, w);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int trans = 0; trans < 2; ++trans)
    for (int lvl = 0; lvl < t.nlevels; ++lvl) {
        for (int it = 0; it < 3; ++it) {
            hipEventRecord(e0);
            launch_factor<double>(trans, A, n, t, lvl, w, 0);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            check_err("factor");
            unsigned long long st[64]; read_stamps(st);
            printf("factor trans=%d level=%d groups=%d: %.1f us | stamps(cyc):", trans, lvl, t.lv[lvl].groups, ms * 1e3);
            for (int k = 1; k <= 6; ++k) printf(" %llu", st[k] - st[k - 1]);
            printf(" | loop phases pub/dot/bar/refl/upd:");
            for (int k = 10; k < 15; ++k) printf(" %llu", st[k]);
            printf("\n");
        }
    }
    for (int trans = 0; trans < 2; ++trans) {
        for (int it = 0; it < 3; ++it) {
            hipEventRecord(e0);
            launch_apply<double>(trans, A, n, t, 0, n - b, w, 0);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            check_err("apply");
            double fl = 4.0 * b * n * (double)(n - b);
            printf("apply trans=%d level0 M=%d ncols=%d: %.1f us  %.1f TF/s  %.0f GB/s\n", trans, n, n - b, ms * 1e3,
                   fl / (ms * 1e-3) / 1e12, 16.0 * n * (double)(n - b) / (ms * 1e-3) / 1e9);
        }
    }
    printf("%s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
