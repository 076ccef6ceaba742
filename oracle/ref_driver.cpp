// TEST INFRASTRUCTURE ONLY.  A thin C-ABI driver around the reference's own
// CPU algorithm headers, compiled from the sources where they lie under
// /root/reference (never copied).  Built by `make -C oracle ref` into
// oracle/_ref/libref.so (git-ignored).  Used to validate the oracle
// restatement on inputs beyond the fixtures and to generate golden vectors
// for the sizes whose fixtures the reference does not ship (1024).
#include "svd_parallel.h"   // csc586::parallel::brd_p1 / brd_p2 (svd_parallel.h:411, :640)
#include <cstring>

template <typename T>
static void to_matrix(const T *a, int n, csc586::Matrix<T> &M) {
    M = csc586::Matrix<T>(a, (size_t)n, (size_t)n);
}

template <typename T>
static void from_matrix(csc586::Matrix<T> &M, T *a, int n) {
    for (int i = 0; i < n; ++i)
        std::memcpy(a + (size_t)i * n, M[i].data(), sizeof(T) * n);
}

template <typename T>
static int p1(T *a, int n, int t) {
    if (t <= 0 || n % t) return -1;
    csc586::Matrix<T> M;
    to_matrix(a, n, M);
    csc586::parallel::brd_p1<T>(M, (size_t)t);
    from_matrix(M, a, n);
    return 0;
}

template <typename T>
static int p2(T *a, int n, int b) {
    csc586::Matrix<T> M;
    to_matrix(a, n, M);
    csc586::parallel::brd_p2<T>(M, (size_t)b);
    from_matrix(M, a, n);
    return 0;
}

extern "C" {
int ref_brd_p1_f32(float *a, int n, int t) { return p1<float>(a, n, t); }
int ref_brd_p1_f64(double *a, int n, int t) { return p1<double>(a, n, t); }
int ref_brd_p2_f32(float *a, int n, int b) { return p2<float>(a, n, b); }
int ref_brd_p2_f64(double *a, int n, int b) { return p2<double>(a, n, b); }
int ref_set_threads(int nt) { omp_set_num_threads(nt); return nt; }
}
