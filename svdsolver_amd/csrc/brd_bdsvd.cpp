// Singular values of an upper bidiagonal matrix (d, e) on the host:
// brd_bdsvd_f64 / brd_bdsvd_f32 (include/brd.h).  SURVEY.md 8(f) rank 2 --
// the step after stage 2 that the reference provides as serial::qrd
// (svd_serial.h:368-422, Demmel & Kahan's implicit zero-shift chase with a
// fixed 1e-6 relative threshold and the `500*n^2` XOR iteration cap,
// svd_serial.h:164).
//
// This is the Golub-Kahan SVD step with a Wilkinson shift (Golub & Van Loan,
// Matrix Computations, Alg. 8.6.1 / 8.6.2), values only: deflate wherever
// |e_i| <= eps (|d_i| + |d_{i+1}|), split off zero diagonals by a Givens
// chase, run shifted QR sweeps on the bottom unreduced block.  Convergence is
// cubic per singular value, so the cost is O(n^2) (about 2 s at n = 8192 on
// one core), against the zero-shift chase's linear convergence; accuracy is
// absolute (|sigma_i - sigma_i^exact| ~ eps sigma_max), the same as the
// stage-1/2 reductions that produce (d, e).  Stage 2's sigma-preserving mode
// (BRD_SIGMA) makes these the singular values of the input matrix.
#include "brd_internal.h"
#include "brd.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>
#include <vector>

namespace {

// c, s, r with [c s; -s c] [f; g] = [r; 0]
template <typename T>
inline void givens(T f, T g, T &c, T &s, T &r) {
    if (g == (T)0) { c = (T)1; s = (T)0; r = f; return; }
    if (f == (T)0) { c = (T)0; s = (T)1; r = g; return; }
    r = std::hypot(f, g);
    c = f / r;
    s = g / r;
}

// One shifted Golub-Kahan step on the unreduced block d[0..m), e[0..m-1), m >= 2.
template <typename T>
void gk_step(T *d, T *e, int m) {
    // Wilkinson shift: the eigenvalue of the trailing 2 x 2 of B^T B closer to its last entry
    const T dm1 = d[m - 2], dm = d[m - 1], em1 = e[m - 2];
    const T em2 = m > 2 ? e[m - 3] : (T)0;
    const T t11 = dm1 * dm1 + em2 * em2, t12 = dm1 * em1, t22 = dm * dm + em1 * em1;
    const T delta = (t11 - t22) / (T)2;
    const T den = delta + std::copysign(std::hypot(delta, t12), delta);
    const T mu = den != (T)0 ? t22 - t12 * t12 / den : t22;
    T y = d[0] * d[0] - mu, z = d[0] * e[0];
    for (int k = 0; k < m - 1; ++k) {
        T c, s, r;
        // right rotation on columns k, k+1: [y z] -> [r 0]
        givens(y, z, c, s, r);
        if (k > 0) e[k - 1] = r;
        T dk = c * d[k] + s * e[k];
        T ek = -s * d[k] + c * e[k];
        const T below = s * d[k + 1];   // B[k+1][k]
        d[k + 1] = c * d[k + 1];
        // left rotation on rows k, k+1: [dk; below] -> [r; 0]
        givens(dk, below, c, s, r);
        d[k] = r;
        e[k] = c * ek + s * d[k + 1];
        d[k + 1] = -s * ek + c * d[k + 1];
        if (k < m - 2) {
            z = s * e[k + 1];           // B[k][k+2]
            e[k + 1] = c * e[k + 1];
            y = e[k];
        }
    }
}

template <typename T>
int bdsvd(const T *d_in, const T *e_in, int n, T *sv) {
    if (!d_in || !sv || (n > 1 && !e_in)) return brd::api_fail(BRD_EINVAL, "d, e or sv is NULL");
    if (n < 1) return brd::api_fail(BRD_EINVAL, "n < 1");
    std::vector<T> d(d_in, d_in + n), e(n > 1 ? n - 1 : 1, (T)0);
    if (n > 1) std::copy(e_in, e_in + n - 1, e.begin());
    const T eps = std::numeric_limits<T>::epsilon();
    T bnorm = 0;
    for (int i = 0; i < n; ++i) {
        if (!std::isfinite(d[i]) || (i + 1 < n && !std::isfinite(e[i])))
            return brd::api_fail(BRD_EINVAL, "d / e hold a non-finite value");
        bnorm = std::max(bnorm, std::fabs(d[i]) + (i + 1 < n ? std::fabs(e[i]) : (T)0));
    }
    // scale to bnorm ~ 1 by a power of two (exact): the shifts and rotations
    // square their arguments, which would leave the exponent range for
    // entries near its ends (LAPACK's dbdsqr scales the same way)
    int ex = 0;
    if (bnorm > (T)0) std::frexp(bnorm, &ex);
    for (int i = 0; i < n; ++i) d[i] = std::ldexp(d[i], -ex);
    for (int i = 0; i + 1 < n; ++i) e[i] = std::ldexp(e[i], -ex);
    bnorm = std::ldexp(bnorm, -ex);
    const T tiny = eps * bnorm;
    long iters = 0;
    const long max_iters = 30L * n + 100;
    int q = n;   // d[q..n) are converged singular values
    while (q > 1) {
        // deflate negligible super-diagonal entries
        for (int i = 0; i < q - 1; ++i)
            if (std::fabs(e[i]) <= eps * (std::fabs(d[i]) + std::fabs(d[i + 1])) || std::fabs(e[i]) <= tiny)
                e[i] = (T)0;
        while (q > 1 && e[q - 2] == (T)0) --q;
        if (q <= 1) break;
        int p = q - 2;   // unreduced block [p, q)
        while (p > 0 && e[p - 1] != (T)0) --p;
        if (++iters > max_iters) return brd::api_fail(BRD_EINVAL, "bidiagonal SVD did not converge");
        // a (numerically) zero diagonal entry splits the block
        int z = -1;
        for (int i = p; i < q; ++i)
            if (std::fabs(d[i]) <= tiny) { z = i; break; }
        if (z >= 0) {
            d[z] = (T)0;
            if (z < q - 1) {   // chase row z's super-diagonal to the right (left rotations)
                T f = e[z];
                e[z] = (T)0;
                for (int j = z + 1; j < q && f != (T)0; ++j) {
                    T c, s, r;
                    givens(d[j], f, c, s, r);
                    d[j] = r;
                    if (j < q - 1) {
                        f = -s * e[j];
                        e[j] = c * e[j];
                    }
                }
            } else {           // last diagonal zero: chase column q-1's entry upward (right rotations)
                T f = e[q - 2];
                e[q - 2] = (T)0;
                for (int k = q - 2; k >= p && f != (T)0; --k) {
                    T c, s, r;
                    givens(d[k], f, c, s, r);
                    d[k] = r;
                    if (k > p) {
                        f = -s * e[k - 1];
                        e[k - 1] = c * e[k - 1];
                    }
                }
            }
            continue;
        }
        gk_step(d.data() + p, e.data() + p, q - p);
    }
    for (int i = 0; i < n; ++i) sv[i] = std::ldexp(std::fabs(d[i]), ex);
    std::sort(sv, sv + n, std::greater<T>());
    return BRD_OK;
}

}  // namespace

extern "C" int brd_bdsvd_f64(const double *d, const double *e, int n, double *sv) { return bdsvd(d, e, n, sv); }
extern "C" int brd_bdsvd_f32(const float *d, const float *e, int n, float *sv) { return bdsvd(d, e, n, sv); }
