// Singular values of an upper bidiagonal matrix on the GPU: multisection on
// the Golub-Kahan tridiagonal.  SURVEY.md 8(f) rank 2 ("bidiagonal -> singular
// values on host/GPU"); the host twin is brd_bdsvd.cpp (Golub-Kahan QR), the
// reference's is serial::qrd (svd_serial.h:368-422).
//
// The bidiagonal B (d[0..n), e[0..n-1)) has the singular values sigma_i; the
// 2n x 2n symmetric tridiagonal T_GK with zero diagonal and off-diagonal
// (d0, e0, d1, e1, ..., e_{n-2}, d_{n-1}) has the eigenvalues +-sigma_i
// (Golub & Kahan 1965; LAPACK dbdsvdx bisects the same matrix).  For x > 0 the
// Sturm count of T_GK - x I (negative pivots of its LDL^T, q_1 = -x,
// q_i = -x - a_{i-1}^2 / q_{i-1}) is n + #{sigma_i < x}, so every singular
// value can be bracketed on its own: value k (ascending) is the x where the
// count of sigma < x passes k.
//
// One group of G lanes per singular value: each lane evaluates the count at
// one of G interior points of the value's interval [lo, hi], a ballot over the
// group picks the sub-interval that holds the value (log2(G + 1) bits per
// round, ~13 rounds for fp64 with G = 16), and every lane of the group
// recomputes the points itself, so the group never exchanges data beyond the
// ballot.  All lanes of a wave walk the same squared off-diagonals a^2 in the
// same order (broadcast loads).  The matrix is scaled by its largest entry so
// the squares can neither overflow nor underflow for any finite input that
// does not itself underflow.
//
// Accuracy: the loop stops once hi - lo <= max(2 eps hi, eps bound) -- the
// absolute accuracy of the host QR (|sigma - sigma_exact| ~ eps sigma_max),
// relative for the values well above eps sigma_max.
#include "brd_internal.h"

#include <cfloat>

namespace brd {

// Lanes per singular value (n = 8192 fp64, same box: 4 lanes 22.9 ms, 8 17.0,
// 16 15.6; the count loop unrolled by 4: 16 lanes 13.5 ms, 8 13.9; the IEEE
// division instead of the refined reciprocal: 26.5 at 8 lanes).
#ifndef BRD_BD_LANES
#define BRD_BD_LANES 16
#endif
#ifndef BRD_BD_UNROLL
#define BRD_BD_UNROLL 4
#endif
constexpr int kBdG = BRD_BD_LANES;
static_assert(kBdG >= 2 && kBdG <= 16 && (kBdG & (kBdG - 1)) == 0, "2..16 lanes, a power of two");
constexpr int kBdBlock = 256;   // threads per workgroup (32 values)

template <typename T> struct BdEps;
template <> struct BdEps<double> { static constexpr double eps = DBL_EPSILON, tiny = DBL_MIN; };
template <> struct BdEps<float> { static constexpr float eps = FLT_EPSILON, tiny = FLT_MIN; };

// a2[0 .. 2n-1): squared off-diagonals of T_GK / scale^2; ws[2n-1] = scale,
// ws[2n] = the Gershgorin bound of T_GK / scale (max row sum of |a|).
// One workgroup (the setup is O(n) against the O(n^2) multisection).
template <typename T>
__global__ void __launch_bounds__(1024) k_bd_prep(const T *__restrict__ d, const T *__restrict__ e, int n,
                                                  T *__restrict__ ws)
{
    __shared__ T red[1024 / 64];
    const int tid = threadIdx.x;
    T mx = (T)0;
    for (int i = tid; i < n; i += blockDim.x) {
        mx = fmax(mx, fabs(d[i]));
        if (i < n - 1) mx = fmax(mx, fabs(e[i]));
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    if (tid < 64) {
        T v = tid < (int)(blockDim.x / 64) ? red[tid] : (T)0;
        for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
        if (tid == 0) red[0] = v;
    }
    __syncthreads();
    const T scale = red[0] > (T)0 ? red[0] : (T)1;
    const T inv = (T)1 / scale;
    T bound = (T)0;
    for (int i = tid; i < 2 * n - 1; i += blockDim.x) {
        const T a = (i & 1) ? e[i >> 1] * inv : d[i >> 1] * inv;
        ws[i] = a * a;
        // row i+1 of T_GK holds a_i and a_{i+1}
        const T an = i + 1 < 2 * n - 1 ? (((i + 1) & 1) ? e[(i + 1) >> 1] : d[(i + 1) >> 1]) * inv : (T)0;
        bound = fmax(bound, fabs(a) + fabs(an));
    }
    if (n == 1) bound = fabs(d[0]) * inv;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) bound = fmax(bound, __shfl_xor(bound, o));
    if ((tid & 63) == 0) red[tid >> 6] = bound;
    __syncthreads();
    if (tid == 0) {
        T v = (T)0;
        for (int w = 0; w < (int)(blockDim.x / 64); ++w) v = fmax(v, red[w]);
        ws[2 * n - 1] = scale;
        ws[2 * n] = v * ((T)1 + (T)4 * BdEps<T>::eps) + BdEps<T>::tiny;
    }
}

// 1/q: the hardware reciprocal refined by Newton steps to full precision
// (fewer instructions than the IEEE division sequence; the count only needs
// the sign of each pivot, which the refined quotient keeps).
__device__ __forceinline__ double bd_rcp(double q) {
    double r = __builtin_amdgcn_rcp(q);
    r = fma(r, fma(-q, r, 1.0), r);
    r = fma(r, fma(-q, r, 1.0), r);
    return r;
}
__device__ __forceinline__ float bd_rcp(float q) {
    const float r = __builtin_amdgcn_rcpf(q);
    return fmaf(r, fmaf(-q, r, 1.0f), r);
}

// #{sigma < x} for x > 0: negative pivots of T_GK - x I, less n.
template <typename T>
__device__ __forceinline__ int bd_count(const T *__restrict__ a2, int m, T x, T pivmin) {
    T q = -x;
    int neg = 1;   // q_1 = -x < 0
#pragma unroll BRD_BD_UNROLL
    for (int i = 0; i < m; ++i) {
        if (fabs(q) < pivmin) q = -pivmin;
#ifdef BRD_BD_IEEE_DIV
        q = -x - a2[i] / q;
#else
        q = fma(-a2[i], bd_rcp(q), -x);
#endif
        neg += q < (T)0 ? 1 : 0;
    }
    return neg - (m + 1) / 2;
}

template <typename T>
__global__ void __launch_bounds__(kBdBlock) k_bd_bisect(const T *__restrict__ ws, int n, T *__restrict__ sv)
{
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = gid / kBdG;                // ascending index of this group's value
    const int l = threadIdx.x % kBdG;        // this lane's point in the interval
    const int m = 2 * n - 1;
    const T scale = ws[m], bound = ws[m + 1];
    const T eps = BdEps<T>::eps;
    // LAPACK-style pivot floor: safe minimum x max(1, max a^2) (a^2 <= 1 after scaling)
    const T pivmin = BdEps<T>::tiny;
    const bool live = k < n;
    T lo = (T)0, hi = bound;
    const int gbase = (threadIdx.x & 63) & ~(kBdG - 1);   // first lane of the group within the wave
    for (int it = 0; it < 200; ++it) {
        const bool done = !live || hi - lo <= fmax((T)2 * eps * hi, eps * bound);
        // the whole wave runs the count while any group still needs it
        if (__all(done)) break;
        const T w = (hi - lo) / (T)(kBdG + 1);
        const T x = lo + w * (T)(l + 1);
        const bool above = done ? true : bd_count<T>(ws, m, x, pivmin) > k;
        const unsigned long long bal = __ballot(above);
        const unsigned grp = (unsigned)(bal >> gbase) & ((1u << kBdG) - 1u);
        if (!done) {
            // smallest point whose count passes k: the value lies below it
            const int first = grp ? __builtin_ctz(grp) : kBdG;
            const T nhi = first < kBdG ? lo + w * (T)(first + 1) : hi;
            const T nlo = first > 0 ? lo + w * (T)first : lo;
            lo = nlo;
            hi = nhi;
        }
    }
    if (live && l == 0) sv[n - 1 - k] = (T)0.5 * (lo + hi) * scale;
}

template <typename T>
hipError_t launch_bdsvd_dev(const T *d, const T *e, int n, T *sv, T *ws, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_bd_prep<T>), dim3(1), dim3(1024), 0, s, d, e, n, ws);
    const long threads = (long)n * kBdG;
    const int grid = (int)((threads + kBdBlock - 1) / kBdBlock);
    hipLaunchKernelGGL((k_bd_bisect<T>), dim3(grid), dim3(kBdBlock), 0, s, (const T *)ws, n, sv);
    return hipGetLastError();
}

template hipError_t launch_bdsvd_dev<double>(const double *, const double *, int, double *, double *, hipStream_t);
template hipError_t launch_bdsvd_dev<float>(const float *, const float *, int, float *, float *, hipStream_t);

}  // namespace brd
