// Blocked stage 1: the panel QR (CholeskyQR2 / shifted CholeskyQR3 with
// basis-kernel reconstruction), k_cqr_gram / k_cqr_q1 / k_cqr_v (gfx950).
#include "brd_blk.h"

namespace brd {
namespace blk {

// ==========================================================================
// k_cqr_*: QR of a tall M x 32 panel P as an orthogonal block reflector
// Q' = I - V T V^T with Q'^T P = [R; 0], by nwg = ceil(M / 256) workgroups,
// one thread per row, in three kernels (the kernel boundaries are the
// panel-wide synchronisations, so no workgroup ever waits for another and
// nothing requires co-residency -- several lanes' kernels share the chip):
//   k_cqr_gram  per workgroup: the rows, their largest power-of-two exponent,
//               the Gram partial of the prescaled rows
//   k_cqr_q1    every workgroup: the partials summed in fixed order (each
//               rescaled to the panel's exponent), R1 = chol(G1) (redundantly,
//               wave 0), Q1 = P 2^-e R1^-1 for its rows (to the workspace),
//               the Gram partial of Q1
//   k_cqr_v     every workgroup: G2 = Q1^T Q1, R2 = chol(G2) (first order
//               when G2 = I + E with |E| < 1e-8), V = Q = Q1 R2^-1 for its
//               rows >= 32 (basis-kernel form: V = Q - [S; 0]); workgroup 0:
//               the modified LU of the top block, Q_t - S = L U (s_j = -sign
//               of the pivot, Ballard et al. 2015), V's top rows Q_t - S,
//               T = -S (U^-1 L^-1)^T and the band block R = S R2 R1 2^e.
// (Q' is orthogonal and Q' [S; 0] = Q for any sign matrix S with W_t = Q_t - S
// invertible -- the basis-kernel representation of Sun and Bischof; the
// modified LU's sign choice keeps W_t well conditioned, as in the Householder
// reconstruction.)  All arithmetic in fp64.  A first-pass Cholesky pivot
// that is not positive or below 1e-7 x the largest (panel condition number
// beyond ~1e7, where CholeskyQR2 loses orthogonality) switches the panel to
// shifted CholeskyQR3 (k_cqr_q1's shift, cqr_shifted_pass); a breakdown
// after that sets the error word (3).
// ==========================================================================
// Gram partial of this wave's rows (one per lane) accumulated into gacc
// (the three distinct 16 x 16 blocks of the symmetric 32 x 32)
// (staged in two halves of 32 rows, k-steps 0-7 then 8-15: the same MFMA
// chain as one 64-row staging, in half the LDS -- CqrLdsS)
template <class LDS>
__device__ __forceinline__ void gram_wave(LDS &L, int w, int lane, const double (&x)[32], double (&gacc)[3][4]) {
    typedef Mf<double>::v4 v4;
    const int qq = lane >> 4, l15 = lane & 15;
    v4 a00 = {gacc[0][0], gacc[0][1], gacc[0][2], gacc[0][3]};
    v4 a01 = {gacc[1][0], gacc[1][1], gacc[1][2], gacc[1][3]};
    v4 a11 = {gacc[2][0], gacc[2][1], gacc[2][2], gacc[2][3]};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if ((lane >> 5) == h) {
#pragma unroll
            for (int t = 0; t < 32; ++t) L.q[w][lane & 31][t] = x[t];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int s = 8 * h; s < 8 * h + 8; ++s) {
            const int k = 4 * s + qq - 32 * h;
            const double v0 = L.q[w][k][l15], v1 = L.q[w][k][16 + l15];
            a00 = Mf<double>::mma(v0, v0, a00);
            a01 = Mf<double>::mma(v0, v1, a01);
            a11 = Mf<double>::mma(v1, v1, a11);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) { gacc[0][g] = a00[g]; gacc[1][g] = a01[g]; gacc[2][g] = a11[g]; }
}

// Cholesky G = R^T R (R upper) by one wave, lane c holding column c in
// registers, row j of R broadcast by readlanes; R and 1/diag into LDS.
// False on a non-positive or tiny pivot.
// DEF (the sCQR3 middle pass, cqr_shifted_pass): a tiny or non-positive pivot
// j instead marks column j deficient (bit j of *mask) -- the direction of
// Q1's column j is numerically inside the span of its earlier columns, i.e.
// the panel is (numerically) rank deficient there.  Row j of R is written as
// zeros (R~': Q1 = y R~' up to the dropped residual, whose contribution to the
// panel is of the size of the panel's singular value in that direction) and
// Rw's row j as the unit row (y's column j is left for the caller to replace
// by a completion vector); column j takes no part in the elimination.  False
// only on a non-finite pivot.
template <bool DEF = false>
__device__ __forceinline__ bool chol_wave(const double (&G)[32][kSP], double (&R)[32][kSP], double (&Rw)[32][kSP], int lane,
                                          unsigned *mask = nullptr) {
    // lane c: column c in registers; row j of R goes through LDS (R itself)
    // and comes back as 16-byte broadcast reads: no readlane per element
    typedef double d2 __attribute__((ext_vector_type(2)));
    const int c = lane & 31;
    double col[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) col[i] = G[i][c];
    bool ok = true;
    double dmax = 0;
    unsigned dm = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const double piv = rdl(col[j], j);
        const bool good = piv > 0 && piv < 1e300;
        // 1/sqrt by the hardware estimate and two Newton steps (the division and
        // IEEE square root sit on the 32-step chain)
        const double pv = good ? piv : 1.0;
        double invd = __builtin_amdgcn_rsq(pv);
        invd = invd * fma(-0.5 * pv * invd, invd, 1.5);
        invd = invd * fma(-0.5 * pv * invd, invd, 1.5);
        double d = pv * invd;
        bool defic = false;
        if constexpr (DEF) {
            if (!(piv == piv) || piv >= 1e300) ok = false;   // NaN / overflow: a real failure
            defic = !good || d < 1e-7 * dmax;
            if (defic) { dm |= 1u << j; invd = 0.0; d = 0.0; }
        } else {
            if (!good || d < 1e-7 * dmax) ok = false;
        }
        dmax = fmax(dmax, d);
        const double r = col[j] * invd;   // R[j][c] (meaningful for c >= j; 0 for a deficient j)
        if (lane < 32) {
            R[j][c] = c >= j ? r : 0.0;
            Rw[j][c] = c > j ? r : (c == j ? (defic ? 1.0 : invd) : 0.0);
        }
        if (j == 31) break;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        d2 rr[16];
#pragma unroll
        for (int p = (j + 1) / 2; p < 16; ++p) rr[p] = *(const d2 *)&R[j][2 * p];
#pragma unroll
        for (int i = j + 1; i < 32; ++i) col[i] = fma(-((i & 1) ? rr[i >> 1].y : rr[i >> 1].x), r, col[i]);
    }
    if constexpr (DEF) {
        // the trsm form's column j above the diagonal zeroed too: y's column j
        // is then x's column j itself, so the caller may put the completion
        // into x before the solve (no extra live values beside trsm_row)
        if (lane < 32 && (dm >> c & 1u)) {
#pragma unroll
            for (int k = 0; k < 32; ++k)
                if (k < c) Rw[k][c] = 0.0;
        }
        *mask = dm;
    }
    return ok;
}

// x <- x R^-1, right-looking.  (No scheduling groups: with
// sched_group_barrier pairs per step -- the next row's LDS reads first, then
// the step's VALU -- the k_cqr_* kernels measured 19.9 / 19.7 us against 19.7 /
// 20.5 without (round 3), and the translation unit took 12 min to compile
// instead of 30 s.)  Rw: R (upper) with the reciprocal of its
// diagonal in place of the diagonal, in LDS.  Row k + 1 of Rw is read (as
// 16-byte pairs, a wave-uniform address: one LDS broadcast per pair) while
// step k computes, so the reads' latency is hidden behind the FMAs.
typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void trsm_row(double (&x)[32], const double (&Rw)[32][kSP]) {
    d2v cur[16], nxt[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) cur[p] = *(const d2v *)&Rw[0][2 * p];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        if (k + 1 < 32) {
#pragma unroll
            for (int p = (k + 1) / 2; p < 16; ++p) nxt[p] = *(const d2v *)&Rw[k + 1][2 * p];
        }
        x[k] *= (k & 1) ? cur[k >> 1].y : cur[k >> 1].x;
        const double xk = x[k];
#pragma unroll
        for (int i = k + 1; i < 32; ++i) x[i] = fma(-xk, (i & 1) ? cur[i >> 1].y : cur[i >> 1].x, x[i]);
        if (k + 1 < 32) {
#pragma unroll
            for (int p = (k + 1) / 2; p < 16; ++p) cur[p] = nxt[p];
        }
    }
}

// x <- x Ri for an upper-triangular Ri in LDS (all products independent:
// x[t] = sum_{k <= t} x[k] Ri[k][t], k ascending).
__device__ __forceinline__ void umul_row(double (&x)[32], const double (&Ri)[32][kSP]) {
    double acc[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) acc[t] = 0.0;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        d2v rr[16];
#pragma unroll
        for (int p = k / 2; p < 16; ++p) rr[p] = *(const d2v *)&Ri[k][2 * p];
#pragma unroll
        for (int t = k; t < 32; ++t) acc[t] = fma(x[k], (t & 1) ? rr[t >> 1].y : rr[t >> 1].x, acc[t]);
    }
#pragma unroll
    for (int t = 0; t < 32; ++t) x[t] = acc[t];
}

// The cluster's Gram partials (workgroup-major [nwg][1024]) summed by every
// workgroup on its own, in fixed order (deterministic), scaled by the
// per-partial powers of two scl[k]: one cluster barrier per Gram instead of a
// slice-sum, a second barrier and a read-back.
#ifndef BRD_GRAM_BATCH
#define BRD_GRAM_BATCH 8    // partials per batch of loads in flight (A/B knob, tools/variant_lib.sh)
#endif
template <class LDS>
__device__ __forceinline__ void gram_sum_all(LDS &L, const double *gp, const double *scl, int nwg, long gs = 1024) {
    const int tid = threadIdx.x;
    constexpr int GB = BRD_GRAM_BATCH;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < nwg; k0 += GB) {
        double v[GB][4];
#pragma unroll
        for (int k = 0; k < GB; ++k) {
            const int kc = min(k0 + k, nwg - 1);
#pragma unroll
            for (int u = 0; u < 4; ++u) v[k][u] = gp[(size_t)kc * gs + tid + kCT * u];
        }
#pragma unroll
        for (int k = 0; k < GB; ++k) {
            const double sk = k0 + k < nwg ? scl[k0 + k] : 0.0;
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = fma(sk, v[k][u], acc[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int el = tid + kCT * u;
        L.g[el >> 5][el & 31] = acc[u];
    }
}

// this thread's row of P (zeros past M), as doubles
template <typename T>
__device__ __forceinline__ void cqr_load_row(const CqrArgs &a, int i, double (&x)[32]) {
    const T *src = (const T *)a.src;
    const int ic = i < a.M ? i : 0;
    const T *srow = src + (size_t)ic * a.si;
    if (a.st == 1) {   // a row of 32 contiguous elements: 16-byte loads
        typedef typename G2<T>::v2 v2;
#pragma unroll
        for (int t = 0; t < 32; t += 2) {
            const v2 v = *(const v2 *)(srow + t);
            x[t] = (double)v.x;
            x[t + 1] = (double)v.y;
        }
    } else {
        const long st = a.st;
#pragma unroll
        for (int t = 0; t < 32; ++t) x[t] = (double)srow[t * st];
    }
    if (i >= a.M) {
#pragma unroll
        for (int t = 0; t < 32; ++t) x[t] = 0.0;
    }
}

// Gram partial of the workgroup's rows (one per thread) -> dst (1024 doubles):
// the four waves' partials summed in fixed order
// (coh: agent-scope stores, for the distributed form's last-arriver sum in
// the same kernel, cqr_to_record)
template <class LDS>
__device__ __forceinline__ void cqr_gram_partial(LDS &L, const double (&x)[32], double *dst, bool coh = false) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double gacc[3][4] = {};
    gram_wave(L, w, lane, x, gacc);
    __syncthreads();
    double(*gw)[32][33] = reinterpret_cast<double(*)[32][33]>(&L.q[0][0][0]);   // [4][32][33] over the staging
    const int qq = lane >> 4, l15 = lane & 15;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int rr = Mf<double>::crow(qq, g);
        gw[w][rr][l15] = gacc[0][g];
        gw[w][rr][16 + l15] = gacc[1][g];
        gw[w][16 + l15][rr] = gacc[1][g];
        gw[w][16 + rr][16 + l15] = gacc[2][g];
    }
    __syncthreads();
    for (int el = tid; el < 1024; el += kCT) {
        const int i = el >> 5, t = el & 31;
        const double v = (gw[0][i][t] + gw[1][i][t]) + (gw[2][i][t] + gw[3][i][t]);
        if (coh) __hip_atomic_store(dst + el, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else     dst[el] = v;
    }
}

// the panel's exponent e (INT_MIN: the panel is zero) and the partials' scale
// factors 2^(2 (e_k - e)) into L.scl
template <class LDS>
__device__ __forceinline__ int cqr_exponent(LDS &L, const double *ew, int nwg, bool ones, long es = 1) {
    const int tid = threadIdx.x;
    __shared__ int ewl[kCW];
    if (tid < kCW) ewl[tid] = tid < nwg ? (int)ew[(size_t)tid * es] : INT_MIN;
    __syncthreads();
    int e = INT_MIN;
    for (int k = 0; k < nwg; ++k) e = max(e, ewl[k]);
    if (tid < kCW) L.scl[tid] = ones ? 1.0 : ((tid < nwg && ewl[tid] != INT_MIN) ? ldexp(1.0, 2 * (ewl[tid] - e)) : 0.0);
    __syncthreads();
    return e;
}

// ---- the distributed form (CqrArgs::rec): per-rank records ------------------
// The last workgroup of a kernel to arrive sums the kernel's partials (gp
// [nwg][1024], agent-scope stores; exponents ew, or none) in fixed order into
// this rank's record of bank `bank`: the 32 x 32 Gram of this rank's rows
// (scaled by 2^-2e_r) and e_r.  The caller all-gathers the bank; the next
// kernel sums the nrec records in rank order (cqr_gram_src), so every rank
// holds the same panel-wide Gram, bit for bit.
__device__ __forceinline__ double *cqr_bank(const CqrArgs &a, int bank) {
    return a.rec + (size_t)bank * a.nrec * kCqrRec;
}
template <class LDS>
__device__ void cqr_to_record(LDS &L, const CqrArgs &a, const double *gp, const double *ew, int bank) {
    const int tid = threadIdx.x, nwg = gridDim.x;
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's partial stores have landed
    __syncthreads();
    if (tid == 0) {
        const int old = __hip_atomic_fetch_add(a.rctr + bank, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        last = old == nwg - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(a.rctr + bank, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (!last) return;
    __shared__ int ewl[kCW];
    if (tid < kCW)
        ewl[tid] = (ew && tid < nwg) ? (int)__hip_atomic_load(ew + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : INT_MIN;
    __syncthreads();
    int e = INT_MIN;
    if (ew)
        for (int k = 0; k < nwg; ++k) e = max(e, ewl[k]);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < nwg; ++k) {
        const double sk = !ew ? 1.0 : (ewl[k] == INT_MIN ? 0.0 : ldexp(1.0, 2 * (ewl[k] - e)));
#pragma unroll
        for (int u = 0; u < 4; ++u)
            acc[u] = fma(sk, __hip_atomic_load(gp + (size_t)k * 1024 + tid + kCT * u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT), acc[u]);
    }
    double *r = cqr_bank(a, bank) + (size_t)a.rme * kCqrRec;
#pragma unroll
    for (int u = 0; u < 4; ++u) r[tid + kCT * u] = acc[u];
    if (tid == 0) r[1024] = (double)e;
}
// the panel-wide Gram's source: the records of bank `bank` (distributed) or
// this kernel's own partials
struct GramSrc {
    const double *gp, *ew;
    int n;
    long gs, es;
};
__device__ __forceinline__ GramSrc cqr_gram_src(const CqrArgs &a, int bank, const double *gp, const double *ew) {
    if (a.rec) {
        const double *b = cqr_bank(a, bank);
        return GramSrc{b, b + 1024, a.nrec, kCqrRec, kCqrRec};
    }
    return GramSrc{gp, ew, (int)gridDim.x, 1024, 1};
}

template <typename T>
__global__ void __launch_bounds__(kCT, 1) k_cqr_gram(CqrArgs a) {
    __shared__ CqrLdsS L;
    const int tid = threadIdx.x, lane = tid & 63, wg = blockIdx.x;
    CqrWs W(a.ws);
    double x[32];
    cqr_load_row<T>(a, wg * kCT + tid, x);
    double m = 0;
#pragma unroll
    for (int t = 0; t < 32; ++t) m = fmax(m, fabs(x[t]));
    for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    if (tid == 0) L.e_w = INT_MIN;
    __syncthreads();
    if (lane == 0) {
        int e = INT_MIN;
        if (m > 0) frexp(m, &e);
        atomicMax(&L.e_w, e);
    }
    __syncthreads();
    const int e_w = L.e_w;
    if (e_w != INT_MIN) {
#pragma unroll
        for (int t = 0; t < 32; ++t) x[t] = ldexp(x[t], -e_w);
    }
    const bool coh = a.rec != nullptr;
    cqr_gram_partial(L, x, W.gp1 + (size_t)wg * 1024, coh);
    if (tid == 0) {
        if (coh) __hip_atomic_store(W.ew + wg, (double)e_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else     W.ew[wg] = (double)e_w;
    }
    if (coh) cqr_to_record(L, a, W.gp1, W.ew, 0);
}

// BRD_CQR_STAMPS (diagnostic builds, tools/cqr_stamps.py): per-workgroup
// phase timestamps of the k_cqr_v launches whose a.M equals the target the
// host set (k_cqr_v's register allocation is unchanged by them; stamps in
// k_cqr_q1 made it spill, so it has none)
#ifdef BRD_CQR_STAMPS
__device__ unsigned long long g_cqr_st[64][12];
__device__ long g_cqr_target;
#define CQR_ST(P)                                                                          \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 64 && (long)a.M == g_cqr_target)               \
            g_cqr_st[blockIdx.x][P] = __builtin_amdgcn_s_memrealtime();                    \
    } while (0)
#else
#define CQR_ST(P) \
    do {          \
    } while (0)
#endif

template <typename T>
__global__ void __launch_bounds__(kCT, 1) k_cqr_q1(CqrArgs a) {
    __shared__ CqrLdsS L;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wg = blockIdx.x;
    CqrWs W(a.ws);
    if (tid == 0) L.flags = 0;
    const int i = wg * kCT + tid;
    double x[32];
    cqr_load_row<T>(a, i, x);   // in flight under the Gram sum and the Cholesky
    const GramSrc g1 = cqr_gram_src(a, 0, W.gp1, W.ew);
    const int e = cqr_exponent(L, g1.ew, g1.n, false, g1.es);
    if (e == INT_MIN) {   // zero panel: k_cqr_v writes V = [I; 0], T = 0, R = 0
        if (wg == 0 && tid == 0) W.shifted[0] = 0.0;
        return;
    }
    gram_sum_all(L, g1.gp, L.scl, g1.n, g1.gs);
    __syncthreads();
    if (w == 0) {
        bool good = chol_wave(L.g, L.r1, L.r1w, lane);
        if (!good) {
            // an ill-conditioned panel (cond > ~1e7, e.g. numerically rank
            // deficient): the shifted Cholesky of sCQR3 (Fukaya et al. 2020),
            // G + s I with s = 11 (32 M + 32 33) u tr(G); then Q1 has
            // cond ~ 1e3 and k_cqr_v's cqr_shifted_pass re-orthogonalises it once more
            double tr = 0;
#pragma unroll
            for (int k = 0; k < 32; ++k) tr += L.g[k][k];
            const double sh = 11.0 * (32.0 * (a.rec ? a.Mg : a.M) + 32.0 * 33.0) * 0x1p-53 * tr;
            if (lane < 32) L.g[lane][lane] += sh;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            good = chol_wave(L.g, L.r1, L.r1w, lane);
            if (lane == 0) L.flags = good ? 2 : 1;
        }
    }
    __syncthreads();
    if (L.flags == 1 && tid == 0) __hip_atomic_store(a.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wg == 0) {
        for (int el = tid; el < 1024; el += kCT) W.r1[el] = L.r1[el >> 5][el & 31];
        if (tid == 0) W.shifted[0] = L.flags == 2 ? 1.0 : 0.0;
    }
    // Q1 = (P 2^-e) R1^-1
#pragma unroll
    for (int t = 0; t < 32; ++t) x[t] = ldexp(x[t], -e);
    trsm_row(x, L.r1w);
    if (i >= a.M) {
#pragma unroll
        for (int t = 0; t < 32; ++t) x[t] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < 32; ++t) W.q1[t * kQS + i] = x[t];
    cqr_gram_partial(L, x, W.gp2 + (size_t)wg * 1024, a.rec != nullptr);
    if (a.rec) cqr_to_record(L, a, W.gp2, nullptr, 1);
}

// After a shifted first pass only (W.shifted): sCQR3's middle pass, run by
// every workgroup of k_cqr_v on its own (the same reads in the same order,
// so the same result everywhere; no kernel of its own, which the common
// unshifted panel would pay for as a launch): R = chol(Q1^T Q1), the Gram of
// Q1 R^-1 over ALL rows into L.g (the four waves' sums in fixed order),
// R R1 into L.r1 and this thread's row of Q1 R^-1 into x.  Every workgroup
// walks all rows (the rare ill-conditioned panel pays ~0.1-0.2 ms).
//
// Exact (or numerical) rank deficiency: a panel with a zero
// column, duplicate columns or rank < 32 has Q1 columns inside the span of
// earlier ones, and Q1^T Q1 a (numerically) zero pivot.  The Cholesky here
// marks such columns deficient (chol_wave<true>) and the walk replaces y's
// column j by a completion vector (a fixed pseudo-random function of the row
// index, the same in every workgroup): y = [Q1 R~^-1 | completion].  One more
// CholeskyQR pass over all rows (walk A: Gram(y) -> Ra) makes y well
// conditioned whatever the completions' overlap with the kept columns, and
// k_cqr_v's final pass orthonormalises it as usual, so Q stays orthonormal
// and spans the panel; the band block is R2 Ra R~' R1 2^e (R~': the deficient
// rows zeroed).  A full-rank panel takes exactly the previous path (mask 0).
__device__ __forceinline__ double cqr_completion(int i, int j, double scale) {
    unsigned h = (unsigned)i * 0x9E3779B1u ^ ((unsigned)j + 1u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    h *= 0x297A2D39u;
    h ^= h >> 15;
    return ((double)h * 0x1p-31 - 1.0) * scale;   // uniform in [-1, 1) times scale
}

// 32 x 32 Gram from the four waves' MFMA partials (fixed order) into G
__device__ __forceinline__ void gram_collect(CqrLds &L, double (&G)[32][kSP], const double (&gacc)[3][4]) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double(*gw)[32][33] = reinterpret_cast<double(*)[32][33]>(&L.q[0][0][0]);
    const int qq = lane >> 4, l15 = lane & 15;
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int rr = Mf<double>::crow(qq, g);
        gw[w][rr][l15] = gacc[0][g];
        gw[w][rr][16 + l15] = gacc[1][g];
        gw[w][16 + l15][rr] = gacc[1][g];
        gw[w][16 + rr][16 + l15] = gacc[2][g];
    }
    __syncthreads();
    for (int el = tid; el < 1024; el += kCT) {
        const int i2 = el >> 5, t = el & 31;
        G[i2][t] = (gw[0][i2][t] + gw[1][i2][t]) + (gw[2][i2][t] + gw[3][i2][t]);
    }
}

// the deficiency-detecting Cholesky as a call of its own: inlined, its
// per-step selects raised k_cqr_v from 60 to 256 AGPRs (register allocation
// of the whole kernel); the call is on the rare shifted path only
__device__ __attribute__((noinline)) bool chol_def(const double (&G)[32][kSP], double (&R)[32][kSP], double (&Rw)[32][kSP],
                                                   int lane, unsigned *mask) {
    return chol_wave<true>(G, R, Rw, lane, mask);
}

__device__ __forceinline__ void cqr_shifted_pass(CqrLds &L, const CqrWs &W, const CqrArgs &a, int nwg, double (&x)[32]) {
    const int M = a.M;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    __shared__ unsigned dmask;
    gram_sum_all(L, W.gp2, L.scl, nwg);
    __syncthreads();
    if (w == 0) {
        unsigned mk = 0;
        const bool good = chol_def(L.g, L.r2, L.r2w, lane, &mk);
        if (lane == 0) {
            if (!good) L.flags = 1;
            dmask = mk;
        }
    }
    for (int el = tid; el < 1024; el += kCT) L.r1[el >> 5][el & 31] = W.r1[el];
    __syncthreads();
    const unsigned mask = dmask;
    const double cscale = 1.0 / sqrt((double)max(M, 1));
    // this thread's row i of y = Q1 R~^-1, deficient columns replaced
    auto yrow = [&](int i, double (&y)[32]) {
#pragma unroll
        for (int t = 0; t < 32; ++t) y[t] = W.q1[t * kQS + i];
        if (mask) {   // (chol_wave<true> made the solve leave these columns alone)
#pragma unroll
            for (int t = 0; t < 32; ++t)
                if (mask >> t & 1u) y[t] = cqr_completion(i, t, cscale);
        }
        trsm_row(y, L.r2w);
        if (i >= M) {
#pragma unroll
            for (int t = 0; t < 32; ++t) y[t] = 0.0;
        }
    };
    if (mask) {   // walk A: Ra = chol(Gram(y)) (L.u / L.mm: free until the finish)
        double gacc[3][4] = {};
        for (int chunk = 0; chunk < nwg; ++chunk) {
            double y[32];
            yrow(chunk * kCT + tid, y);
            gram_wave(L, w, lane, y, gacc);
        }
        gram_collect(L, L.g, gacc);
        __syncthreads();
        if (w == 0) {
            const bool good = chol_wave(L.g, L.u, L.mm, lane);
            if (lane == 0 && !good) L.flags = 1;
        }
        __syncthreads();
    }
    double gacc[3][4] = {};
    for (int chunk = 0; chunk < nwg; ++chunk) {
        const int i = chunk * kCT + tid;
        double y[32];
        yrow(i, y);
        if (mask) {
            __builtin_amdgcn_sched_barrier(0);   // the two solves one after the other (register pressure)
            trsm_row(y, L.mm);
            if (i >= M) {
#pragma unroll
                for (int t = 0; t < 32; ++t) y[t] = 0.0;
            }
        }
        if (chunk == (int)blockIdx.x) {
#pragma unroll
            for (int t = 0; t < 32; ++t) x[t] = y[t];
        }
        gram_wave(L, w, lane, y, gacc);
    }
    // R R1 (waves 0-3: one tile each, into registers first: L.r1 is an operand);
    // with deficient columns Ra (R~' R1)
    const int ti = w >> 1, tj = w & 1;
    for (int pass = 0; pass < (mask ? 2 : 1); ++pass) {
        Mf<double>::v4 rt = {0.0, 0.0, 0.0, 0.0};
        if (tj >= ti) rt = tile_mm(pass ? L.u : L.r2, L.r1, ti, tj, lane, 16 * ti, 32);
        __syncthreads();
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int i2 = 16 * ti + Mf<double>::crow(lane >> 4, g), c = 16 * tj + (lane & 15);
            L.r1[i2][c] = i2 <= c ? rt[g] : 0.0;
        }
        __syncthreads();
    }
    gram_collect(L, L.g, gacc);
}

// The distributed form's sCQR3 middle pass (CqrArgs::rec; on one GPU
// k_cqr_v runs it inside, walking all rows: cqr_shifted_pass).  After a
// shifted first pass: R~ = chol(G2) from the records (deficient columns
// marked, chol_def), this rank's rows of y = Q1 R~^-1 (completion vectors in
// the deficient columns) back into Q1's place, y's Gram into bank 2, and
// R~ R1 into R1's place (workgroup 0); k_cqr_v then runs its usual final
// pass on y with the Gram from bank 2.  (With deficient columns that is one
// CholeskyQR pass on y where cqr_shifted_pass makes two -- a third Gram would
// need a fourth collective -- so Q's orthogonality there is ~ cond(y)^2 u.)
// Every rank launches it (the collective after it is unconditional); an
// unshifted panel returns at once and bank 2 is not read.
template <typename T>
__global__ void __launch_bounds__(kCT, 1) k_cqr_mid(CqrArgs a) {
    __shared__ CqrLds L;
    __shared__ unsigned dmask;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = blockIdx.x * kCT + tid;
    CqrWs W(a.ws);
    if (W.shifted[0] == 0.0) return;
    if (tid == 0) L.flags = 0;
    if (tid < kCW) L.scl[tid] = 1.0;
    double y[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) y[t] = W.q1[t * kQS + i];
    __syncthreads();
    gram_sum_all(L, cqr_bank(a, 1), L.scl, a.nrec, kCqrRec);
    __syncthreads();
    if (w == 0) {
        unsigned mk = 0;
        const bool good = chol_def(L.g, L.r2, L.r2w, lane, &mk);
        if (lane == 0) {
            if (!good) L.flags = 1;
            dmask = mk;
        }
    }
    __syncthreads();
    const unsigned mask = dmask;
    if (mask) {
        const double cscale = 1.0 / sqrt((double)max(a.Mg, 1L));
#pragma unroll
        for (int t = 0; t < 32; ++t)
            if (mask >> t & 1u) y[t] = cqr_completion((int)(i + a.goff), t, cscale);
    }
    trsm_row(y, L.r2w);
    if (i >= a.M) {
#pragma unroll
        for (int t = 0; t < 32; ++t) y[t] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < 32; ++t) W.q1[t * kQS + i] = y[t];
    if (L.flags && tid == 0) __hip_atomic_store(a.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) {   // R~ R1 (waves 0-3: one 16 x 16 tile each) into R1's place
        for (int el = tid; el < 1024; el += kCT) L.r1[el >> 5][el & 31] = W.r1[el];
        __syncthreads();
        const int ti = w >> 1, tj = w & 1;
        Mf<double>::v4 rt = {0.0, 0.0, 0.0, 0.0};
        if (tj >= ti) rt = tile_mm(L.r2, L.r1, ti, tj, lane, 16 * ti, 32);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int i2 = 16 * ti + Mf<double>::crow(lane >> 4, g), c = 16 * tj + (lane & 15);
            W.r1[i2 * 32 + c] = i2 <= c ? rt[g] : 0.0;
        }
    }
    cqr_gram_partial(L, y, W.gp3 + (size_t)blockIdx.x * 1024, true);
    cqr_to_record(L, a, W.gp3, nullptr, 2);
}

// INLINE (the last LQ panel of a block, whose U's top block the block update
// reads straight away): workgroup 0 also runs cqr_finish itself and patches
// V's top block to Q_t - S in place.
template <typename T, bool INLINE>
__global__ void __launch_bounds__(kCT, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) k_cqr_v(CqrArgs a, FinArgs fin) {
    __shared__ CqrLds L;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wg = blockIdx.x, nwg = gridDim.x;
    CqrWs W(a.ws);
    CQR_ST(0);
    if (tid == 0) L.flags = 0;
    const GramSrc g1 = cqr_gram_src(a, 0, W.gp1, W.ew);
    const int e = cqr_exponent(L, g1.ew, g1.n, true, g1.es);   // (L.scl: ones)
    CQR_ST(1);
    const bool zero = e == INT_MIN;   // V = [I; 0], T = 0, R = 0
    const int i = wg * kCT + tid;
    T *ap = (T *)a.apan;
    T *vd = (T *)a.vdst;
    T *vd2 = (T *)a.vdst2;
    double x[32];
    const bool sh = !zero && W.shifted[0] != 0.0;
    if (!zero && (!sh || a.rec)) {   // this thread's row of Q1 (or y), in flight under the Gram sum
#pragma unroll
        for (int t = 0; t < 32; ++t) x[t] = W.q1[t * kQS + i];
    }
    if (!zero) {
        if (sh && !a.rec) {
            cqr_shifted_pass(L, W, a, nwg, x);
        } else {   // (distributed, shifted: x = y and its Gram in bank 2, k_cqr_mid)
            const GramSrc g2 = cqr_gram_src(a, sh ? 2 : 1, W.gp2, nullptr);
            gram_sum_all(L, g2.gp, L.scl, g2.n, g2.gs);
        }
        __syncthreads();
        CQR_ST(2);
        // G2 = Q1^T Q1 = I + E with E ~ cond(P)^2 eps.  When max|E| < 1e-8 the
        // Cholesky factor is I + U1 + O(E^2) (U1: the upper triangle of E with
        // half its diagonal) and its inverse I - U1 + O(E^2): both to working
        // accuracy, without the 32-step factorization.  Every wave decides
        // (the same reads, the same result).
        bool fast;
        {
            const int c = lane & 31, i0 = (lane >> 5) * 16;
            double em = 0;
#pragma unroll
            for (int ii = 0; ii < 16; ++ii) em = fmax(em, fabs(L.g[i0 + ii][c] - (i0 + ii == c ? 1.0 : 0.0)));
            for (int o = 32; o >= 1; o >>= 1) em = fmax(em, __shfl_xor(em, o, 64));
            fast = em < 1e-8;   // uniform over the workgroup
        }
        if (fast) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int el = tid + kCT * u, r = el >> 5, c = el & 31;
                const double u1 = r < c ? L.g[r][c] : (r == c ? 0.5 * (L.g[c][c] - 1.0) : 0.0);
                L.r2[r][c] = (r == c ? 1.0 : 0.0) + u1;
                L.r2w[r][c] = (r == c ? 1.0 : 0.0) - u1;
            }
        } else if (w == 0) {
            const bool good = chol_wave(L.g, L.r2, L.r2w, lane);
            if (lane == 0 && !good) L.flags = 1;
        }
        __syncthreads();
        CQR_ST(3);
        // Q = Q1 R2^-1, this thread's row
        if (fast) umul_row(x, L.r2w);
        else      trsm_row(x, L.r2w);
        CQR_ST(4);
        if (i >= a.M) {
#pragma unroll
            for (int t = 0; t < 32; ++t) x[t] = 0.0;
        }
    } else {
#pragma unroll
        for (int t = 0; t < 32; ++t) x[t] = 0.0;
    }
    if (wg == 0 && tid < 32) {
#pragma unroll
        for (int t = 0; t < 32; ++t) L.tq[tid][t] = x[t];   // Q_t for the LU
    }

    // ---- V's rows into vdst (and vdst2), zeros into the panel's rows >= 32.
    // Destinations with unit column stride are written coalesced: the wave's
    // 64 rows are staged in its LDS tile and each store instruction covers 4
    // rows x 32 contiguous elements (a lane per row would touch 64 rows per
    // instruction).  Rows in [rlo, rhi) of this wave only.
    const int wrow0 = wg * kCT + 64 * w;   // first row of this wave
    auto store_v = [&](const double (&v)[32], int rlo, int rhi) {
        typedef typename G2<T>::v2 v2;
        const bool mine = i >= rlo && i < rhi && i < a.M;
        if (a.vst == 1 || (vd2 && a.vst2 == 1)) {
#pragma unroll
            for (int t = 0; t < 32; ++t) L.q[w][lane][t] = v[t];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        auto rowmajor = [&](T *base, long rs) {
#pragma unroll 4
            for (int it = 0; it < 16; ++it) {
                const int r = 4 * it + (lane >> 4), row = wrow0 + r, cp = 2 * (lane & 15);
                if (row >= rlo && row < rhi && row < a.M)
                    *(v2 *)(base + (size_t)row * rs + cp) = v2{(T)L.q[w][r][cp], (T)L.q[w][r][cp + 1]};
            }
        };
        if (a.vst == 1) rowmajor(vd, a.vsi);
        else if (mine) {
            T *vr = vd + (size_t)i * a.vsi;
#pragma unroll
            for (int t = 0; t < 32; ++t) vr[t * a.vst] = (T)v[t];
        }
        if (vd2) {
            if (a.vst2 == 1) rowmajor(vd2, a.vsi2);
            else if (mine) {
                T *vr2 = vd2 + (size_t)i * a.vsi2;
#pragma unroll
                for (int t = 0; t < 32; ++t) vr2[t * a.vst2] = (T)v[t];
            }
        }
    };
    store_v(x, 0, INT_MAX);   // V' = Q (the top rows get - S after the LU: k_vsum)
    CQR_ST(5);
    if (a.azero) {   // zeros below the panel's R block
        typedef typename G2<T>::v2 v2;
        const int zlo = a.top ? 32 : 0;
        if (a.ast == 1) {
#pragma unroll 4
            for (int it = 0; it < 16; ++it) {
                const int row = wrow0 + 4 * it + (lane >> 4), cp = 2 * (lane & 15);
                if (row >= zlo && row < a.M) *(v2 *)(ap + (size_t)row * a.asi + cp) = v2{(T)0, (T)0};
            }
        } else if (i >= zlo && i < a.M) {
            T *arow = ap + (size_t)i * a.asi;
#pragma unroll
            for (int t = 0; t < 32; ++t) arow[t * a.ast] = (T)0;
        }
    }
    if (L.flags && tid == 0) __hip_atomic_store(a.err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    CQR_ST(6);
    if (wg != 0) return;

    // ---- workgroup 0: Q_t and the zero flag for the LU (k_rpass's finishing
    // workgroup), and R' = R2 R1 2^e into the panel (its rows get S there) ----
    if (tid < 32) {
#pragma unroll
        for (int t = 0; t < 32; ++t) W.qt[tid * 32 + t] = x[t];
    }
    if (tid == 0) W.zero[0] = zero ? 1.0 : 0.0;
    if (a.qcopy) {
        if (tid < 32) {
#pragma unroll
            for (int t = 0; t < 32; ++t) a.qcopy[tid * 32 + t] = x[t];
        }
        if (tid == 0) a.qcopy[1024] = zero ? 1.0 : 0.0;
    }
    if (w == 3 && ap && a.top) {
        if (!sh || a.rec)   // (after a one-GPU shifted pass L.r1 already holds R R1)
            for (int el = lane; el < 1024; el += 64) L.r1[el >> 5][el & 31] = zero ? 0.0 : W.r1[el];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4) {
            const int ti = t4 >> 1, tj = t4 & 1;
            Mf<double>::v4 rt = {0.0, 0.0, 0.0, 0.0};
            if (tj >= ti && !zero) rt = tile_mm(L.r2, L.r1, ti, tj, lane, 16 * ti, 32);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int i2 = 16 * ti + Mf<double>::crow(lane >> 4, g), c = 16 * tj + (lane & 15);
                ap[(size_t)i2 * a.asi + (size_t)c * a.ast] = (T)(i2 <= c ? ldexp(rt[g], e) : 0.0);
            }
        }
    }
    if constexpr (INLINE) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // R' and Q_t stores landed (read back below)
        __syncthreads();
        cqr_finish<T>(L.u, L.tq, L.r1w, L.mm, L.sgn, fin, tid, true);
        __syncthreads();
        if (tid < 32) {   // V's top block: Q_t - S on the diagonal, both copies
            T *p1 = vd + (size_t)tid * a.vsi + (size_t)tid * a.vst;
            *p1 = (T)((double)*p1 - L.sgn[tid]);
            if (vd2) {
                T *p2 = vd2 + (size_t)tid * a.vsi2 + (size_t)tid * a.vst2;
                *p2 = (T)((double)*p2 - L.sgn[tid]);
            }
        }
    }
}



template <typename T>
void launch_k_cqr(CqrKernel which, int nwg, const CqrArgs &a, const FinArgs &f, hipStream_t s) {
    switch (which) {
        case kCqrGram: blk_launch("s1_cqr", 0.0, 0.0, k_cqr_gram<T>, dim3(nwg), dim3(kCT), s, a); break;
        case kCqrQ1:   blk_launch("s1_cqr", 0.0, 0.0, k_cqr_q1<T>, dim3(nwg), dim3(kCT), s, a); break;
        case kCqrV:    blk_launch("s1_cqr", 0.0, 0.0, k_cqr_v<T, false>, dim3(nwg), dim3(kCT), s, a, f); break;
        case kCqrMid:  blk_launch("s1_cqr", 0.0, 0.0, k_cqr_mid<T>, dim3(nwg), dim3(kCT), s, a); break;
        default:       blk_launch("s1_cqr", 0.0, 0.0, k_cqr_v<T, true>, dim3(nwg), dim3(kCT), s, a, f); break;
    }
}
template void launch_k_cqr<double>(CqrKernel, int, const CqrArgs &, const FinArgs &, hipStream_t);
template void launch_k_cqr<float>(CqrKernel, int, const CqrArgs &, const FinArgs &, hipStream_t);

}  // namespace blk
}  // namespace brd

#ifdef BRD_CQR_STAMPS
extern "C" int brd_debug_cqr_target(long m) {   // and clears the stamps
    static unsigned long long zero[64 * 12];
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(brd::blk::g_cqr_st), zero, sizeof(zero));
    if (e != hipSuccess) return (int)e;
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(brd::blk::g_cqr_target), &m, sizeof(m));
}
extern "C" int brd_debug_cqr_stamps(unsigned long long *out) {   // [64][12] ticks of 10 ns
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(brd::blk::g_cqr_st), sizeof(brd::blk::g_cqr_st));
}
#endif
