// Blocked stage 1: the read passes k_rpass (Y = A^T V, X = A U, split-K on the
// matrix cores) and the virtual tile's partial sum k_vsum (gfx950).
#include "brd_blk.h"

namespace brd {
namespace blk {

// ==========================================================================
// k_rpass: D = B^T S (Y pass) or S B (X pass) for a tall "skinny" operand B
// (K x 32) and a source S, summed over one split of the K range.
//   Y pass (YP): S(k, m) = src[k*ld + m] (row-major A, k = rows, m = columns),
//                D[t][m] = sum_k B[k][t] S(k, m); partials stored [split][t][m].
//   X pass     : S(k, m) = src[m*ld + k] (k = columns, m = rows),
//                D[m][t] = sum_k S(k, m) B[k][t]; partials stored [split][m][t].
// B(k, t) = bsrc[k*bld + t] in both.  Every wave streams its own 64 values of
// m straight from HBM into MFMA operand registers (no LDS, no barriers):
//   Y: one 16-byte load per lane and 4 rows gives 2 x 16 columns (even / odd
//      column tiles), 4 rows x 256 contiguous bytes per instruction;
//   X: one 16-byte load per lane gives 2 k of one row: 16 rows x 64 bytes per
//      instruction, two K steps each;
// with kSU steps of loads in flight (static register ring).  The "virtual"
// workgroups (the first ksplit of the grid) compute the same product with
// S = vsrc (256 wide); they meet at a counter and each sums one slice of
// their partials into vout in fixed order (deterministic).
// ==========================================================================
template <typename T, bool YP, typename FA>
__global__ void __launch_bounds__(kRT, 1) k_rpass(RpArgs a, FA fin) {
    typedef typename G2<T>::v2 v2;
    typedef typename Mf<T>::v4 v4;
    const int tid = threadIdx.x, lane = tid & 63, w = (tid >> 6) & 3, kh = tid >> 8;
    const int q = lane >> 4, l15 = lane & 15;
    // one LDS block for the K halves' reduction and (workgroup 0) cqr_finish:
    // 64 KB, so two workgroups share a CU
    __shared__ __attribute__((aligned(16))) double rp_lds[kRpLds];
    if (a.has_fin && blockIdx.x == 0) {   // the previous panel's LU, T and R signs, beside the pass
        cqr_finish_entry<T>(fin, tid, rp_lds);
        return;
    }
    const int bid = blockIdx.x - a.has_fin;
    const bool virt = bid < a.nvirt;
    int mx, ks;
    if (virt) { mx = 0; ks = bid; }
    else      { const int r = bid - a.nvirt; mx = r % a.mtiles; ks = r / a.mtiles; }
    const T *S;
    long ld;
    int M;
    if (virt) { S = (const T *)a.vsrc; ld = a.vld; M = kMT; }
    else      { S = (const T *)a.src + (YP ? (long)mx * kMT : (long)mx * kMT * a.ld); ld = a.ld; M = min(kMT, a.M - mx * kMT); }
    const T *B = (const T *)a.bsrc;
    // waves w and w + 4 take the two halves of the workgroup's K range (in
    // whole 8-row step pairs) and meet in LDS: two waves per SIMD in flight
    const int kb0 = ks * a.kper, ke0 = min(a.K, kb0 + a.kper);
    const int khalf = ke0 > kb0 ? ((ke0 - kb0 + 15) / 16) * 8 : 0;
    const int kbeg = kh ? min(ke0, kb0 + khalf) : kb0, kend = kh ? ke0 : min(ke0, kb0 + khalf);
    const int mb = kWM * w;
    v4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = v4{0, 0, 0, 0};

    if constexpr (YP) {
        // acc[h*4 + p*2 + e]: t-half h, column pair group p (32 columns), parity e
        const int nst = kend > kbeg ? (kend - kbeg + 3) / 4 : 0;
        v2 ra[kSU][2];
        T rb[kSU][2];
        auto load = [&](int s, v2 (&va)[2], T (&vb)[2]) {
            const int k = kbeg + 4 * s + q;
            const bool kv = k < kend;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int m = mb + 32 * p + 2 * l15;
                v2 v = {(T)0, (T)0};
                if (kv && m < M) {
                    const T *src = S + (long)k * ld + m;
                    if (m + 1 < M) v = *(const v2 *)src; else v.x = src[0];
                }
                va[p] = v;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) vb[h] = kv ? B[(long)k * a.bld + 16 * h + l15] : (T)0;
        };
#pragma unroll
        for (int u = 0; u < kSU; ++u)
            if (u < nst) load(u, ra[u], rb[u]);
        for (int s0 = 0; s0 < nst; s0 += kSU) {
#pragma unroll
            for (int u = 0; u < kSU; ++u) {
                const int s = s0 + u;
                if (s < nst) {
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int p = 0; p < 2; ++p) {
                            acc[h * 4 + p * 2 + 0] = Mf<T>::mma(rb[u][h], ra[u][p].x, acc[h * 4 + p * 2 + 0]);
                            acc[h * 4 + p * 2 + 1] = Mf<T>::mma(rb[u][h], ra[u][p].y, acc[h * 4 + p * 2 + 1]);
                        }
                    if (s + kSU < nst) load(s + kSU, ra[u], rb[u]);
                }
            }
        }
    } else {
        // acc[p*2 + h]: row tile p (16 rows), t-half h; one step pair = 8 k
        const int npr = kend > kbeg ? (kend - kbeg + 7) / 8 : 0;
        constexpr int kSP2 = kSU / 2;
        v2 ra[kSP2][4];
        T rb[kSP2][2][2];
        auto load = [&](int s2, v2 (&va)[4], T (&vb)[2][2]) {
            const int k = kbeg + 8 * s2 + 2 * q;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int m = mb + 16 * p + l15;
                v2 v = {(T)0, (T)0};
                if (m < M && k < kend) {
                    const T *src = S + (long)m * ld + k;
                    if (k + 1 < kend) v = *(const v2 *)src; else v.x = src[0];
                }
                va[p] = v;
            }
#pragma unroll
            for (int e = 0; e < 2; ++e)
#pragma unroll
                for (int h = 0; h < 2; ++h) vb[e][h] = (k + e < kend) ? B[(long)(k + e) * a.bld + 16 * h + l15] : (T)0;
        };
#pragma unroll
        for (int u = 0; u < kSP2; ++u)
            if (u < npr) load(u, ra[u], rb[u]);
        for (int s0 = 0; s0 < npr; s0 += kSP2) {
#pragma unroll
            for (int u = 0; u < kSP2; ++u) {
                const int s2 = s0 + u;
                if (s2 < npr) {
#pragma unroll
                    for (int p = 0; p < 4; ++p)
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            acc[p * 2 + h] = Mf<T>::mma(ra[u][p].x, rb[u][0][h], acc[p * 2 + h]);
                            acc[p * 2 + h] = Mf<T>::mma(ra[u][p].y, rb[u][1][h], acc[p * 2 + h]);
                        }
                    if (s2 + kSP2 < npr) load(s2 + kSP2, ra[u], rb[u]);
                }
            }
        }
    }

    // ---- the second half's sums into the first half's, fixed order ----------
    {
        T (*red)[32][64] = reinterpret_cast<T (*)[32][64]>(rp_lds);
        if (kh) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) red[w][4 * i + g][lane] = acc[i][g];
        }
        __syncthreads();
        if (!kh) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) acc[i][g] += red[w][4 * i + g][lane];
        }
    }
    // ---- partials ----------------------------------------------------------
    T *out;
    long mp;
    if (virt) { out = (T *)a.vpart + (size_t)ks * 32 * kMT; mp = kMT; }
    else      { out = (T *)a.part + (size_t)ks * 32 * a.mp + (size_t)mx * kMT * (YP ? 1 : 32); mp = a.mp; }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (kh) break;
            const int r = Mf<T>::crow(q, g);
            if (YP) {
                const int h = i >> 2, p = (i >> 1) & 1, e = i & 1;
                const int t = 16 * h + r, m = mb + 32 * p + 2 * l15 + e;
                if (m < M) out[(size_t)t * mp + m] = acc[i][g];
            } else {
                const int p = i >> 1, h = i & 1;
                const int m = mb + 16 * p + r, t = 16 * h + l15;
                if (m < M) out[(size_t)m * 32 + t] = acc[i][g];
            }
        }
}

// The virtual tile's split-K partials summed in fixed order (one element per
// thread, every partial's load in flight at once): a kernel of its own, so
// no workgroup of the read pass waits for another.
// Workgroup 0 also patches the diagonal of the finished panel's top block
// from V' = Q to V = Q - S (pbase[t (pstride)] -= s_t), read from here on.
template <typename T>
__global__ void __launch_bounds__(256) k_vsum(const T *vpart, T *vout, int nvirt, T *pbase, long pstride,
                                              const double *sgn) {
    const int e = blockIdx.x * 256 + threadIdx.x;   // < 32 kMT
    if (blockIdx.x == 0 && threadIdx.x < 32 && pbase)
        pbase[(size_t)threadIdx.x * pstride] = (T)((double)pbase[(size_t)threadIdx.x * pstride] - sgn[threadIdx.x]);
    T v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = vpart[(size_t)min(k, nvirt - 1) * 32 * kMT + e];
    T s = v[0];
#pragma unroll
    for (int k = 1; k < 32; ++k)
        if (k < nvirt) s += v[k];
    vout[e] = s;
}

template <typename T>
void launch_k_rpass(bool yp, dim3 grid, const RpArgs &a, const FinArgs &f, hipStream_t s, double fl, double by) {
    if (yp) blk_launch("s1_rpass", fl, by, k_rpass<T, true, FinArgs>, grid, dim3(kRT), s, a, f);
    else    blk_launch("s1_rpass", fl, by, k_rpass<T, false, FinArgs>, grid, dim3(kRT), s, a, f);
}
template <typename T>
void launch_k_vsum(const T *vpart, T *vout, int nvirt, T *pbase, long pstride, const double *sgn, hipStream_t s) {
    blk_launch("s1_prep", 0.0, 0.0, k_vsum<T>, dim3(32 * kMT / 256), dim3(256), s, vpart, vout, nvirt, pbase, pstride,
               sgn);
}
template void launch_k_rpass<double>(bool, dim3, const RpArgs &, const FinArgs &, hipStream_t, double, double);
template void launch_k_rpass<float>(bool, dim3, const RpArgs &, const FinArgs &, hipStream_t, double, double);
template void launch_k_vsum<double>(const double *, double *, int, double *, long, const double *, hipStream_t);
template void launch_k_vsum<float>(const float *, float *, int, float *, long, const double *, hipStream_t);

}  // namespace blk
}  // namespace brd
