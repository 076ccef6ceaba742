// Stage 1 (dense -> band) kernels for gfx950 (MI355X / CDNA4).
//
// Replaces the reference's GPU band reduction cuda_brd_p1
// (svd_cuda_2.cu:1117-1220) and its per-column kernel chain
// (hh_kernel :221, wy_compact_cuda :838, qr_cuda :881, lq_cuda :959,
// qr_apply_cuda :1039, lq_apply_cuda :1081) with two kernels:
//
//   k_factor  Householder QR of one logical tile of <= kRmax rows x bk <= 32
//             columns, held in registers (one column per lane, 32 rows per
//             thread), one workgroup-wide reduction per column.  Produces V,
//             V^T and the compact-WY T factor (Q = I - V T V^T) in a
//             workspace and writes R (upper) / zeros back into the matrix.
//             A panel taller than kRmax rows is factored as a reduction tree:
//             leaves = row chunks, inner nodes = stacks of the children's R.
//   k_apply   X <- (I - V T^T V^T) X for one logical tile of <= kRmax rows x
//             kSlab columns staged in LDS; W = V^T X, W2 = T^T W and
//             X -= V W2 on the matrix cores (v_mfma_f64_16x16x4_f64 /
//             v_mfma_f32_16x16x4_f32).
//
// Both kernels read the matrix through a "logical view": element (r,c) is
// base[r*ld + c] (TR = false, QR of a column panel / left update) or
// base[c*ld + r] (TR = true, LQ of a row panel / right update as the
// transposed left update).  See DESIGN.md "Stage 1".
#include "brd_internal.h"

namespace brd {

// --------------------------------------------------------------------------
// MFMA wrappers.  Both shapes are 16x16x4 with one operand element per lane:
//   A operand lane l: A[m = l&15][k = l>>4],  B operand lane l: B[k = l>>4][n = l&15].
// C/D accumulators: we always use "register g of lane l holds logical row
// (l>>4) + 4g, column l&15".  That is the native f64 layout; for f32 the
// hardware's D row index is 4*(l>>4)+g, so we relabel rows: the A operand
// lane l then supplies logical row arow(l) = ((l&15)>>2) + 4*((l&15)&3).
// --------------------------------------------------------------------------
template <typename T> struct Mfma;
template <> struct Mfma<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(double a, double b, v4 c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int arow(int l) { return l & 15; }
};
template <> struct Mfma<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(float a, float b, v4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int arow(int l) {
        const int m = l & 15;
        return (m >> 2) + 4 * (m & 3);
    }
};

// --------------------------------------------------------------------------
// Reduction-tree row maps (host Tree / TreeLevel mirror, brd_api.cpp).
// --------------------------------------------------------------------------
struct LvArgs {
    int M, G0, bk, level, stride, F, nprev;
};

__device__ __forceinline__ int leaf_start(int g, const LvArgs &a) {
    return (int)(((long long)g * a.M) / a.G0);
}
__device__ __forceinline__ int group_nrows(int grp, const LvArgs &a) {
    if (a.level == 0) return leaf_start(grp + 1, a) - leaf_start(grp, a);
    int nch = min(a.F, a.nprev - grp * a.F);
    return nch * a.bk;
}
// Logical panel row of local row rr of group grp.
__device__ __forceinline__ int group_row(int rr, int grp, const LvArgs &a) {
    if (a.level == 0) return leaf_start(grp, a) + rr;
    const int q = rr / a.bk, t = rr - q * a.bk;
    return leaf_start((grp * a.F + q) * a.stride, a) + t;
}

template <bool TR, typename T>
__device__ __forceinline__ T *vptr(T *base, long ld, int r, int c) {
    return TR ? base + (long)c * ld + r : base + (long)r * ld + c;
}

// ==========================================================================
// k_factor: Householder QR of one tree node.
// 512 threads = 16 row groups (rg) x 32 columns (c); thread (rg,c) keeps
// rows rg, rg+16, ... of column c in registers.  Per column j one
// workgroup reduction yields G_c = sum_{i>j} X[i][j] X[i][c] for every c,
// from which the reflector, the projections w_c = v_j^T X[:,c] (c>j) and the
// inner products v_c^T v_j (c<j, for T) all follow.
// Columns are kept unscaled ("raw") while the panel is factored:
// v_j = X[:,j] / u1_j below the diagonal.
// ==========================================================================
constexpr int kQ = kRmax / 16;   // rows per thread
constexpr int kFS = 33;          // LDS row stride of the staging tile

template <typename T, bool TR>
__global__ void __launch_bounds__(512)
k_factor(T *__restrict__ base, long ld, LvArgs la, T *__restrict__ Vws, T *__restrict__ VTws,
         T *__restrict__ Tws)
{
    __shared__ T sX[kRmax * kFS];   // staging tile; during the column loop it
                                     // holds the broadcast column buffers instead
    __shared__ T sRed[2][8][32];
    __shared__ T sRow[2][32];
    __shared__ T sZ[32][33];
    __shared__ T sT[32][33];
    __shared__ T sU1[32], sTau[32];

    const int grp = blockIdx.x;
    const int tid = threadIdx.x;
    const int c = tid & 31, rg = tid >> 5, lane = tid & 63, w = tid >> 6;
    const int nr = group_nrows(grp, la);
    const int bk = la.bk;
    const int qn = (nr + 15) >> 4;

    // ---- stage the tile into registers ------------------------------------
    T xr[kQ];
    if (!TR) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = rg + 16 * q;
            T v = (T)0;
            if (q < qn && i < nr && c < bk) v = *vptr<false>(base, ld, group_row(i, grp, la), c);
            xr[q] = v;
        }
    } else {
        // coalesced: consecutive threads read consecutive logical rows (= physical columns)
        for (int r = tid; r < kRmax; r += 512) {
            const int pr = r < nr ? group_row(r, grp, la) : 0;
            for (int cc = 0; cc < 32; ++cc) {
                T v = (T)0;
                if (r < nr && cc < bk) v = *vptr<true>(base, ld, pr, cc);
                sX[r * kFS + cc] = v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kQ; ++q) xr[q] = sX[(rg + 16 * q) * kFS + c];
        __syncthreads();   // sX is reused for sCol below
    }

    const int kk = min(nr, bk);
    T colj[kQ];
    for (int j = 0; j < kk; ++j) {
        const int pb = j & 1;
        T *sColj = sX + pb * kRmax;   // broadcast buffer of column j (aliases sX)
        // (0) owner of column j publishes it to its own wave (same rg pair)
        if (c == j) {
#pragma unroll
            for (int q = 0; q < kQ; ++q)
                if (q < qn) sColj[rg + 16 * q] = xr[q];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // (1)+(2) partial G_c over this thread's rows i > j
        T p = (T)0;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = rg + 16 * q;
            T cv = (T)0;
            if (q < qn) cv = sColj[i];
            colj[q] = cv;
            if (q < qn && i > j && i < nr) p += cv * xr[q];
        }
        p += __shfl_xor(p, 32);
        if ((lane >> 5) == 0) sRed[pb][w][c] = p;
        if (rg == (j & 15)) {
            T rv = (T)0;
#pragma unroll
            for (int q = 0; q < kQ; ++q)
                if (q == (j >> 4)) rv = xr[q];
            sRow[pb][c] = rv;
        }
        __syncthreads();
        // (3) reflector (LAPACK-style: tau = 0 when the sub-column is 0)
        T Gc = (T)0, Gj = (T)0;
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) {
            Gc += sRed[pb][ww][c];
            Gj += sRed[pb][ww][j];
        }
        const T x0 = sRow[pb][j];
        T alpha = x0, u1 = (T)1, tau = (T)0;
        if (Gj != (T)0) {
            const T nrm = sqrt(x0 * x0 + Gj);
            alpha = x0 >= (T)0 ? -nrm : nrm;
            u1 = x0 - alpha;
            tau = -u1 / alpha;
        }
        const T inv_u1 = (T)1 / u1;
        const T wc = sRow[pb][c] + Gc * inv_u1;   // v_j^T X[:,c]  (c != j)
        if (c > j && c < bk) {
            const T tw = tau * wc;
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int i = rg + 16 * q;
                if (q < qn && i >= j && i < nr) {
                    const T v = (i == j) ? (T)1 : colj[q] * inv_u1;
                    xr[q] -= tw * v;
                }
            }
        } else if (c == j) {
            if (rg == (j & 15)) {
#pragma unroll
                for (int q = 0; q < kQ; ++q)
                    if (q == (j >> 4)) xr[q] = alpha;
            }
            if (rg == 0) { sU1[j] = u1; sTau[j] = tau; }
        } else if (c < j && rg == 0) {
            sZ[c][j] = wc / sU1[c];               // v_c^T v_j
        }
    }
    __syncthreads();

    // ---- T factor (LAPACK larft, forward/columnwise): lane a owns row a ----
    if (tid < 32) {
        const int a = tid;
        for (int j = 0; j < 32; ++j) {
            T v = (T)0;
            if (j < kk) {
                if (a < j) {
                    T s = (T)0;
                    for (int cc = a; cc < j; ++cc) s += sT[a][cc] * sZ[cc][j];
                    v = -sTau[j] * s;
                } else if (a == j) {
                    v = sTau[j];
                }
            }
            sT[a][j] = v;
        }
    }
    // ---- everything back into LDS for coalesced output --------------------
#pragma unroll
    for (int q = 0; q < kQ; ++q) sX[(rg + 16 * q) * kFS + c] = xr[q];
    __syncthreads();

    T *V = Vws + (size_t)grp * kRmax * 32;
    T *VT = VTws + (size_t)grp * 32 * kRmax;
    T *Tm = Tws + (size_t)grp * 32 * 32;
    // V (kRmax x 32, row-major) -- thread (rg, c)
    for (int i = rg; i < kRmax; i += 16) {
        T v = (T)0;
        if (c < kk && i < nr) v = i < c ? (T)0 : (i == c ? (T)1 : sX[i * kFS + c] / sU1[c]);
        V[(size_t)i * 32 + c] = v;
    }
    // VT (32 x kRmax) -- thread = row
    for (int i = tid; i < kRmax; i += 512) {
        for (int cc = 0; cc < 32; ++cc) {
            T v = (T)0;
            if (cc < kk && i < nr) v = i < cc ? (T)0 : (i == cc ? (T)1 : sX[i * kFS + cc] / sU1[cc]);
            VT[(size_t)cc * kRmax + i] = v;
        }
    }
    for (int e = tid; e < 32 * 32; e += 512) Tm[e] = sT[e >> 5][e & 31];
    // R (upper) and zeros back into the matrix
    if (!TR) {
        for (int i = rg; i < nr; i += 16) {
            if (c < bk) *vptr<false>(base, ld, group_row(i, grp, la), c) = (c >= i) ? sX[i * kFS + c] : (T)0;
        }
    } else {
        for (int i = tid; i < nr; i += 512) {
            const int pr = group_row(i, grp, la);
            for (int cc = 0; cc < bk; ++cc) *vptr<true>(base, ld, pr, cc) = (cc >= i) ? sX[i * kFS + cc] : (T)0;
        }
    }
}

// ==========================================================================
// k_apply: X <- X - V (T^T (V^T X)) on one tile: rows = one tree node's row
// list (<= kRmax), columns = one kSlab-wide slab of the trailing matrix.
// 512 threads = 8 waves.  LDS image of the tile:
//   TR = false: [row][col ^ 16*(row&1)]  (row stride 32)
//   TR = true:  [col][row] with row stride kRmax + 2
// both conflict-free for the MFMA fragment reads (a half-wave touches rows
// r, r+1 x 16 columns).
// ==========================================================================
constexpr int kPT = kRmax + 2;

template <bool TR>
__device__ __forceinline__ int xidx(int r, int c) {
    return TR ? c * kPT + r : r * 32 + (c ^ ((r & 1) << 4));
}

template <typename T, bool TR>
__global__ void __launch_bounds__(512)
k_apply(T *__restrict__ base, long ld, LvArgs la, int ncols, const T *__restrict__ Vws,
        const T *__restrict__ VTws, const T *__restrict__ Tws)
{
    typedef typename Mfma<T>::v4 v4;
    __shared__ T sX[32 * kPT];
    __shared__ T sW[32][33];
    __shared__ T sW2[32][33];
    __shared__ T sRed[4][256];

    const int grp = blockIdx.x, slab = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l15 = lane & 15;
    const int nr = group_nrows(grp, la);
    const int nrp = (nr + 15) & ~15;
    const int nblk = nrp >> 4;
    const int c0 = slab * kSlab;
    const int nc = min(kSlab, ncols - c0);
    const T *V = Vws + (size_t)grp * kRmax * 32;
    const T *VT = VTws + (size_t)grp * 32 * kRmax;
    const T *Tm = Tws + (size_t)grp * 32 * 32;
    const int ksteps = (la.bk + 3) >> 2;   // V/VT/T are zero beyond bk

    // ---- 1. stage the tile (rows < nrp; zero padding) ---------------------
    if (!TR) {
        const int cc = tid & 31;
        for (int r = tid >> 5; r < nrp; r += 16) {
            T v = (T)0;
            if (r < nr && cc < nc) v = *vptr<false>(base, ld, group_row(r, grp, la), c0 + cc);
            sX[xidx<false>(r, cc)] = v;
        }
    } else {
        for (int r = tid; r < nrp; r += 512) {
            const int pr = r < nr ? group_row(r, grp, la) : 0;
            for (int cc = 0; cc < 32; ++cc) {
                T v = (T)0;
                if (r < nr && cc < nc) v = *vptr<true>(base, ld, pr, c0 + cc);
                sX[xidx<true>(r, cc)] = v;
            }
        }
    }
    __syncthreads();

    // ---- 2. W = V^T X  (32 x 32 = 4 MFMA tiles, K split over 2 wave halves) -
    {
        const int tile = w & 3, half = w >> 2;
        const int ab = tile >> 1, cb = tile & 1;
        const int nb2 = (nblk + 1) >> 1;
        const int b0 = half * nb2, b1 = min(nblk, b0 + nb2);
        v4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        const int acol = ab * 16 + Mfma<T>::arow(lane);
        const int xcol = cb * 16 + l15;
        for (int blk = b0; blk < b1; ++blk) {
#pragma unroll
            for (int s = 0; s < 4; s += 2) {
                const int r0 = blk * 16 + q + 4 * s;
                const int r1 = r0 + 4;
                acc0 = Mfma<T>::mma(V[(size_t)r0 * 32 + acol], sX[xidx<TR>(r0, xcol)], acc0);
                acc1 = Mfma<T>::mma(V[(size_t)r1 * 32 + acol], sX[xidx<TR>(r1, xcol)], acc1);
            }
        }
        v4 acc = acc0 + acc1;
        if (half == 1) {
#pragma unroll
            for (int g = 0; g < 4; ++g) sRed[tile][lane * 4 + g] = acc[g];
        }
        __syncthreads();
        if (half == 0) {
#pragma unroll
            for (int g = 0; g < 4; ++g) sW[ab * 16 + q + 4 * g][cb * 16 + l15] = acc[g] + sRed[tile][lane * 4 + g];
        }
        __syncthreads();
    }
    // ---- 3. W2 = -(T^T W) --------------------------------------------------
    if (w < 4) {
        const int ab = w >> 1, cb = w & 1;
        v4 acc = {0, 0, 0, 0};
        const int acol = ab * 16 + Mfma<T>::arow(lane);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int k = 4 * s + q;
            acc = Mfma<T>::mma(Tm[k * 32 + acol], sW[k][cb * 16 + l15], acc);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) sW2[ab * 16 + q + 4 * g][cb * 16 + l15] = -acc[g];
    }
    __syncthreads();
    // ---- 4. X += V W2 (64 MFMA tiles, wave w: row blocks w, w+8, ...) ------
    {
        T bw[2][8];
#pragma unroll
        for (int cb = 0; cb < 2; ++cb)
#pragma unroll
            for (int s = 0; s < 8; ++s) bw[cb][s] = sW2[4 * s + q][cb * 16 + l15];
        for (int blk = w; blk < nblk; blk += 8) {
            const int arr = blk * 16 + Mfma<T>::arow(lane);
            T av[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) av[s] = (s < ksteps) ? VT[(size_t)(4 * s + q) * kRmax + arr] : (T)0;
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
                const int col = cb * 16 + l15;
                v4 acc;
#pragma unroll
                for (int g = 0; g < 4; ++g) acc[g] = sX[xidx<TR>(blk * 16 + q + 4 * g, col)];
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s < ksteps) acc = Mfma<T>::mma(av[s], bw[cb][s], acc);
#pragma unroll
                for (int g = 0; g < 4; ++g) sX[xidx<TR>(blk * 16 + q + 4 * g, col)] = acc[g];
            }
        }
    }
    __syncthreads();
    // ---- 5. write back -----------------------------------------------------
    if (!TR) {
        const int cc = tid & 31;
        if (cc < nc)
            for (int r = tid >> 5; r < nr; r += 16)
                *vptr<false>(base, ld, group_row(r, grp, la), c0 + cc) = sX[xidx<false>(r, cc)];
    } else {
        for (int r = tid; r < nr; r += 512) {
            const int pr = group_row(r, grp, la);
            for (int cc = 0; cc < nc; ++cc) *vptr<true>(base, ld, pr, c0 + cc) = sX[xidx<true>(r, cc)];
        }
    }
}

// --------------------------------------------------------------------------
// Host launchers
// --------------------------------------------------------------------------
static LvArgs lv_args(const Tree &t, int level) {
    LvArgs a;
    a.M = t.M;
    a.G0 = t.G0;
    a.bk = t.bk;
    a.level = level;
    a.stride = t.lv[level].stride;
    a.F = t.F;
    a.nprev = level > 0 ? t.lv[level - 1].groups : 0;
    return a;
}

template <typename T>
hipError_t launch_factor(bool trans, T *base, long ld, const Tree &t, int level, const TreeWs &ws,
                         hipStream_t s)
{
    LvArgs a = lv_args(t, level);
    dim3 grid(t.lv[level].groups), block(512);
    T *V = (T *)ws.V[level], *VT = (T *)ws.VT[level], *Tm = (T *)ws.T[level];
    if (trans)
        hipLaunchKernelGGL((k_factor<T, true>), grid, block, 0, s, base, ld, a, V, VT, Tm);
    else
        hipLaunchKernelGGL((k_factor<T, false>), grid, block, 0, s, base, ld, a, V, VT, Tm);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_apply(bool trans, T *base, long ld, const Tree &t, int level, int ncols,
                        const TreeWs &ws, hipStream_t s)
{
    if (ncols <= 0) return hipSuccess;
    LvArgs a = lv_args(t, level);
    dim3 grid(t.lv[level].groups, (ncols + kSlab - 1) / kSlab), block(512);
    const T *V = (const T *)ws.V[level], *VT = (const T *)ws.VT[level], *Tm = (const T *)ws.T[level];
    if (trans)
        hipLaunchKernelGGL((k_apply<T, true>), grid, block, 0, s, base, ld, a, ncols, V, VT, Tm);
    else
        hipLaunchKernelGGL((k_apply<T, false>), grid, block, 0, s, base, ld, a, ncols, V, VT, Tm);
    return hipGetLastError();
}

template hipError_t launch_factor<double>(bool, double *, long, const Tree &, int, const TreeWs &, hipStream_t);
template hipError_t launch_factor<float>(bool, float *, long, const Tree &, int, const TreeWs &, hipStream_t);
template hipError_t launch_apply<double>(bool, double *, long, const Tree &, int, int, const TreeWs &, hipStream_t);
template hipError_t launch_apply<float>(bool, float *, long, const Tree &, int, int, const TreeWs &, hipStream_t);

}  // namespace brd
