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
//   k_apply   X <- (I - V T^T V^T) X for one tree node (<= kRmax rows) and a
//             run of 16-column slabs of the trailing matrix.  The
//             node's V stays in registers (MFMA fragments) for the whole run,
//             each slab is staged through LDS while the next one is already
//             in flight, and W = V^T X, W2 = T^T W, X -= V W2 run on the
//             matrix cores (v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32).
//
// Both kernels read the matrix through a "logical view": element (r,c) is
// base[r*ld + c] (TR = false: QR of a column panel / left update) or
// base[c*ld + r] (TR = true: LQ of a row panel / the right update written
// as a left update of the transpose).  See DESIGN.md "Stage 1".
#include "brd_internal.h"

#include <algorithm>

namespace brd {

#ifdef BRD_STAMPS
// Debug build only (make STAMPS=1): per-phase s_memtime stamps of workgroup 0.
__device__ unsigned long long g_stamps[64];
#define STAMP(k)                                                                   \
    do {                                                                           \
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                \
            g_stamps[k] = __builtin_amdgcn_s_memtime();                            \
    } while (0)
hipError_t read_stamps(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps));
}
#else
#define STAMP(k) do {} while (0)
#endif

// --------------------------------------------------------------------------
// MFMA wrappers.  Both shapes are 16x16x4 with one operand element per lane:
//   A operand lane l: A[m = l&15][k = l>>4],  B operand lane l: B[k = l>>4][n = l&15].
// C/D accumulators: "register g of lane l holds logical row (l>>4) + 4g,
// column l&15".  That is the native f64 layout; for f32 the hardware's D row
// index is 4*(l>>4)+g, so rows are relabelled: the A operand lane l then
// supplies logical row arow(l) = ((l&15)>>2) + 4*((l&15)&3).
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
    return (int)(((unsigned)g * (unsigned)a.M) / (unsigned)a.G0);
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

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ==========================================================================
// k_factor: Householder QR of one tree node.
// 512 threads = 16 row groups (rg) x 32 columns (c); thread (rg,c) keeps
// rows rg, rg+16, ... of column c in registers (rows >= nr are zero).  Per
// column j one workgroup reduction yields G_c = sum_{i>j} X[i][j] X[i][c] for
// every c, from which the reflector, the projections w_c = v_j^T X[:,c]
// (c > j) and the inner products v_c^T v_j (c < j, for T) all follow.
// Columns are kept unscaled ("raw") while the panel is factored:
// v_j = X[:,j] / u1_j below the diagonal.
// ==========================================================================
constexpr int kFT = 512;         // threads per factor workgroup
constexpr int kRG = kFT / 32;    // row groups
constexpr int kQ = kRmax / kRG;  // rows per thread
constexpr int kFS = 33;          // LDS row stride of the staging tile

// Row j < 32 of the tile lives in register slot j / kRG, i.e. slot 0 or 1:
// two-way selects keep every register index static (no scratch).
static_assert(kRG >= 16, "row j < 32 must live in register slot 0 or 1");
template <typename T, int N>
__device__ __forceinline__ T slot01_get(const T (&x)[N], int q) { return q == 0 ? x[0] : x[1]; }
template <typename T, int N>
__device__ __forceinline__ void slot01_set(T (&x)[N], int q, T v) {
    if (q == 0) x[0] = v; else x[1] = v;
}

template <typename T, bool TR>
__global__ void __launch_bounds__(kFT)
k_factor(T *__restrict__ base, long ld, LvArgs la, T *__restrict__ Vws, T *__restrict__ VTws,
         T *__restrict__ Tws)
{
    __shared__ T sX[kRmax * kFS];   // staging tile; during the column loop it
                                     // holds the broadcast column buffers instead
    __shared__ T sRed[2][kFT / 64][32];
    __shared__ T sRow[2][32];
    __shared__ T sZ[32][33];
    __shared__ T sT[32][33];
    __shared__ T sU1[32], sTau[32];
    __shared__ int sMap[kRmax];

    const int grp = blockIdx.x;
    const int tid = threadIdx.x;
    const int c = tid & 31, rg = tid >> 5, lane = tid & 63, w = tid >> 6;
    const int nr = group_nrows(grp, la);
    const int bk = la.bk;
    const int kk = min(nr, bk);
    STAMP(0);

    if (tid < nr) sMap[tid] = group_row(tid, grp, la);
    for (int e = tid; e < 32 * 33; e += kFT) {
        (&sZ[0][0])[e] = (T)0;
        (&sT[0][0])[e] = (T)0;
    }
    if (tid < 32) { sU1[tid] = (T)1; sTau[tid] = (T)0; }   // sU1: 1/u1 per column
    __syncthreads();

    // ---- stage the tile into registers ------------------------------------
    STAMP(1);
    T xr[kQ];
    if (!TR) {
        T tmp[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = rg + kRG * q;
            const bool ok = i < nr && c < bk;
            const int pr = ok ? sMap[i] : 0;
            tmp[q] = ok ? *vptr<false>(base, ld, pr, c) : (T)0;
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) xr[q] = tmp[q];
    } else {
        // coalesced: consecutive threads read consecutive logical rows (= physical columns)
        const int r = tid % kRmax;
        const bool rok = r < nr;
        const int pr = rok ? sMap[r] : 0;
#pragma unroll
        for (int h = tid / kRmax; h < 2; h += kFT / kRmax) {
            T tmp[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int cc = h * 16 + k;
                tmp[k] = (rok && cc < bk) ? *vptr<true>(base, ld, pr, cc) : (T)0;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) sX[r * kFS + h * 16 + k] = tmp[k];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kQ; ++q) xr[q] = sX[(rg + kRG * q) * kFS + c];
        __syncthreads();   // sX is reused for the column buffers below
    }

    STAMP(2);
    T colj[kQ];
    for (int j = 0; j < kk; ++j) {
        const int pb = j & 1;
        const int jq = j / kRG, jr = j % kRG;      // row j = (rg jr, slot jq)
        T *sColj = sX + pb * kRmax;   // column j below the diagonal, zero elsewhere
        if (j == 1) STAMP(3);
        // (0) the owner of column j publishes its sub-diagonal part to its own wave
        if (c == j) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) sColj[rg + kRG * q] = (rg + kRG * q > j) ? xr[q] : (T)0;
        }
        wave_sync();
        // (1) partial G_c = sum_{i>j} X[i][j] X[i][c] over this thread's rows
        //     (four independent chains)
        T p4[4] = {(T)0, (T)0, (T)0, (T)0};
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            colj[q] = sColj[rg + kRG * q];
            p4[q & 3] = fma(colj[q], xr[q], p4[q & 3]);
        }
        T p = (p4[0] + p4[1]) + (p4[2] + p4[3]);
        p += __shfl_xor(p, 32);
        if ((lane >> 5) == 0) sRed[pb][w][c] = p;
        if (rg == jr) sRow[pb][c] = slot01_get(xr, jq);
        __syncthreads();
        // (2) reflector (LAPACK-style: tau = 0 when the sub-column is zero)
        T Gc, Gj;
        {
            T gc[kFT / 64], gj[kFT / 64];
#pragma unroll
            for (int ww = 0; ww < kFT / 64; ++ww) { gc[ww] = sRed[pb][ww][c]; gj[ww] = sRed[pb][ww][j]; }
#pragma unroll
            for (int h = kFT / 128; h >= 1; h >>= 1)
#pragma unroll
                for (int ww = 0; ww < h; ++ww) { gc[ww] += gc[ww + h]; gj[ww] += gj[ww + h]; }
            Gc = gc[0];
            Gj = gj[0];
        }
        const T x0 = sRow[pb][j];
        T alpha = x0, u1 = (T)1, tau = (T)0;
        if (Gj != (T)0) {
            const T nrm = sqrt(fma(x0, x0, Gj));
            alpha = x0 >= (T)0 ? -nrm : nrm;
            u1 = x0 - alpha;
            tau = -u1 / alpha;
        }
        const T inv_u1 = (T)1 / u1;
        const T wc = fma(Gc, inv_u1, sRow[pb][c]);      // v_j^T X[:,c]  (c != j)
        // (3) rank-1 update of the columns right of j: X[i][c] -= tau w_c v_i
        if (c > j && c < bk) {
            const T tw = tau * wc, twu = tw * inv_u1;
#pragma unroll
            for (int q = 0; q < kQ; ++q) xr[q] = fma(-twu, colj[q], xr[q]);   // rows i > j
            if (rg == jr) slot01_set(xr, jq, slot01_get(xr, jq) - tw);         // row j (v_j = 1)
        } else if (c == j) {
            if (rg == jr) slot01_set(xr, jq, alpha);
            if (rg == 0) { sU1[j] = inv_u1; sTau[j] = tau; }
        } else if (c < j && rg == 0) {
            sZ[c][j] = wc * sU1[c];                      // v_c^T v_j  (sU1 holds 1/u1)
        }
    }
    __syncthreads();
    STAMP(4);

    // ---- T (LAPACK larft): T[:, j] = -tau_j T[:, :j] (V^T v_j)[:j], T[j][j] = tau_j
    // Lane a of wave 0 keeps row a of T in registers (fully unrolled, static
    // indices); z = V^T V (strict upper part) is read from sZ as broadcasts.
    T *Tm = Tws + (size_t)grp * 32 * 32;
    if (tid < 32) {
        const int a = tid;
        T trow[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            T s = (T)0;
#pragma unroll
            for (int cc = 0; cc < j; ++cc) s = fma(trow[cc], sZ[cc][j], s);
            const T tj = j < kk ? sTau[j] : (T)0;
            trow[j] = a < j ? -tj * s : (a == j ? tj : (T)0);
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) sT[a][j] = trow[j];
    }
    STAMP(5);
    // ---- outputs ------------------------------------------------------------
    T *V = Vws + (size_t)grp * kRmax * 32;
    T *VT = VTws + (size_t)grp * 32 * kRmax;
    const int nrp = (nr + 15) & ~15;
    const T iu = sU1[c];
    // V (kRmax x 32, row-major, rows < nrp) from registers; scaled copy to LDS for VT
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
        const int i = rg + kRG * q;
        T v = (T)0;
        if (c < kk && i < nr) v = i < c ? (T)0 : (i == c ? (T)1 : xr[q] * iu);
        if (i < nrp) V[(size_t)i * 32 + c] = v;
        sX[i * kFS + c] = v;
    }
    // R (upper) and zeros back into the matrix (TR=false straight from registers)
    if (!TR) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int i = rg + kRG * q;
            if (i < nr && c < bk) *vptr<false>(base, ld, sMap[i], c) = (c >= i) ? xr[q] : (T)0;
        }
    }
    __syncthreads();
    for (int e = tid; e < 32 * 32; e += kFT) Tm[e] = sT[e >> 5][e & 31];
    // VT (32 x kRmax) -- consecutive threads -> consecutive rows, coalesced
    {
        const int i = tid % kRmax;
        if (i < nrp) {
            for (int h = tid / kRmax; h < 2; h += kFT / kRmax) {
#pragma unroll
                for (int k = 0; k < 16; ++k) VT[(size_t)(16 * h + k) * kRmax + i] = sX[i * kFS + 16 * h + k];
            }
        }
    }
    if (TR) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kQ; ++q) sX[(rg + kRG * q) * kFS + c] = xr[q];
        __syncthreads();
        const int i = tid % kRmax;
        if (i < nr) {
            const int pr = sMap[i];
            for (int h = tid / kRmax; h < 2; h += kFT / kRmax) {
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int cc = 16 * h + k;
                    if (cc < bk) *vptr<true>(base, ld, pr, cc) = (cc >= i) ? sX[i * kFS + cc] : (T)0;
                }
            }
        }
    }
    STAMP(6);
}

// ==========================================================================
// k_apply: X <- X - V (T^T (V^T X)) for one tree node (rows = the node's row
// list, <= kRmax) and a run of kASlab-wide column slabs.
// 512 threads = 8 waves; wave w owns the 16-row blocks w, w+8, w+16, w+24.
// Registers: the node's V as MFMA fragments in both orientations (A operand
// of V^T for W, A operand of V for the update) for the whole run, and the
// next slab in flight.  LDS: the current slab, W (summed across waves with
// ds_add), W2, T.  LDS slab image:
//   TR = false: [row][16 cols]   (a half-wave's rows r, r+1 fall on disjoint banks)
//   TR = true:  [col][row] with row stride kRmax + 2
// both conflict-free for the fragment reads (a half-wave reads rows r, r+1
// x 16 columns) and for the coalesced global<->LDS copies.
// ==========================================================================
constexpr int kPT = kRmax + 2;
constexpr int kASlab = 16;                  // columns per slab
constexpr int kAT = 512;                    // threads per apply workgroup
constexpr int kAW = kAT / 64;               // waves
constexpr int kAB = (kRmax / 16) / kAW;     // 16-row blocks per wave
constexpr int kXN = kRmax * kASlab / kAT;   // slab elements staged per thread

template <bool TR>
__device__ __forceinline__ int xidx(int r, int c) {
    return TR ? c * kPT + r : r * kASlab + c;
}

// Workgroup barrier that orders LDS only.  __syncthreads() would also wait
// for every outstanding global load (vmcnt(0)) and so drain the next slab's
// prefetch at the first barrier of the slab.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Slab staging.  TR = false: thread -> column tid%16, rows tid/16 + 32p.
// TR = true: thread -> row tid (< kRmax), all 16 columns.
template <typename T, bool TR>
__device__ __forceinline__ void slab_load(const T *base, long ld, const int *sMap, int nr, int c0, int nc,
                                          int tid, T (&xn)[kXN]) {
    if (!TR) {
        const int cc = tid & (kASlab - 1);
#pragma unroll
        for (int p = 0; p < kXN; ++p) {
            const int r = (tid / kASlab) + (kAT / kASlab) * p;
            const bool ok = r < nr && cc < nc;
            const int pr = ok ? sMap[r] : 0;
            xn[p] = ok ? base[(long)pr * ld + c0 + cc] : (T)0;
        }
    } else {
        const int r = tid;
        const bool rok = r < nr;
        const int pr = rok ? sMap[r] : 0;
#pragma unroll
        for (int k = 0; k < kXN; ++k) xn[k] = (rok && k < nc) ? base[(long)(c0 + k) * ld + pr] : (T)0;
    }
}

template <typename T, bool TR>
__device__ __forceinline__ void slab_to_lds(T *sX, int nrp, int tid, const T (&xn)[kXN]) {
    if (!TR) {
        const int cc = tid & (kASlab - 1);
#pragma unroll
        for (int p = 0; p < kXN; ++p) {
            const int r = (tid / kASlab) + (kAT / kASlab) * p;
            if (r < nrp) sX[xidx<false>(r, cc)] = xn[p];
        }
    } else {
        const int r = tid;
        if (r < nrp) {
#pragma unroll
            for (int k = 0; k < kXN; ++k) sX[xidx<true>(r, k)] = xn[k];
        }
    }
}

template <typename T, bool TR>
__global__ void __launch_bounds__(kAT)
k_apply(T *__restrict__ base, long ld, LvArgs la, int ncols, int spw, const T *__restrict__ Vws,
        const T *__restrict__ VTws, const T *__restrict__ Tws)
{
    typedef typename Mfma<T>::v4 v4;
    __shared__ T sX[kASlab * kPT];
    __shared__ T sW[32 * 17];
    __shared__ T sW2[32 * 17];
    __shared__ T sT[32 * 32];
    __shared__ int sMap[kRmax];

    const int grp = blockIdx.x;
    const int nslabs = (ncols + kASlab - 1) / kASlab;
    const int s0 = blockIdx.y * spw, s1 = min(nslabs, s0 + spw);
    if (s0 >= s1) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l15 = lane & 15;
    const int nr = group_nrows(grp, la);
    const int nrp = (nr + 15) & ~15;
    const int nblk = nrp >> 4;
    const T *V = Vws + (size_t)grp * kRmax * 32;
    const T *VT = VTws + (size_t)grp * 32 * kRmax;
    const T *Tm = Tws + (size_t)grp * 32 * 32;
    const int ksteps = (la.bk + 3) >> 2;   // V/VT/T are zero beyond bk
    const int arw = Mfma<T>::arow(lane);

    if (tid < nr) sMap[tid] = group_row(tid, grp, la);
    for (int e = tid; e < 32 * 32; e += kAT) sT[e] = Tm[e];
    for (int e = tid; e < 32 * 17; e += kAT) sW[e] = (T)0;

    // ---- V fragments for this wave's row blocks (registers, whole run) -----
    T Vw[kAB][4][2];   // W phase, A operand of V^T: V[blk*16 + q + 4s][ab*16 + arow]
    T Vu[kAB][8];      // update,  A operand of V  : V[blk*16 + arow][4s + q]
#pragma unroll
    for (int jb = 0; jb < kAB; ++jb) {
        const int blk = w + kAW * jb;     // < 32: V/VT hold kRmax (zero-padded) rows
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ab = 0; ab < 2; ++ab) Vw[jb][s][ab] = V[(size_t)(blk * 16 + q + 4 * s) * 32 + ab * 16 + arw];
#pragma unroll
        for (int s = 0; s < 8; ++s) Vu[jb][s] = VT[(size_t)(4 * s + q) * kRmax + blk * 16 + arw];
    }
    __syncthreads();

    T xn[kXN];
    slab_load<T, TR>(base, ld, sMap, nr, s0 * kASlab, min(kASlab, ncols - s0 * kASlab), tid, xn);
    slab_to_lds<T, TR>(sX, nrp, tid, xn);
    __syncthreads();

    for (int slab = s0; slab < s1; ++slab) {
        const int c0 = slab * kASlab;
        const int nc = min(kASlab, ncols - c0);
        if (slab + 1 < s1)   // next slab in flight while this one computes
            slab_load<T, TR>(base, ld, sMap, nr, c0 + kASlab, min(kASlab, ncols - c0 - kASlab), tid, xn);

        // ---- W = V^T X (32 x 16): partial over this wave's rows, ds_add ------
        {
            v4 acc[2] = {v4{0, 0, 0, 0}, v4{0, 0, 0, 0}};
#pragma unroll
            for (int jb = 0; jb < kAB; ++jb) {
                const int blk = w + kAW * jb;
                if (blk < nblk) {
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        const T bx = sX[xidx<TR>(blk * 16 + q + 4 * s, l15)];
#pragma unroll
                        for (int ab = 0; ab < 2; ++ab) acc[ab] = Mfma<T>::mma(Vw[jb][s][ab], bx, acc[ab]);
                    }
                }
            }
            if (w < nblk) {
#pragma unroll
                for (int ab = 0; ab < 2; ++ab)
#pragma unroll
                    for (int g = 0; g < 4; ++g) atomicAdd(&sW[(ab * 16 + q + 4 * g) * 17 + l15], acc[ab][g]);
            }
        }
        lds_barrier();
        // ---- W2 = -(T^T W) -------------------------------------------------
        if (w < 2) {
            const int ab = w;
            v4 acc = {0, 0, 0, 0};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int k = 4 * s + q;
                acc = Mfma<T>::mma(sT[k * 32 + ab * 16 + arw], sW[k * 17 + l15], acc);
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) sW2[(ab * 16 + q + 4 * g) * 17 + l15] = -acc[g];
        }
        lds_barrier();
        for (int e = tid; e < 32 * 17; e += kAT) sW[e] = (T)0;   // ready for the next slab
        // ---- X += V W2 ----------------------------------------------------
        {
            T bw[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) bw[s] = sW2[(4 * s + q) * 17 + l15];
#pragma unroll
            for (int jb = 0; jb < kAB; ++jb) {
                const int blk = w + kAW * jb;
                if (blk < nblk) {
                    v4 acc;
#pragma unroll
                    for (int g = 0; g < 4; ++g) acc[g] = sX[xidx<TR>(blk * 16 + q + 4 * g, l15)];
#pragma unroll
                    for (int s = 0; s < 8; ++s)
                        if (s < ksteps) acc = Mfma<T>::mma(Vu[jb][s], bw[s], acc);
                    if (!TR) {
                        // straight to HBM: 4 rows x 16 consecutive elements per store
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            const int r = blk * 16 + q + 4 * g;
                            if (r < nr && l15 < nc) base[(long)sMap[r] * ld + c0 + l15] = acc[g];
                        }
                    } else {
#pragma unroll
                        for (int g = 0; g < 4; ++g) sX[xidx<TR>(blk * 16 + q + 4 * g, l15)] = acc[g];
                    }
                }
            }
        }
        lds_barrier();
        if (TR) {   // coalesced write-back: consecutive threads -> consecutive physical columns
            const int r = tid;
            if (r < nr) {
                const int pr = sMap[r];
#pragma unroll
                for (int k = 0; k < kXN; ++k)
                    if (k < nc) base[(long)(c0 + k) * ld + pr] = sX[xidx<true>(r, k)];
            }
            lds_barrier();
        }
        if (slab + 1 < s1) {
            slab_to_lds<T, TR>(sX, nrp, tid, xn);
            lds_barrier();
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
    dim3 grid(t.lv[level].groups), block(kFT);
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
    const int groups = t.lv[level].groups;
    const int nslabs = (ncols + kASlab - 1) / kASlab;
    // one resident workgroup per CU (LDS bound): aim for about one wave of workgroups
    const int target = 256;
    const int spw = std::max(1, (groups * nslabs + target - 1) / target);
    dim3 grid(groups, (nslabs + spw - 1) / spw), block(kAT);
    const T *V = (const T *)ws.V[level], *VT = (const T *)ws.VT[level], *Tm = (const T *)ws.T[level];
    if (trans)
        hipLaunchKernelGGL((k_apply<T, true>), grid, block, 0, s, base, ld, a, ncols, spw, V, VT, Tm);
    else
        hipLaunchKernelGGL((k_apply<T, false>), grid, block, 0, s, base, ld, a, ncols, spw, V, VT, Tm);
    return hipGetLastError();
}

template hipError_t launch_factor<double>(bool, double *, long, const Tree &, int, const TreeWs &, hipStream_t);
template hipError_t launch_factor<float>(bool, float *, long, const Tree &, int, const TreeWs &, hipStream_t);
template hipError_t launch_apply<double>(bool, double *, long, const Tree &, int, int, const TreeWs &, hipStream_t);
template hipError_t launch_apply<float>(bool, float *, long, const Tree &, int, int, const TreeWs &, hipStream_t);

}  // namespace brd
