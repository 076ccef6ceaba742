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

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

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
// per-phase cycle accumulators of the k_factor column loop (wave 0 of workgroup 0)
#define PH_DECL unsigned long long ph_t = __builtin_amdgcn_s_memtime(), ph_acc[5] = {0, 0, 0, 0, 0}
#define PH(k)                                                                      \
    do {                                                                           \
        const unsigned long long ph_n = __builtin_amdgcn_s_memtime();              \
        ph_acc[k] += ph_n - ph_t;                                                  \
        ph_t = ph_n;                                                               \
    } while (0)
#define PH_STORE                                                                   \
    do {                                                                           \
        if (blockIdx.x == 0 && threadIdx.x == 0)                                   \
            for (int k = 0; k < 5; ++k) g_stamps[10 + k] = ph_acc[k];              \
    } while (0)
// per-phase cycle accumulators of the apply slab loop (wave 0 of workgroup (0,0))
#define APH_DECL unsigned long long aph_t = __builtin_amdgcn_s_memtime(), aph_acc[6] = {0, 0, 0, 0, 0, 0}
#define APH(k)                                                                     \
    do {                                                                           \
        const unsigned long long aph_n = __builtin_amdgcn_s_memtime();             \
        aph_acc[k] += aph_n - aph_t;                                               \
        aph_t = aph_n;                                                             \
    } while (0)
#define APH_STORE                                                                  \
    do {                                                                           \
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                \
            for (int k = 0; k < 6; ++k) g_stamps[20 + k] = aph_acc[k];             \
    } while (0)
#else
#define APH_DECL do {} while (0)
#define APH(k) do {} while (0)
#define APH_STORE do {} while (0)
#define STAMP(k) do {} while (0)
#define PH_DECL do {} while (0)
#define PH(k) do {} while (0)
#define PH_STORE do {} while (0)
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
// Cross-lane helpers (gfx950).  wave_sum: butterfly over the 64 lanes --
// DPP xor-1 / xor-2 (quad_perm), mirror-8, mirror-16, then v_permlane16_swap
// (row pairs) and v_permlane32_swap (halves); every lane gets the total.
// ==========================================================================
#define BRD_DPP32(x, ctrl) __builtin_amdgcn_update_dpp(0, (x), (ctrl), 0xf, 0xf, false)

__device__ __forceinline__ double dpp64(double x, int) = delete;
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    return __hiloint2double(BRD_DPP32(__double2hiint(x), CTRL), BRD_DPP32(__double2loint(x), CTRL));
}
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __int_as_float(BRD_DPP32(__float_as_int(x), CTRL));
}
__device__ __forceinline__ double swap_add16(double v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ double swap_add32(double v) {
    const auto a = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    return __hiloint2double(b[0], a[0]) + __hiloint2double(b[1], a[1]);
}
__device__ __forceinline__ float swap_add16(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(a[0]) + __int_as_float(a[1]);
}
__device__ __forceinline__ float swap_add32(float v) {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(a[0]) + __int_as_float(a[1]);
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp<0x141>(v);   // row_half_mirror
    v += dpp<0x140>(v);   // row_mirror
    v = swap_add16(v);
    return swap_add32(v);
}
// permlane swaps on whole values: {a', b'} per v_permlane{16,32}_swap_b32
// (16: odd rows of a <-> even rows of b; 32: upper half of a <-> lower half of b)
__device__ __forceinline__ void swap16(double &a, double &b) {
    const auto l = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
    a = __hiloint2double(h[0], l[0]);
    b = __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ void swap32(double &a, double &b) {
    const auto l = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
    a = __hiloint2double(h[0], l[0]);
    b = __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ void swap16(float &a, float &b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(a), __float_as_int(b), false, false);
    a = __int_as_float(r[0]);
    b = __int_as_float(r[1]);
}
__device__ __forceinline__ void swap32(float &a, float &b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(b), false, false);
    a = __int_as_float(r[0]);
    b = __int_as_float(r[1]);
}
// Four wave sums at once (transpose-reduce): a 32-swap folds columns {0,2}
// and {1,3} into one register each (low / high half), a 16-swap leaves
// column c in row c (lanes 16c .. 16c+15), four in-row DPP steps finish.
// Returns the lane's row total; column c's sum is in lane 16c.
template <typename T>
__device__ __forceinline__ T wave_sum4(T v0, T v1, T v2, T v3) {
    swap32(v0, v2);
    swap32(v1, v3);
    T s02 = v0 + v2, s13 = v1 + v3;   // lanes < 32: col 0 / 1; lanes >= 32: col 2 / 3
    swap16(s02, s13);
    T t = s02 + s13;                  // row r: column r
    t += dpp<0xB1>(t);
    t += dpp<0x4E>(t);
    t += dpp<0x141>(t);
    t += dpp<0x140>(t);
    return t;
}
__device__ __forceinline__ double readlane(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ float readlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// ==========================================================================
// k_factor: Householder QR of one tree node (<= kRmax rows x bk <= 32 cols).
// 512 threads = 8 waves; wave w owns columns 4w .. 4w+3 of the whole node,
// lane l rows l + 64k (k = 0..7), in registers.  Per column j:
//   * the owner of column j has published v_j's raw sub-diagonal part and
//     (1/u1, tau, alpha) in LDS;
//   * every wave forms w_c = v_j^T X[:,c] for its four columns with in-wave
//     butterfly sums (no cross-wave reduction), updates X[:,c] -= tau w_c v_j
//     for c > j, and records v_c^T v_j = w_c / u1_c for c < j (the T factor);
//   * the owner of column j+1 forms its reflector (norm by a butterfly sum)
//     and publishes it; one barrier.
// The row-major view's tile is read (and its R written back) through LDS
// staging, 256-byte rows at a time.
// Columns stay unscaled ("raw") while the panel is factored: v_j =
// X[:,j] / u1_j below the diagonal.  The j loop is unrolled by 4 so that the
// owner's column index is static (no register-array indexing).
// ==========================================================================
constexpr int kFT = 512;          // threads per factor workgroup
constexpr int kFR = kRmax / 64;   // rows per lane

template <typename T>
struct Reflector {
    T inv_u1, tau, alpha;
};
// LAPACK-style (tau = 0 when the sub-column is zero) from the squared norm
// of the sub-column and the diagonal entry x0.
// (BRD_S1_IEEE_REFL: the IEEE sqrt and divisions instead of the hardware
// reciprocal square root / reciprocal refined by Newton steps -- the scalars
// sit on the column loop's critical path, once per column of every panel)
// The hardware estimates flush denormal inputs and results, so arguments
// near the ends of the exponent range are rescaled by a power of two first
// (exact): a squared norm below 2^-960 (fp64) / 2^-100 (fp32), a reciprocal
// argument outside 2^+-960 / 2^+-100.
__device__ __forceinline__ double refl_rsq(double q) {
    const bool tiny = q < 0x1p-960;
    const double qs = tiny ? q * 0x1p+1000 : q;
    double r = __builtin_amdgcn_rsq(qs);
    const double h = 0.5 * qs;
    r = r * fma(-h * r, r, 1.5);
    r = r * fma(-h * r, r, 1.5);
    return tiny ? r * 0x1p+500 : r;
}
__device__ __forceinline__ float refl_rsq(float q) {
    const bool tiny = q < 0x1p-100f;
    const float qs = tiny ? q * 0x1p+100f : q;
    const float r = __builtin_amdgcn_rsqf(qs);
    const float rr = r * fmaf(-0.5f * qs * r, r, 1.5f);
    return tiny ? rr * 0x1p+50f : rr;
}
__device__ __forceinline__ double refl_rcp(double u) {
    const double au = fabs(u);
    const double sc = au < 0x1p-960 ? 0x1p+960 : (au > 0x1p+960 ? 0x1p-960 : 1.0);
    const double us = u * sc;
    double y = __builtin_amdgcn_rcp(us);
    y = fma(y, fma(-us, y, 1.0), y);
    y = fma(y, fma(-us, y, 1.0), y);
    return y * sc;
}
__device__ __forceinline__ float refl_rcp(float u) {
    const float au = fabsf(u);
    const float sc = au < 0x1p-100f ? 0x1p+100f : (au > 0x1p+100f ? 0x1p-100f : 1.0f);
    const float us = u * sc;
    const float y = __builtin_amdgcn_rcpf(us);
    return fmaf(y, fmaf(-us, y, 1.0f), y) * sc;
}
template <typename T>
__device__ __forceinline__ Reflector<T> make_reflector(T sub2, T x0) {
    Reflector<T> h{(T)1, (T)0, x0};
    if (sub2 != (T)0) {
#ifdef BRD_S1_IEEE_REFL
        const T nrm = sqrt(fma(x0, x0, sub2));
        h.alpha = x0 >= (T)0 ? -nrm : nrm;
        const T u1 = x0 - h.alpha;
        h.tau = -u1 / h.alpha;
        h.inv_u1 = (T)1 / u1;
#else
        const T s2 = fma(x0, x0, sub2);
        const T r = refl_rsq(s2);   // 1 / ||x||
        const T nrm = s2 * r;
        h.alpha = x0 >= (T)0 ? -nrm : nrm;
        const T u1 = x0 - h.alpha;
        h.tau = x0 >= (T)0 ? u1 * r : -u1 * r;   // -u1 / alpha
        h.inv_u1 = refl_rcp(u1);
#endif
    }
    return h;
}

template <typename T>
struct FactorLds {
    T sV[2][kRmax];        // published reflector column (raw, rows > j), double-buffered
    T sH[2][4];            // its 1/u1, tau, alpha
    T sZ[32][33];          // v_c^T v_j (c < j)
    T sT[32][33];
    T sU1[32], sTau[32];   // 1/u1 and tau per column
    int sMap[kRmax];
    T sStage[kRmax / 2][33];   // row-major <-> register-layout staging, half a node at a time
    T sX0[kRmax][5];           // wave 0's columns for the output (pitch 5: conflict-free)
};

// The factor of node grp (k_factor, or the factor role of k_apply_factor).
template <typename T, bool TR>
__device__ __forceinline__ void factor_body(FactorLds<T> &L, const int grp, T *__restrict__ base, long ld, LvArgs la,
                                            T *__restrict__ Vws, T *__restrict__ VTws, T *__restrict__ Tws)
{
    auto &sV = L.sV;
    auto &sH = L.sH;
    auto &sZ = L.sZ;
    auto &sT = L.sT;
    auto &sU1 = L.sU1;
    auto &sTau = L.sTau;
    auto &sMap = L.sMap;
    auto &sStage = L.sStage;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nr = group_nrows(grp, la);
    const int bk = la.bk;
    const int kk = min(nr, bk);
    STAMP(0);

    if (tid < nr) sMap[tid] = group_row(tid, grp, la);
    for (int e = tid; e < 32 * 33; e += kFT) {
        (&sZ[0][0])[e] = (T)0;
        (&sT[0][0])[e] = (T)0;
    }
    if (tid < 32) { sU1[tid] = (T)1; sTau[tid] = (T)0; }
    __syncthreads();

    // ---- the tile into registers: x[k][cc] = X[lane + 64k][4w + cc] ----------
    STAMP(1);
    T x[kFR][4];
    if constexpr (TR) {
        // column-major view: lanes -> consecutive rows of one column (coalesced)
#pragma unroll
        for (int k = 0; k < kFR; ++k) {
            const int i = lane + 64 * k;
            const int pr = i < nr ? sMap[i] : 0;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int c = 4 * w + cc;
                x[k][cc] = (i < nr && c < bk) ? *vptr<TR>(base, ld, pr, c) : (T)0;
            }
        }
    } else {
        // row-major view: the register layout would touch 64 rows per load
        // instruction; instead 32 threads read one 256-byte row (all 32 rows
        // of a thread in flight at once) and the tile is redistributed through
        // the staging array, half a node at a time.
        constexpr int kLE = kRmax * 32 / kFT;   // elements per thread
        const int c = tid & 31;
        T lv[kLE];
#pragma unroll
        for (int e = 0; e < kLE; ++e) {
            const int i = (tid >> 5) + (kFT / 32) * e;
            lv[e] = (i < nr && c < bk) ? base[(long)sMap[i] * ld + c] : (T)0;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int e = 0; e < kLE / 2; ++e) sStage[(tid >> 5) + (kFT / 32) * e][c] = lv[e + kLE / 2 * h];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kFR / 2; ++k)
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) x[k + kFR / 2 * h][cc] = sStage[lane + 64 * k][4 * w + cc];
            __syncthreads();
        }
    }
    STAMP(2);

    // publish column j (owner wave, static local column CC)
    auto publish = [&](int j, auto cc_tag) {
        constexpr int CC = decltype(cc_tag)::value;
        T p = (T)0;
#pragma unroll
        for (int k = 0; k < kFR; ++k) {
            const T v = (lane + 64 * k > j) ? x[k][CC] : (T)0;
            p = fma(v, v, p);
            sV[j & 1][lane + 64 * k] = v;
        }
        const T sub2 = wave_sum(p);
        const T x0 = readlane(x[0][CC], j);   // row j lives in lane j, k = 0 (j < 32)
        const Reflector<T> h = make_reflector(sub2, x0);
        if (lane == 0) {
            sH[j & 1][0] = h.inv_u1;
            sH[j & 1][1] = h.tau;
            sH[j & 1][2] = h.alpha;
            sU1[j] = h.inv_u1;
            sTau[j] = h.tau;
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    if (kk > 0 && w == 0) publish(0, I0{});
    __syncthreads();

    PH_DECL;
    for (int m = 0; m < 8; ++m) {
        if (4 * m >= kk) break;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = 4 * m + t;
            if (j >= kk) break;
            if (j == 1) STAMP(3);
            const int pb = j & 1;
            // (1) the reflector column and its scalars
            T vcol[kFR];
#pragma unroll
            for (int k = 0; k < kFR; ++k) vcol[k] = sV[pb][lane + 64 * k];
            const T inv_u1 = sH[pb][0], tau = sH[pb][1], alpha = sH[pb][2];
            PH(0);
            // (2) w_c = X[j][c] + (sum_{i>j} x_ij x_ic) / u1 for the wave's four columns
            T wcol[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                T p0 = (T)0, p1 = (T)0;
#pragma unroll
                for (int k = 0; k < kFR; k += 2) {
                    p0 = fma(vcol[k], x[k][cc], p0);
                    p1 = fma(vcol[k + 1], x[k + 1][cc], p1);
                }
                wcol[cc] = p0 + p1;
            }
            {
                const T tsum = wave_sum4(wcol[0], wcol[1], wcol[2], wcol[3]);
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) wcol[cc] = fma(readlane(tsum, 16 * cc), inv_u1, readlane(x[0][cc], j));
            }
            PH(1);
            // (3) update the columns right of j; v^T v for the columns left of j
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int c = 4 * w + cc;
                if (c > j && c < bk) {
                    const T tw = tau * wcol[cc], twu = tw * inv_u1;
#pragma unroll
                    for (int k = 0; k < kFR; ++k) x[k][cc] = fma(-twu, vcol[k], x[k][cc]);   // rows > j
                    if (lane == j) x[0][cc] -= tw;                                          // row j (v_j = 1)
                } else if (c == j) {
                    if (lane == j) x[0][cc] = alpha;
                } else if (c < j) {
                    if (lane == 0) sZ[c][j] = wcol[cc] * sU1[c];
                }
            }
            PH(2);
            // (4) the owner of column j+1 publishes its reflector
            if (j + 1 < kk && w == ((j + 1) >> 2)) {
                if (t == 0) publish(j + 1, I1{});
                else if (t == 1) publish(j + 1, I2{});
                else if (t == 2) publish(j + 1, I3{});
                else publish(j + 1, I0{});
            }
            PH(3);
            __syncthreads();
            PH(4);
        }
    }
    PH_STORE;
    STAMP(4);

    // ---- T and the outputs ---------------------------------------------------
    // Wave 0 forms T (LAPACK larft: T[:, j] = -tau_j T[:, :j] (V^T v_j)[:j],
    // T[j][j] = tau_j; lane a keeps row a in registers, fully unrolled; z = V^T V
    // from sZ as broadcasts) and writes it; waves 1..7 meanwhile write V
    // (kRmax x 32 row-major), VT (32 x kRmax, lanes -> consecutive rows) and R /
    // zeros back into the matrix for their own columns and, from an LDS copy,
    // for wave 0's.  R: TR = true along columns from registers (coalesced);
    // TR = false the 32 x 32 triangle from registers and the zeros below it by
    // 256-byte rows.
    T *Tm = Tws + (size_t)grp * 32 * 32;
    T *V = Vws + (size_t)grp * kRmax * 32;
    T *VT = VTws + (size_t)grp * 32 * kRmax;
    const int nrp = (nr + 15) & ~15;
    if (w == 0) {
#pragma unroll
        for (int k = 0; k < kFR; ++k)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) L.sX0[lane + 64 * k][cc] = x[k][cc];
    }
    __syncthreads();
    STAMP(5);
    if (w == 0) {
        if (lane < 32) {
            const int a = lane;
            T trow[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                T s4[4] = {(T)0, (T)0, (T)0, (T)0};
#pragma unroll
                for (int cc = 0; cc < j; ++cc) s4[cc & 3] = fma(trow[cc], sZ[cc][j], s4[cc & 3]);
                const T s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                const T tj = j < kk ? sTau[j] : (T)0;
                trow[j] = a < j ? -tj * s : (a == j ? tj : (T)0);
            }
#pragma unroll
            for (int j = 0; j < 32; ++j) sT[a][j] = trow[j];
        }
        wave_sync();
        for (int e = lane; e < 32 * 32; e += 64) Tm[e] = sT[e >> 5][e & 31];
    } else {
        // rows lane + 64k of columns c0 .. c0+3 (values xv)
        auto emit = [&](const T (&xv)[4], int c0, int k) {
            const int i = lane + 64 * k;
            T v[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int c = c0 + cc;
                v[cc] = (T)0;
                if (c < kk && i < nr) v[cc] = i < c ? (T)0 : (i == c ? (T)1 : xv[cc] * sU1[c]);
            }
            if (i < nrp) {
                // the lane's four V entries are one aligned 4-wide row segment:
                // one vector store instead of four scattered scalar ones
                using T4 = T __attribute__((ext_vector_type(4)));
                *reinterpret_cast<T4 *>(V + (size_t)i * 32 + c0) = T4{v[0], v[1], v[2], v[3]};
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) VT[(size_t)(c0 + cc) * kRmax + i] = v[cc];
            }
            if (i < nr && (TR || i < 32)) {
                const int pr = sMap[i];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) {
                    const int c = c0 + cc;
                    if (c < bk) *vptr<TR>(base, ld, pr, c) = (c >= i) ? xv[cc] : (T)0;
                }
            }
        };
#pragma unroll
        for (int k = 0; k < kFR; ++k) emit(x[k], 4 * w, k);
        for (int k = w - 1; k < kFR; k += kFT / 64 - 1) {
            T x0[4];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) x0[cc] = L.sX0[lane + 64 * k][cc];
            emit(x0, 0, k);
        }
        if constexpr (!TR) {   // zeros below the triangle, rows 32 .. nr-1
            for (int e = tid - 64; e < (nr - 32) * 32; e += kFT - 64) {
                const int i = 32 + (e >> 5), c = e & 31;
                if (c < bk) base[(long)sMap[i] * ld + c] = (T)0;
            }
        }
    }
    STAMP(6);
}

template <typename T, bool TR>
__global__ void __launch_bounds__(kFT)
k_factor(T *__restrict__ base, long ld, LvArgs la, T *__restrict__ Vws, T *__restrict__ VTws,
         T *__restrict__ Tws)
{
    __shared__ FactorLds<T> L;
    factor_body<T, TR>(L, blockIdx.x, base, ld, la, Vws, VTws, Tws);
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

// Raw buffer access (32-bit byte offsets; out-of-range offsets read 0 and
// drop stores).
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ T buf_load(__amdgpu_buffer_rsrc_t r, unsigned off);
template <> __device__ __forceinline__ double buf_load<double>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
template <> __device__ __forceinline__ float buf_load<float>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
template <typename T> __device__ __forceinline__ void buf_store(T v, __amdgpu_buffer_rsrc_t r, unsigned off);
template <> __device__ __forceinline__ void buf_store<double>(double v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)off, 0, 0);
}
template <> __device__ __forceinline__ void buf_store<float>(float v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, 0);
}

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

// Slab staging.  TR = false: thread -> element pair 2(tid%8), 2(tid%8)+1 of
// rows tid/8 + 64p (one 16-byte load per row for fp64, 8 threads per 128-byte
// row); TR = true: thread -> row tid (< kRmax), all 16 columns.  The
// write-back (slab_store) uses the same map, so the row addresses are shared.
constexpr int kXP = kXN / 2;   // TR = false: element pairs per thread

template <typename T>
struct Pair {
    typedef T v2 __attribute__((ext_vector_type(2), aligned(sizeof(T))));
};

template <typename T, bool TR>
__device__ __forceinline__ void slab_load(const T *base, long ld, const int *sMap, int nr, int c0, int nc,
                                          int tid, T (&xn)[kXN]) {
    if (!TR) {
        typedef typename Pair<T>::v2 v2;
        const int c2 = 2 * (tid & 7);
#pragma unroll
        for (int p = 0; p < kXP; ++p) {
            const int r = (tid >> 3) + (kAT / 8) * p;
            const bool ok = r < nr && c2 < nc;
            const int pr = ok ? sMap[r] : 0;
            v2 v = {(T)0, (T)0};
            if (ok) {
                const T *src = base + (long)pr * ld + c0 + c2;
                if (c2 + 1 < nc) v = *(const v2 *)src;
                else v.x = src[0];
            }
            xn[2 * p] = v.x;
            xn[2 * p + 1] = v.y;
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
        typedef typename Pair<T>::v2 v2;
        const int c2 = 2 * (tid & 7);
#pragma unroll
        for (int p = 0; p < kXP; ++p) {
            const int r = (tid >> 3) + (kAT / 8) * p;
            if (r < nrp) *(v2 *)&sX[xidx<false>(r, c2)] = v2{xn[2 * p], xn[2 * p + 1]};
        }
    } else {
        const int r = tid;
        if (r < nrp) {
#pragma unroll
            for (int k = 0; k < kXN; ++k) sX[xidx<true>(r, k)] = xn[k];
        }
    }
}

// Updated slab: LDS -> matrix, coalesced (TR = false: the slab_load map;
// TR = true: consecutive threads -> consecutive physical columns).
template <typename T, bool TR>
__device__ __forceinline__ void slab_store(T *base, long ld, const int *sMap, int nr, int c0, int nc, int tid,
                                           const T *sX) {
    if (!TR) {
        typedef typename Pair<T>::v2 v2;
        const int c2 = 2 * (tid & 7);
#pragma unroll
        for (int p = 0; p < kXP; ++p) {
            const int r = (tid >> 3) + (kAT / 8) * p;
            if (r < nr && c2 < nc) {
                const v2 v = *(const v2 *)&sX[xidx<false>(r, c2)];
                T *dst = base + (long)sMap[r] * ld + c0 + c2;
                if (c2 + 1 < nc) *(v2 *)dst = v;
                else dst[0] = v.x;
            }
        }
    } else {
        const int r = tid;
        if (r < nr) {
            const int pr = sMap[r];
#pragma unroll
            for (int k = 0; k < kXN; ++k)
                if (k < nc) base[(long)(c0 + k) * ld + pr] = sX[xidx<true>(r, k)];
        }
    }
}

template <typename T>
struct ApplyLds {
    T sX[kASlab * kPT];
    T sWp[kAW][32 * 16];   // per-wave partials of W = V^T X, summed in wave order (deterministic)
    T sW[32 * 17];
    T sW2[32 * 17];
    T sT[32 * 32];
    int sMap[kRmax];
};

// The apply of node grp to slab run `run` (k_apply, or the apply role of k_apply_factor).
template <typename T, bool TR, bool DIRECT>
__device__ __forceinline__ void apply_body(ApplyLds<T> &L, const int grp, const int run, T *__restrict__ base, long ld,
                                           LvArgs la, int ncols, int spw, const T *__restrict__ Vws,
                                           const T *__restrict__ VTws, const T *__restrict__ Tws)
{
    typedef typename Mfma<T>::v4 v4;
    static_assert(kAT == 32 * 16, "one thread per element of W in the cross-wave sum");
    auto &sX = L.sX;
    auto &sWp = L.sWp;
    auto &sW = L.sW;
    auto &sW2 = L.sW2;
    auto &sT = L.sT;
    auto &sMap = L.sMap;

    const int nslabs = (ncols + kASlab - 1) / kASlab;
    const int s0 = run * spw, s1 = min(nslabs, s0 + spw);
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
    // LDS-staged path: the run's first slab is in flight together with the V
    // fragments below (one memory latency before the first slab, not two)
    T xn[DIRECT ? 1 : kXN];
    if constexpr (!DIRECT) {
        lds_barrier();
        slab_load<T, TR>(base, ld, sMap, nr, s0 * kASlab, min(kASlab, ncols - s0 * kASlab), tid, xn);
    }
    for (int e = tid; e < 32 * 32; e += kAT) sT[e] = Tm[e];

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

    // ---- the W reduction and W2 = -(T^T W), shared by both slab paths -------
    // acc: this wave's partial W (two 16 x 16 tiles); afterwards sW2 holds W2
    // and the caller reads it after its lds_barrier.
    auto reduce_w2 = [&](v4 (&acc)[2]) {
        if (w < nblk) {
#pragma unroll
            for (int ab = 0; ab < 2; ++ab)
#pragma unroll
                for (int g = 0; g < 4; ++g) sWp[w][(ab * 16 + q + 4 * g) * 16 + l15] = acc[ab][g];
        }
        lds_barrier();
        // cross-wave sum in wave order: the result does not depend on which
        // wave finishes first (stage 1 is bitwise reproducible run to run)
        {
            const int nwp = min(kAW, nblk);
            T sum = sWp[0][tid];
            for (int k = 1; k < nwp; ++k) sum += sWp[k][tid];
            sW[(tid >> 4) * 17 + (tid & 15)] = sum;
        }
        lds_barrier();
        if (w < 2) {
            const int ab = w;
            v4 a2 = {0, 0, 0, 0};
#pragma unroll
            for (int st = 0; st < 8; ++st) {
                const int k = 4 * st + q;
                a2 = Mfma<T>::mma(sT[k * 32 + ab * 16 + arw], sW[k * 17 + l15], a2);
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) sW2[(ab * 16 + q + 4 * g) * 17 + l15] = -a2[g];
        }
        lds_barrier();
    };

    if constexpr (DIRECT) {
        static_assert(!TR, "the register-resident slab path is for the row-major view");
        {
            // ---- row-major view: the slab never touches LDS ----------------
            // The B operand of W = V^T X at step s of row block jb is
            // X[blk*16 + q + 4s][l15], and the accumulator register g of the
            // update X += V W2 is X[blk*16 + q + 4g][l15]: the same element, so
            // one register tile x[jb][.] is loaded from HBM (16 lanes = one
            // 128-byte row segment), feeds both MFMA phases and is stored back.
            // The next slab's tile is in flight while this one computes.
            // the 16 rows of a block are consecutive matrix rows (launch_apply
            // takes this path only when every tree node is made of whole
            // 16-row blocks): one byte offset per block, rows blk*16 + q + 4g.
            // Buffer loads / stores with 32-bit offsets (the view is < 4 GiB):
            // an offset past the end (rows beyond the node, columns beyond the
            // slab) reads 0 and drops the store, so no lane predicates.
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
            constexpr unsigned kOut = 0x80000000u;   // >= num_records: out of range
            unsigned rb[kAB];
#pragma unroll
            for (int jb = 0; jb < kAB; ++jb) {
                const int b16 = (w + kAW * jb) * 16;
                rb[jb] = b16 < nr ? (unsigned)((sMap[b16] + q) * (int)ld + l15) * (unsigned)sizeof(T) : kOut;
            }
            const unsigned ld4b = 4u * (unsigned)ld * (unsigned)sizeof(T);
            auto off = [&](int jb, int g, int c0, int nc) -> unsigned {
                const bool ok = l15 < nc && (w + kAW * jb) * 16 + q + 4 * g < nr;
                return ok ? rb[jb] + (unsigned)g * ld4b + (unsigned)c0 * (unsigned)sizeof(T) : kOut;
            };
            T x[kAB][4], xnx[kAB][4];
            auto load = [&](T (&dst)[kAB][4], int c0, int nc) {
#pragma unroll
                for (int jb = 0; jb < kAB; ++jb)
#pragma unroll
                    for (int g = 0; g < 4; ++g) dst[jb][g] = buf_load<T>(rs, off(jb, g, c0, nc));
            };
            load(x, s0 * kASlab, min(kASlab, ncols - s0 * kASlab));
            for (int slab = s0; slab < s1; ++slab) {
                const int c0 = slab * kASlab;
                const int nc = min(kASlab, ncols - c0);
                if (slab + 1 < s1) load(xnx, c0 + kASlab, min(kASlab, ncols - c0 - kASlab));
                v4 acc[2] = {v4{0, 0, 0, 0}, v4{0, 0, 0, 0}};
#pragma unroll
                for (int jb = 0; jb < kAB; ++jb) {
                    if (w + kAW * jb < nblk) {
#pragma unroll
                        for (int st = 0; st < 4; ++st)
#pragma unroll
                            for (int ab = 0; ab < 2; ++ab) acc[ab] = Mfma<T>::mma(Vw[jb][st][ab], x[jb][st], acc[ab]);
                    }
                }
                reduce_w2(acc);
#pragma unroll
                for (int jb = 0; jb < kAB; ++jb) {
                    if (w + kAW * jb < nblk) {
                        v4 a = {x[jb][0], x[jb][1], x[jb][2], x[jb][3]};
                        // W2 straight from LDS (no register copy: registers are
                        // the limit of this path)
#pragma unroll
                        for (int st = 0; st < 8; ++st)
                            if (st < ksteps) a = Mfma<T>::mma(Vu[jb][st], sW2[(4 * st + q) * 17 + l15], a);
#pragma unroll
                        for (int g = 0; g < 4; ++g) buf_store<T>(a[g], rs, off(jb, g, c0, nc));
                    }
                }
                if (slab + 1 < s1) {
#pragma unroll
                    for (int jb = 0; jb < kAB; ++jb)
#pragma unroll
                        for (int g = 0; g < 4; ++g) x[jb][g] = xnx[jb][g];
                }
            }
        }
    } else {

    slab_to_lds<T, TR>(sX, nrp, tid, xn);
    __syncthreads();
    APH_DECL;

    for (int slab = s0; slab < s1; ++slab) {
        const int c0 = slab * kASlab;
        const int nc = min(kASlab, ncols - c0);
        APH(0);

        // ---- W = V^T X (32 x 16): partial over this wave's rows -------------
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
            // next slab in flight while this one finishes: issued after the W
            // MFMAs, not before them, so that the previous slab's stores drain
            // under those MFMAs instead of stalling the issue of these loads
#ifndef BRD_PF_POS
#define BRD_PF_POS 1
#endif
            if (BRD_PF_POS == 1 && slab + 1 < s1)
                slab_load<T, TR>(base, ld, sMap, nr, c0 + kASlab, min(kASlab, ncols - c0 - kASlab), tid, xn);
            APH(1);
            reduce_w2(acc);   // ---- W2 = -(T^T W) into sW2
            APH(2);
            if (BRD_PF_POS == 2 && slab + 1 < s1)
                slab_load<T, TR>(base, ld, sMap, nr, c0 + kASlab, min(kASlab, ncols - c0 - kASlab), tid, xn);
        }
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
#pragma unroll
                    for (int g = 0; g < 4; ++g) sX[xidx<TR>(blk * 16 + q + 4 * g, l15)] = acc[g];
                }
            }
        }
        lds_barrier();
        APH(3);
        slab_store<T, TR>(base, ld, sMap, nr, c0, nc, tid, sX);
        lds_barrier();
        APH(4);
        if (slab + 1 < s1) {
            slab_to_lds<T, TR>(sX, nrp, tid, xn);
            lds_barrier();
        }
        APH(5);
    }
    APH_STORE;
    }   // LDS-staged path
}

// OCC = apply workgroups per CU the kernel is compiled for (the launch
// bound's second argument is waves per SIMD: 2 OCC).  OCC = 2 (fp32, LDS-staged
// slab, <= 128 VGPRs) is the stream-of-reductions variant, see launch_apply.
template <typename T, bool TR, bool DIRECT, int OCC = 1>
__global__ void __launch_bounds__(kAT, 2 * OCC)
k_apply(T *__restrict__ base, long ld, LvArgs la, int ncols, int spw, const T *__restrict__ Vws,
        const T *__restrict__ VTws, const T *__restrict__ Tws)
{
    __shared__ ApplyLds<T> L;
    apply_body<T, TR, DIRECT>(L, blockIdx.x, blockIdx.y, base, ld, la, ncols, spw, Vws, VTws, Tws);
}

// k_apply_factor: the apply of tree level l (blockIdx.y >= 1) and the factor
// of level l+1 (blockIdx.y = 0, blockIdx.x < nfac) in one launch.  The
// level-(l+1) factor reads only the level-l nodes' R rows of the panel and
// writes only level-(l+1) workspace, the apply only the trailing columns and
// level-l workspace, so the two roles are independent; fusing them replaces
// the side stream and its two event hand-offs per panel side (about 6-7 us of
// idle GPU each, measured).  Row y = 0 is dispatched first, so the factor
// starts at once on a CU of its own.
template <typename T, bool TR, bool DIRECT, int OCC = 1>
__global__ void __launch_bounds__(kAT, 2 * OCC)
k_apply_factor(T *__restrict__ base, long ld, LvArgs la, int ncols, int spw, const T *__restrict__ Vws,
               const T *__restrict__ VTws, const T *__restrict__ Tws, T *__restrict__ fbase, long fld, LvArgs fa,
               int nfac, T *__restrict__ fV, T *__restrict__ fVT, T *__restrict__ fT)
{
    static_assert(kAT == kFT, "one block size for both roles");
    __shared__ union Lds {
        FactorLds<T> f;
        ApplyLds<T> a;
    } L;
    if (blockIdx.y == 0) {
        if ((int)blockIdx.x < nfac) factor_body<T, TR>(L.f, blockIdx.x, fbase, fld, fa, fV, fVT, fT);
        return;
    }
    apply_body<T, TR, DIRECT>(L.a, blockIdx.x, blockIdx.y - 1, base, ld, la, ncols, spw, Vws, VTws, Tws);
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

// One kernel launch; with profiling armed (api_take_launch_events) the launch
// itself stamps the profiler's events at the kernel's start and end.
template <typename F, typename... Args>
static void launch_timed(F kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
    hipEvent_t ea, eb;
    if (api_take_launch_events(&ea, &eb))
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, ea, eb, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}

template <typename T>
hipError_t launch_apply(bool trans, T *base, long ld, const Tree &t, int level, int ncols,
                        const TreeWs &ws, hipStream_t s, int target, T *fuse_panel, long fuse_ld)
{
    if (ncols <= 0) return hipSuccess;
    LvArgs a = lv_args(t, level);
    const int groups = t.lv[level].groups;
    const int nslabs = (ncols + kASlab - 1) / kASlab;
    const bool fuse = fuse_panel && level + 1 < t.nlevels;
    const int nfac = fuse ? t.lv[level + 1].groups : 0;
    // one resident workgroup per CU (registers): aim for about one wave of
    // `target` workgroups, less the CUs the fused factor takes
    // `target` workgroups, less the CUs the fused factor takes.  The smallest
    // run length whose grid fits that many: a grid even one workgroup over it
    // leaves that workgroup a second round behind a whole run of slabs.
    const int tgt = std::max(1, target - nfac);
    int spw = std::max(1, (groups * nslabs + tgt - 1) / tgt);
    while (spw < nslabs && (long)groups * ((nslabs + spw - 1) / spw) > tgt) ++spw;
    spw = std::min(nslabs, std::max(spw, api_min_run(level)));   // (brd_api.cpp)
    const T *V = (const T *)ws.V[level], *VT = (const T *)ws.VT[level], *Tm = (const T *)ws.T[level];
    // Row-major view: the slab can stay in registers (apply_body's direct
    // path).  Measured at N = 8192 (same box): fp32 stage 1 62.7 -> 61.5 ms;
    // fp64 88.5 -> 102.5 ms (the fp64 tile needs more than the 256 VGPRs of a
    // 2-waves-per-SIMD kernel and spills), so fp64 keeps the LDS-staged path.
    // BRD_S1_DIRECT=0 / 1 overrides (tuning).
    static const char *denv = getenv("BRD_S1_DIRECT");
    // fp32 beside other work (brd_set_overlap): the LDS-staged slab compiled
    // for two workgroups per CU (<= 128 VGPRs; another lane's workgroup hides
    // this one's per-slab phases).  N = 8192 fp32 stream, same box, 20 steps,
    // three pairs: 28.8-28.9 -> 29.8-30.2 TFLOP/s; one reduction at a time it
    // was slower (stage 1 60.7 -> 62.9 ms), so alone the one-per-CU variants
    // stay.  BRD_S1_OCC2 = 0 / 1 overrides.
    static const char *oenv = getenv("BRD_S1_OCC2");
    const bool occ2 = sizeof(T) == 4 && (oenv ? oenv[0] == '1' : api_overlap_active());
    const bool want = denv ? denv[0] == '1' : (sizeof(T) == 4 && !occ2);
    const int direct = !trans && want && (level == 0 || t.bk % 16 == 0) &&
                               ((long)t.M * ld + ncols) * (long)sizeof(T) < (1L << 31) ? 1 : 0;
    if (fuse) {
        dim3 grid(groups, 1 + (nslabs + spw - 1) / spw), block(kAT);
        const LvArgs fa = lv_args(t, level + 1);
        T *fV = (T *)ws.V[level + 1], *fVT = (T *)ws.VT[level + 1], *fT = (T *)ws.T[level + 1];
        if constexpr (sizeof(T) == 4) {   // (the two-per-CU build exists for fp32 only)
            if (occ2 && !direct) {
                if (trans)
                    launch_timed((k_apply_factor<T, true, false, 2>), grid, block, s, base, ld, a, ncols, spw, V, VT,
                                 Tm, fuse_panel, fuse_ld > 0 ? fuse_ld : ld, fa, nfac, fV, fVT, fT);
                else
                    launch_timed((k_apply_factor<T, false, false, 2>), grid, block, s, base, ld, a, ncols, spw, V, VT,
                                 Tm, fuse_panel, fuse_ld > 0 ? fuse_ld : ld, fa, nfac, fV, fVT, fT);
                return hipGetLastError();
            }
        }
        if (trans)
            launch_timed((k_apply_factor<T, true, false>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm,
                               fuse_panel, fuse_ld > 0 ? fuse_ld : ld, fa, nfac, fV, fVT, fT);
        else if (direct)
            launch_timed((k_apply_factor<T, false, true>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm,
                               fuse_panel, fuse_ld > 0 ? fuse_ld : ld, fa, nfac, fV, fVT, fT);
        else
            launch_timed((k_apply_factor<T, false, false>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm,
                               fuse_panel, fuse_ld > 0 ? fuse_ld : ld, fa, nfac, fV, fVT, fT);
        return hipGetLastError();
    }
    dim3 grid(groups, (nslabs + spw - 1) / spw), block(kAT);
    if constexpr (sizeof(T) == 4) {
        if (occ2 && !direct) {
            if (trans) launch_timed((k_apply<T, true, false, 2>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm);
            else       launch_timed((k_apply<T, false, false, 2>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm);
            return hipGetLastError();
        }
    }
    if (trans)
        launch_timed((k_apply<T, true, false>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm);
    else if (direct)
        launch_timed((k_apply<T, false, true>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm);
    else
        launch_timed((k_apply<T, false, false>), grid, block, s, base, ld, a, ncols, spw, V, VT, Tm);
    return hipGetLastError();
}

template hipError_t launch_factor<double>(bool, double *, long, const Tree &, int, const TreeWs &, hipStream_t);
template hipError_t launch_factor<float>(bool, float *, long, const Tree &, int, const TreeWs &, hipStream_t);
template hipError_t launch_apply<double>(bool, double *, long, const Tree &, int, int, const TreeWs &, hipStream_t, int, double *, long);
template hipError_t launch_apply<float>(bool, float *, long, const Tree &, int, int, const TreeWs &, hipStream_t, int, float *, long);

}  // namespace brd
