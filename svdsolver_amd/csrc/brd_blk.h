// Blocked stage 1 (dense -> band with a delayed two-sided update): shared
// declarations of the kernels' translation units (brd_blk_rpass.hip,
// brd_blk_prep.hip, brd_blk_cqr.hip, brd_blk_upd.hip) and the host drivers
// (brd_stage1_blk.hip: one GPU; brd_dist.hip: the block-column-sharded
// form).  See brd_stage1_blk.hip for the algorithm.
#pragma once

#include "brd_internal.h"

#include <hip/hip_ext.h>

#include <climits>

namespace brd {
namespace blk {

// --------------------------------------------------------------------------
// MFMA 16x16x4, one operand element per lane:
//   A operand lane l: A[m = l&15][k = l>>4],  B operand lane l: B[k = l>>4][n = l&15]
//   D register g of lane l: row crow(l>>4, g), column l&15
// --------------------------------------------------------------------------
template <typename T> struct Mf;
template <> struct Mf<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(double a, double b, v4 c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int crow(int q, int g) { return q + 4 * g; }
};
template <> struct Mf<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ v4 mma(float a, float b, v4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int crow(int q, int g) { return 4 * q + g; }
};

template <typename T>
struct G2 {   // two consecutive elements: 16 B (fp64) / 8 B (fp32)
    typedef T v2 __attribute__((ext_vector_type(2)));
};

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---- k_rpass (brd_blk_rpass.hip) ----------------------------------------------
constexpr int NBMAX = 4;    // panels per block (Lw / RwT hold 2 NBMAX 32 = 256 vectors)
constexpr int kRT = 512;    // threads: 4 column waves x 2 halves of the workgroup's K range
constexpr int kWM = 64;     // m per wave
constexpr int kMT = 256;    // m per workgroup
#ifndef BRD_BLK_KSU
#define BRD_BLK_KSU 8       // A/B knob (tools/variant_lib.sh)
#endif
constexpr int kSU = BRD_BLK_KSU;   // K steps in flight (Y); X: kSU / 2 step pairs

constexpr int kRpLds = 8192;   // doubles
struct RpArgs {
    const void *src;  long ld;      // source S
    const void *vsrc; long vld;     // virtual tile source (256 wide), or null
    const void *bsrc; long bld;     // skinny operand B (k, t) = bsrc[k*bld + t]
    int K, M;                       // S extents
    int mtiles, ksplit, kper;       // kper: k per split (multiple of 8)
    int tiles, ns, wst;             // k_rpass_d: tiles (virtual first), 16-k stages per tile,
                                    // stages per workgroup (linearised split)
    int nvirt;                      // ksplit if there is a virtual tile, else 0
    void *part; long mp;            // partials [ks][32][mp] (Y) / [ks][mp][32] (X)
    void *vpart;                    // virtual partials [ks][32][256] / [ks][256][32]
    void *vout;                     // virtual result [32][256] / [256][32]
    int *counter;                   // (unused)
    int *err;
    int has_fin;                    // 1: workgroup 0 runs cqr_finish of the panel the pass follows
    int vfold = 0;                  // k_rpass_d: the virtual tile's partials summed in the pass (the
                                    // last of its contributors to arrive, counter *counter) into vout,
                                    // no k_vsum; the consumers patch V's / U's top block themselves
    int va = 0, vb = 0;             // vfold: the virtual result's entries the consumer reads: k in
                                    // [0, va) and [128, 128 + vb) (Y: G^T[t][k]; X: G[k][t])
};

// ---- k_prep_* (brd_blk_prep.hip) ---------------------------------------------
constexpr int kPT = 256;
constexpr int kPI = 32;    // items per workgroup when split: two item waves x two halves of
                           // the K1 range (the correction's MFMA chain over all four SIMDs;
                           // the halves meet in LDS, fixed order); unsplit: 2 kPI items,
                           // four item waves (when the split grid would exceed the CUs)

constexpr int kGramRec = 1040;   // doubles per prep Gram record (1024 + exponent, 128-B lines of its own)
struct PrepArgs {
    void *A; long lda;
    void *Lw; void *RwT; long ldr;
    const void *part; long mp; int ksplit;
    const void *G;            // virtual result of the read pass (LQ: [32][256], QR: [256][32])
    const void *Tm;           // T_j (LQ) / S_{j-1} (QR), 32 x 32 row-major
    void *Qp;                 // the corrected panel, transposed: QpT [32][mq] (both sides)
    long mq;
    int c;                    // panel column
    int j;                    // panel index in the block
    int items;
    int reduce, factor;       // QR side switches
    const double *sgn;        // s_t of the panel whose pass preceded (V' = Q was used: corrections)
    int split;                // 1: kPI items, K1 in two halves; 0: 2 kPI items, one K range
    long cc;                  // column base in A and RwT: LQ the column of item 0 (c + 32 on one
                              // GPU, the rank's first local trailing column when the columns are
                              // sharded); QR the panel's first column (c; its local column)
    int zfill;                // LQ: items [items, zfill) of Qp stored as zeros (the distributed
                              // path's all-gather slot padding)
    // gram = 1: the panel QR's first Gram partials are formed here (k_cqr_gram
    // skipped): every workgroup's partial of its items (prescaled by its own
    // power of two) -> gpp[wg][0, 1024), its exponent gpp[wg][1024] (records
    // kGramRec apart); the last of the workgroups
    // covering a 256-item group (arrival counter gcnt[group], self-resetting)
    // sums them in fixed order -> gout[group][1024], gew[group] (CqrWs gp1 /
    // ew: what k_cqr_gram would have written)
    int vpatch = 0;           // LQ: V_j's top block as Q_t (the read pass folded k_vsum): Lt's
                              // diagonal of V_j gets - sgn here
    int upatch = 0;           // QR: U_{j-1}'s top block as Q_t: Rs's diagonal of U_{j-1} gets - sgn
    int gram = 0;
    double *gpp = nullptr, *gout = nullptr, *gew = nullptr;
    int *gcnt = nullptr;
};

constexpr int kLG = 194;   // LQ pitches (= 2 mod 32: conflict-free A-operand reads)
constexpr int kLW = 226;
constexpr int kQP = 40;    // QR pitch (rows k, k + 2 in opposite bank halves)

// ---- k_cqr_* (brd_blk_cqr.hip) ----------------------------------------------
constexpr int kCT = 256;
constexpr int kSP = 34;   // pitch of the 32 x 32 LDS matrices (even: 16-byte pairs)
constexpr int kCW = 128;  // most workgroups per panel (M <= kCW kCT rows; the distributed LQ panel
                          // is padded per rank: P x roundup(local columns, 256) rows)
constexpr long kQS = (long)kCW * kCT;   // column stride of Q1 in the workspace ([32][kQS]: a lane per row, coalesced)

#ifndef BRD_HANDOFF_RELAXED
#define BRD_HANDOFF_RELAXED 0   // 1: the relaxed (guide-measured) form of the prep / read-pass hand-offs (A/B)
#endif
constexpr int kBlkMaxRanks = 16;   // the blocked distributed path's most ranks (the tail's nranks b <= kRmax)
constexpr int kCqrRec = 1032;      // doubles per rank record: a 32 x 32 Gram, its exponent (128-B lines)
struct CqrArgs {
    const void *src; long si, st;     // P(i, t) = src[i*si + t*st]
    int M;
    void *vdst; long vsi, vst;        // V(i, t)
    void *vdst2; long vsi2, vst2;     // optional second copy of V (null: none)
    void *tout;                       // T (32 x 32)
    void *apan; long asi, ast;        // the panel in A: (i, t)
    double *ws;                       // scratch (cqr_ws_doubles)
    int *err;
    int azero;                        // 1: zeros into the panel's rows >= 32 (apan); 0: the caller zeroes
    double *qcopy;                    // optional copy of Q_t (1024 doubles, row-major) and the zero-panel
                                      // flag (element 1024): the distributed path's broadcast (null: none)
    // The distributed row panel (blk_ge2band_dist): this rank's rows only,
    // the panel-wide Grams from per-rank records all-gathered between the
    // kernels.  rec null: the whole panel is here (one GPU).
    double *rec;                      // record banks [3][nrec][kCqrRec]: G1 (+ exponent), G2, G3
    int nrec, rme;                    // ranks, this rank's record
    int *rctr;                        // 3 arrival counters (self-resetting): the last workgroup of a
                                      // kernel sums the partials into this rank's record
    long Mg;                          // the panel's rows over all ranks (the sCQR3 shift)
    long goff;                        // this rank's first row in the panel (completion vectors)
    int top;                          // 1: rows 0..31 here are the panel's top block (its R' and LU);
                                      // 0: every row here is below it (zeroed in apan from row 0)
};

// scratch (doubles): three slots of Gram partials [kCW][1024] (two used), the
// per-workgroup exponents, R1, the shifted-pass flag, and Q1 [32][kCW kCT]
__host__ __device__ constexpr size_t cqr_ws_doubles() {   // gp3: the distributed middle pass
    return (size_t)3 * 1024 * kCW + kCW + 2048 + 4 + (size_t)kCW * kCT * 32;
}
// Q_t (qt) and the zero flag are read by the next read pass's finishing
// workgroup (cqr_finish)
__host__ __device__ constexpr size_t cqr_ws_qt() { return (size_t)3 * 1024 * kCW + kCW + 1024; }
__host__ __device__ constexpr size_t cqr_ws_zero() { return cqr_ws_qt() + 1024 + 2; }
struct CqrWs {
    double *gp1, *gp2, *gp3, *ew, *r1, *qt, *shifted, *zero, *q1;
    __device__ explicit CqrWs(double *ws)
        : gp1(ws), gp2(ws + 1024 * kCW), gp3(ws + 2048 * kCW), ew(ws + 3072 * kCW), r1(ws + 3072 * kCW + kCW),
          qt(ws + cqr_ws_qt()), shifted(ws + cqr_ws_qt() + 1024), zero(ws + cqr_ws_zero()),
          q1(ws + cqr_ws_zero() + 2) {}
};

struct CqrLds {
    // the 32 x 32 matrices first: their LDS addresses fit the 16-bit offset field
    double g[32][kSP];       // reduced Gram
    double r1[32][kSP];      // R1 (upper, row-major)
    double r2[32][kSP];      // R2
    double u[32][kSP];       // U of the top block's LU (upper)
    double mm[32][kSP];      // L^-1
    double tq[32][kSP];      // Q's top block; then L (strict lower)
    double r1w[32][kSP];     // R1 in trsm_row's form; then U^-1
    double r2w[32][kSP];     // R2^-1 (first order) or R2 in trsm_row's form
    double sgn[32];
    double scl[kCW];         // per-partial scale factors of the Gram sum
    int e_w;
    int flags;
    double q[4][64][33];     // per-wave staging of 64 rows (Gram, coalesced stores); per-wave Gram partials
};
// The LDS of k_cqr_gram / k_cqr_q1: only what they use, the Gram staged in
// halves of 32 rows per wave (gram_wave) -- 61 KB against CqrLds' 139 KB, so
// in a stream of reductions such a workgroup leaves room on its CU for a
// k_blkupd_p workgroup (88 KB) instead of holding the whole CU.
struct CqrLdsS {
    double g[32][kSP];
    double r1[32][kSP];
    double r1w[32][kSP];
    double scl[kCW];
    int e_w;
    int flags;
    double q[4][32][33];
};

__device__ __forceinline__ double rdl(double v, int l) {   // lane l's value, wave-uniform
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

// Modified LU of Q_t - S = L U (Ballard et al. 2015: s_j = -sign of the
// pivot, so every pivot has |.| >= 1) by one wave, lane r holding row r
// (lanes 32-63 mirror).  The pivot row is lane jj's registers, broadcast by
// readlanes (measured: 27 k clocks for the 32 steps; the same loop with the
// pivot row published in LDS by its owner and read back as 16-byte
// broadcasts took 34 k).  On return lane r's rv holds row r of L (strict
// lower, unit diagonal implied) and U (upper); sgn[j] = s_j (LDS).
__device__ __forceinline__ void lu_wave(double (&rv)[32], double *sgn, int lane) {
    const int r = lane & 31;
#pragma unroll
    for (int jj = 0; jj < 32; ++jj) {
        double piv = rdl(rv[jj], jj);
        const double sg = piv >= 0 ? -1.0 : 1.0;
        piv -= sg;                                    // |piv| >= 1
        double inv = __builtin_amdgcn_rcp(piv);
        inv = fma(inv, fma(-piv, inv, 1.0), inv);
        inv = fma(inv, fma(-piv, inv, 1.0), inv);
        if (lane == 0) sgn[jj] = sg;
        const bool below = r > jj;
        const double l = rv[jj] * inv;
        const double lb = below ? l : 0.0;   // rows <= jj: an exact no-op update, no selects
#pragma unroll
        for (int cc = jj + 1; cc < 32; ++cc) {
            const double u = rdl(rv[cc], jj);
            rv[cc] = fma(-lb, u, rv[cc]);
            if (((cc - jj) & 7) == 0) __builtin_amdgcn_sched_barrier(0);   // bounds live scalar registers
        }
        rv[jj] = below ? l : (r == jj ? piv : rv[jj]);
    }
}

// One 16 x 16 tile (ti, tj) of C = A B for 32 x 32 matrices in LDS, K range
// [k0, 32) (k0 a multiple of 4: triangular operands skip their zero blocks).
__device__ __forceinline__ Mf<double>::v4 tile_mm(const double (&A)[32][kSP], const double (&B)[32][kSP], int ti, int tj,
                                                 int lane, int k0, int k1) {
    const int q = lane >> 4, l15 = lane & 15;
    Mf<double>::v4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int k = k0; k < k1; k += 4) acc = Mf<double>::mma(A[16 * ti + l15][k + q], B[k + q][16 * tj + l15], acc);
    return acc;
}
__device__ __forceinline__ void tile_store(double (&C)[32][kSP], const Mf<double>::v4 &t, int ti, int tj, int lane) {
#pragma unroll
    for (int g = 0; g < 4; ++g) C[16 * ti + Mf<double>::crow(lane >> 4, g)][16 * tj + (lane & 15)] = t[g];
}

// --------------------------------------------------------------------------
// cqr_finish: the rest of a panel's reconstruction, run by the first
// workgroup of the read pass that follows the panel (k_rpass), beside the
// pass itself -- the read pass uses V' = Q (the modified LU's signs enter
// only V's top block, and Y_j = A^T V_j T_j is corrected by prep).  Wave 0:
// the modified LU of Q_t - S = L U (s_j = -sign of the pivot); then wave 1
// U^-1, wave 2 L^-1, wave 3 the band block R = S R' in place; then every
// wave one tile of T = -S (U^-1 L^-1)^T.  A zero panel gets S = -I, T = 0.
// All 512 threads of the workgroup pass the barriers; waves 4-7 idle.
// --------------------------------------------------------------------------
struct FinArgs {
    const double *qt;     // Q_t (32 x 32, row-major)
    const double *zero;   // 1: the panel was zero
    double *sgn;          // out: s_j
    void *tout;           // out: T
    void *apan; long asi, ast;   // the band block R' (in place -> S R')
};
struct FinLds {
    double u[32][kSP];       // U (upper)
    double tq[32][kSP];      // Q_t, then L (strict lower)
    double ui[32][kSP];      // U^-1
    double li[32][kSP];      // L^-1
    double sgn[32];
};

// (LDS matrices passed separately: k_cqr_v's inline use maps them onto its
// own; tq_loaded: Q_t is already in tq)
template <typename T>
__device__ __forceinline__ void cqr_finish(double (&Lu)[32][kSP], double (&Ltq)[32][kSP], double (&Lui)[32][kSP],
                                           double (&Lli)[32][kSP], double *Lsgn, const FinArgs &f, int tid,
                                           bool tq_loaded) {
    const int lane = tid & 63, w = tid >> 6;
    const bool zero = f.zero[0] != 0.0;
    if (!tq_loaded)
        for (int el = tid; el < 1024; el += blockDim.x) Ltq[el >> 5][el & 31] = f.qt[el];
    __syncthreads();
    if (w == 0) {
        const int r = lane & 31;
        double rv[32];
#pragma unroll
        for (int cc = 0; cc < 32; ++cc) rv[cc] = Ltq[r][cc];
        if (!zero) {
            lu_wave(rv, Lsgn, lane);
        } else {
#pragma unroll
            for (int jj = 0; jj < 32; ++jj) rv[jj] = r == jj ? 1.0 : 0.0;
            if (lane < 32) Lsgn[lane] = -1.0;
        }
        if (lane < 32) {
#pragma unroll
            for (int cc = 0; cc < 32; ++cc) Lu[r][cc] = cc >= r ? rv[cc] : 0.0;
#pragma unroll
            for (int cc = 0; cc < 32; ++cc) Ltq[r][cc] = cc < r ? rv[cc] : 0.0;
        }
    }
    __syncthreads();
    if (w == 0) {
        if (lane < 32) f.sgn[lane] = Lsgn[lane];
    } else if (w == 1) {
        // U^-1 (lane c = column c, right-looking back substitution)
        const int c = lane & 31;
        double acc[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = k == c ? 1.0 : 0.0;
#pragma unroll
        for (int k = 31; k >= 0; --k) {
            const double d = Lu[k][k];
            double inv = __builtin_amdgcn_rcp(d);
            inv = fma(inv, fma(-d, inv, 1.0), inv);
            inv = fma(inv, fma(-d, inv, 1.0), inv);
            const double xk = acc[k] * inv;
            acc[k] = xk;
#pragma unroll
            for (int i2 = 0; i2 < k; ++i2) acc[i2] = fma(-Lu[i2][k], xk, acc[i2]);
        }
        if (lane < 32) {
#pragma unroll
            for (int k = 0; k < 32; ++k) Lui[k][c] = acc[k];
        }
    } else if (w == 2) {
        // L^-1 (unit lower; lane c = column c, forward substitution)
        const int c = lane & 31;
        double acc[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = k == c ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const double xk = acc[k];
#pragma unroll
            for (int i2 = k + 1; i2 < 32; ++i2) acc[i2] = fma(-Ltq[i2][k], xk, acc[i2]);
        }
        if (lane < 32) {
#pragma unroll
            for (int k = 0; k < 32; ++k) Lli[k][c] = acc[k];
        }
    } else if (w == 3 && f.apan) {
        // R = S R' (upper block, rows scaled by s_i; the distributed path: on
        // the rank holding the band block only)
        T *ap = (T *)f.apan;
        for (int el = lane; el < 1024; el += 64) {
            const int i2 = el >> 5, c = el & 31;
            if (i2 <= c) {
                T *pp = ap + (size_t)i2 * f.asi + (size_t)c * f.ast;
                *pp = (T)(Lsgn[i2] * (double)*pp);
            }
        }
    }
    __syncthreads();
    if (w < 4) {
        // T = -S (U^-1 L^-1)^T: wave w forms tile (w >> 1, w & 1) of U^-1 L^-1
        const int ti = w >> 1, tj = w & 1;
        const Mf<double>::v4 pt = tile_mm(Lui, Lli, ti, tj, lane, 16 * (ti > tj ? ti : tj), 32);
        T *tout = (T *)f.tout;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int i2 = 16 * ti + Mf<double>::crow(lane >> 4, g), j2 = 16 * tj + (lane & 15);
            tout[j2 * 32 + i2] = (T)(zero ? 0.0 : -Lsgn[j2] * pt[g]);
        }
    }
}

template <typename T>
__device__ void cqr_finish_entry(const FinArgs &f, int tid, void *lds) {
    static_assert(sizeof(FinLds) <= kRpLds * sizeof(double), "cqr_finish's LDS exceeds the read pass's block");
    FinLds &FL = *reinterpret_cast<FinLds *>(lds);
    cqr_finish<T>(FL.u, FL.tq, FL.ui, FL.li, FL.sgn, f, tid, false);
}

// ---- k_blkupd (brd_blk_upd.hip) ---------------------------------------------
constexpr int kGT = 256;
constexpr int kGM = 128;
constexpr int kGKC = 16;
constexpr int kGBP = kGM + 16;

struct GemmArgs {
    void *C; long ldc;
    int rows, cols;                 // extent of the updated region
    const void *Lw; const void *RwT; long ldr;
    int K;                          // 256
    int tiles_c;                    // column tiles
    int ntiles;                     // tiles
    int nfull = 0, nh = 0;          // k_blkupd_p: nh > 0: tiles [0, nfull) whole, then
                                    // nh half tiles (64 rows) of tiles nfull, nfull + 1, ...
    int xsr = 0, xsc = 0;           // k_blkupd_p: > 0: per-XCD super-tiles of xsr x xsc tiles
                                    // (xsr xsc = grid / 8; blkupd_tile), else row-major order
};

// k_blkupd_p's tile order.  Tile q of the order -> (tile row, tile column).
// With super-tiles (xsr > 0) the full xsr x xsc blocks come first, each one's
// tiles row-major, then the right strip and the bottom strip row-major;
// otherwise row-major.
__host__ __device__ inline void blkupd_tile(const GemmArgs &a, int q, int &tr, int &tc) {
    if (a.xsr <= 0) { tr = q / a.tiles_c; tc = q % a.tiles_c; return; }
    const int tiles_r = a.ntiles / a.tiles_c, nsc = a.tiles_c / a.xsc;
    const int Rf = (tiles_r / a.xsr) * a.xsr, Cf = nsc * a.xsc, per = a.xsr * a.xsc;
    if (q < Rf * Cf) {
        const int st = q / per, w = q - st * per;
        tr = (st / nsc) * a.xsr + w / a.xsc;
        tc = (st % nsc) * a.xsc + w % a.xsc;
        return;
    }
    int e = q - Rf * Cf;
    const int rw = a.tiles_c - Cf;
    if (e < Rf * rw) { tr = e / rw; tc = Cf + e % rw; return; }
    e -= Rf * rw;
    tr = Rf + e / a.tiles_c;
    tc = e % a.tiles_c;
}

// ---- LDS-DMA and raw buffer accesses (k_blkupd_p, k_rpass_d) -----------------
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// 16 bytes per lane from a raw buffer (offset past num_records reads 0) into
// LDS at lds_byte + 16 lane; counted by vmcnt, invisible to the compiler
// (soffset: a wave-uniform byte offset added to voff)
__device__ __forceinline__ void dma16(u32x4_t rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_byte)),
                   "s"(__builtin_amdgcn_readfirstlane(soff))
                 : "memory");
}
// raw buffer descriptor: base address, stride 0, num_records 2^31 - 1, the
// same flags word as __builtin_amdgcn_make_buffer_rsrc(..., 0x00020000)
// the same with the non-temporal policy (nt): once-read streams
__device__ __forceinline__ void dma16_nt(u32x4_t rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_byte)),
                   "s"(__builtin_amdgcn_readfirstlane(soff)) : "memory");
}
__device__ __forceinline__ u32x4_t rsrc_of(const void *base) {
    const unsigned long long p = (unsigned long long)(uintptr_t)base;
    return u32x4_t{(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)p),
                   (unsigned)__builtin_amdgcn_readfirstlane((int)((unsigned)(p >> 32) & 0xffffu)), 0x7fffffffu,
                   0x00020000u};
}
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
// AUX: the cache-policy bits (gfx950: 1 sc0, 2 nt, 16 sc1)
template <typename T, int AUX = 0> __device__ __forceinline__ T buf_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
    if constexpr (sizeof(T) == 8)
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, AUX));
    else
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, AUX));
}
template <typename T, int AUX = 0> __device__ __forceinline__ void buf_st(T v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    if constexpr (sizeof(T) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, (int)off, 0, AUX);
    else
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, 0, AUX);
}

// ---- launches ----------------------------------------------------------------
// Every launch of the blocked path goes through blk_launch: with brd_profile
// on, the launch itself stamps its start and end (hipExtLaunchKernel), tagged
// with the kernel's algorithmic flops and HBM bytes (bench.py's roofline
// objects).
template <typename F, typename... Args>
static inline void blk_launch(const char *kind, double flops, double bytes, F kernel, dim3 grid, dim3 block,
                              hipStream_t s, Args... args) {
    hipEvent_t ea, eb;
    if (api_prof_launch_events(kind, flops, bytes, &ea, &eb, (int)(grid.x * grid.y)))
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, ea, eb, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}

// host launchers, one per kernel family, defined beside the kernels
// k_rpass_d (the LDS-DMA read pass) runs this pass: no 16-byte vector
// straddling a source's end, rows 16-byte aligned, not disabled by
// BRD_RPASS_DMA=0; its stages hold rpass_stage_k(elem) k each
bool rpass_dma_ok(bool yp, int K, int M, size_t elem, const void *src, long ld, const void *vsrc, long vld,
                  const void *bsrc, long bld);
int rpass_stage_k(size_t elem);
template <typename T>
void launch_k_rpass(bool yp, dim3 grid, const RpArgs &a, const FinArgs &f, hipStream_t s, double fl, double by);
template <typename T>
void launch_k_vsum(const T *vpart, T *vout, int nvirt, T *pbase, long pstride, const double *sgn, hipStream_t s);
template <typename T>
void launch_k_prep(bool lq, dim3 grid, const PrepArgs &p, hipStream_t s);
enum CqrKernel { kCqrGram, kCqrQ1, kCqrV, kCqrVInline, kCqrMid };
template <typename T>
void launch_k_cqr(CqrKernel which, int nwg, const CqrArgs &a, const FinArgs &f, hipStream_t s);
template <typename T>
void launch_k_blkupd(dim3 grid, const GemmArgs &g, hipStream_t s, double fl, double by);
// the distributed path's data movement (brd_blk_comm.hip)
template <typename T>
void launch_dist_unpack_v(const T *src, T *dst, int M, hipStream_t s);
template <typename T>
void launch_dist_psum(const T *part, int ks, long mp, int rows, T *buf, hipStream_t s);

}  // namespace blk
}  // namespace brd
