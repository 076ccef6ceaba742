// Stage 1, blocked: dense -> band with a delayed two-sided update (gfx950).
//
// Replaces, for panels of width 32, the per-panel structure of the
// reference's cuda_brd_p1 (svd_cuda_2.cu:1117-1220: QR of the column panel,
// qr_apply_cuda :1039 over the whole trailing matrix, LQ of the row panel,
// lq_apply_cuda :1081 over it again).  Inside a block of nb panels the
// trailing matrix is not written; it is kept as
//
//     A_cur = A - Lw RwT          Lw  (m x 256) = [V_0..V_3 | X_0..X_3]
//                                 RwT (256 x n) = [Y_0..Y_3 | U_0..U_3]^T
//
// (left reflectors I - V_j T_j V_j^T, right reflectors I - U_j S_j U_j^T,
// Y_j = A_cur^T V_j T_j, X_j = A_cur U_j S_j) and updated once per block by
// k_blkupd, a rank-2 nb 32 product on the matrix cores.  Per panel:
//
//   k_rpass (Y)  partial sums of A^T V_j over row splits, and G = Lw^T V_j
//   k_prep (LQ)  Y_j = (A^T V_j - Rw G) T_j, the corrected row panel
//   k_cqr        QR of the row panel's transpose: CholeskyQR2 + Householder
//                reconstruction -> U_j, S_j, the band's L block
//   k_rpass (X)  partial sums of A U_j over column splits, and G = Rw^T U_j
//   k_prep (QR)  X_j = (A U_j - Lw G) S_j, the next corrected column panel
//   k_cqr        QR of the column panel -> V_{j+1}, T_{j+1}, the band's R block
//
// The executable specification (same steps, same workspaces) is
// tests/s1_model.py; DESIGN.md "Stage 1, blocked" has the roofline of each
// kernel.  This file is the host driver; the kernels live in brd_blk_*.hip
// (brd_blk.h).
#include "brd_blk.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace brd {

// --------------------------------------------------------------------------
// Host side
// --------------------------------------------------------------------------
using namespace blk;

// Workspace of the blocked path (elements of T unless noted), carved from one
// device buffer: Lw m x 256, RwT 256 x ldr, partials, Qp, virtual partials
// and result, T/S factors, cluster scratch (doubles) and counters (ints).
struct BlkLayout {
    size_t lw, rwt, ub, part, vpart, vout, qp, tf, cws, ctr, sg, total;
    long ldr, mp;
    int ksmax, cwg;
};

static BlkLayout blk_layout(int m, int n, size_t elem) {
    BlkLayout L;
    L.ldr = (n + 1) & ~1L;
    L.mp = (std::max(m, n) + 1) & ~1L;
    L.ksmax = 32;
    L.cwg = kCW;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    L.lw = take((size_t)m * 256 * elem);
    L.rwt = take((size_t)256 * L.ldr * elem);
    L.ub = take((size_t)n * 32 * elem);
    L.part = take((size_t)L.ksmax * 32 * L.mp * elem);
    L.vpart = take((size_t)L.ksmax * 32 * 256 * elem);
    L.vout = take((size_t)32 * 256 * elem);
    L.qp = take((size_t)32 * L.mp * elem);
    L.tf = take((size_t)8 * 1024 * elem);
    L.cws = take(cqr_ws_doubles() * sizeof(double));
    L.ctr = take(64 * sizeof(int));
    L.sg = take((size_t)(2 * NBMAX + 1) * 32 * sizeof(double));   // s_j per panel and side; zeros
    L.total = off;
    return L;
}

size_t blk_ws_bytes(int m, int n, size_t elem) { return blk_layout(m, n, elem).total; }

int blk_columns(int m, int n, int b) {
    // panels of up to kCW x 256 rows (the panel QR's workgroup count)
    if (b != 32 || m > kCW * kCT || n > kCW * kCT) return 0;
    int k0 = 0;
    while (n - k0 >= (NBMAX + 1) * 32) k0 += NBMAX * 32;
    return k0;
}

// the prep kernels' grid: split K halves (kPI items per workgroup) while
// that grid fits the CUs the stream may use (one workgroup per CU: LDS),
// else 2 kPI items per workgroup, one K range per wave
static dim3 prep_grid(PrepArgs &p, int cus) {
    const int n1 = (p.items + kPI - 1) / kPI;
    p.split = n1 <= cus ? 1 : 0;
    return dim3(p.split ? n1 : (p.items + 2 * kPI - 1) / (2 * kPI));
}

template <typename T>
static hipError_t launch_rpass(bool yp, const T *src, long ld, int K, int M, const T *bsrc, long bld, const T *vsrc,
                               long vld, char *ws, const BlkLayout &Ly, int *counter, int *err, hipStream_t s,
                               int target, int *ksplit_out, const FinArgs *fin, T *pbase, long pstride,
                               const double *psgn) {
    RpArgs a;
    a.src = src; a.ld = ld; a.vsrc = vsrc; a.vld = vld; a.bsrc = bsrc; a.bld = bld;
    a.K = K; a.M = M;
    a.mtiles = (M + kMT - 1) / kMT;
    static const int rpx = getenv("BRD_BLK_RPX") ? std::max(1, atoi(getenv("BRD_BLK_RPX"))) : 1;   // tuning
    target *= rpx;
    int ks = std::max(1, target / std::max(1, a.mtiles + 1));
    ks = std::min(ks, std::max(1, K / 64));
    ks = std::min(ks, Ly.ksmax);
    a.kper = ((K + ks - 1) / ks + 7) / 8 * 8;
    ks = (K + a.kper - 1) / a.kper;
    a.ksplit = ks;
    a.nvirt = vsrc ? ks : 0;
    a.part = ws + Ly.part; a.mp = Ly.mp;
    a.vpart = ws + Ly.vpart; a.vout = ws + Ly.vout;
    a.counter = counter;
    a.err = err;
    a.has_fin = fin ? 1 : 0;
    const FinArgs fa = fin ? *fin : FinArgs{};
    *ksplit_out = ks;
    dim3 grid(a.has_fin + a.nvirt + a.mtiles * ks);
    // algorithmic: the K x M source read once, 2 x 32 flops per element
    const double fl = 2.0 * 32 * K * M, by = (double)K * M * sizeof(T);
    launch_k_rpass<T>(yp, grid, a, fa, s, fl, by);
    if (a.nvirt > 0) launch_k_vsum<T>((const T *)a.vpart, (T *)a.vout, a.nvirt, pbase, pstride, psgn, s);
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_cqr(const T *src, long si, long st, int M, T *vdst, long vsi, long vst, T *vdst2, long vsi2,
                             long vst2, T *tout, T *apan, long asi, long ast, char *ws, const BlkLayout &Ly, int *err,
                             hipStream_t s, bool inl, const FinArgs &fin) {
    CqrArgs a;
    a.src = src; a.si = si; a.st = st; a.M = M;
    a.vdst = vdst; a.vsi = vsi; a.vst = vst;
    a.vdst2 = vdst2; a.vsi2 = vsi2; a.vst2 = vst2;
    a.tout = tout; a.apan = apan; a.asi = asi; a.ast = ast;
    const int nwg = (M + kCT - 1) / kCT;
    if (nwg > Ly.cwg) return hipErrorInvalidValue;
    a.ws = (double *)(ws + Ly.cws);
    a.err = err;
    launch_k_cqr<T>(kCqrGram, nwg, a, fin, s);
    launch_k_cqr<T>(kCqrQ1, nwg, a, fin, s);
    launch_k_cqr<T>(inl ? kCqrVInline : kCqrV, nwg, a, fin, s);
    return hipGetLastError();
}

// Blocked stage 1 over columns [0, kend) (kend = blk_columns(m, n, 32) > 0);
// the caller finishes the remaining panels with the per-panel path.
template <typename T>
hipError_t blk_ge2band(T *A, int m, int n, long lda, void *wsv, hipStream_t s, int target, int *err) {
    char *ws = (char *)wsv;
    const BlkLayout Ly = blk_layout(m, n, sizeof(T));
    const int kend = blk_columns(m, n, 32);
    T *Lw = (T *)(ws + Ly.lw), *RwT = (T *)(ws + Ly.rwt), *Ub = (T *)(ws + Ly.ub);
    T *tf = (T *)(ws + Ly.tf);   // T_j at tf + 1024 j, S_j at tf + 1024 (4 + j)
    int *ctr = (int *)(ws + Ly.ctr);
    const long ldr = Ly.ldr;
    hipError_t e = hipMemsetAsync(ctr, 0, 64 * sizeof(int), s);
    if (e != hipSuccess) return e;
    double *sgq = (double *)(ws + Ly.sg), *sgl = sgq + NBMAX * 32, *sg0 = sgq + 2 * NBMAX * 32;
    e = hipMemsetAsync(sg0, 0, 32 * sizeof(double), s);   // "no correction"
    if (e != hipSuccess) return e;
    const double *cws = (const double *)(ws + Ly.cws);
    // A panel's reconstruction finishes (modified LU, T, the band block's
    // signs) in the first workgroup of the read pass that follows it, which
    // uses V' = Q; the last LQ panel of a block finishes inline (the block
    // update reads its U straight away).
    auto fin_of = [&](double *sg, T *tout, T *apan, long asi, long ast) {
        FinArgs f;
        f.qt = cws + cqr_ws_qt(); f.zero = cws + cqr_ws_zero(); f.sgn = sg;
        f.tout = tout; f.apan = apan; f.asi = asi; f.ast = ast;
        return f;
    };
    int ks_x = 1;
    const double *sg_prev = sg0;   // s of the previous LQ panel (prep_qr's correction)
    for (int k0 = 0; k0 < kend; k0 += NBMAX * 32) {
        for (int j = 0; j < NBMAX; ++j) {
            const int c = k0 + 32 * j;
            const int mr = m - c;          // rows of the column panel
            const int n2 = n - c - 32;     // columns right of it
            T *Tj = tf + 1024 * j, *Sj = tf + 1024 * (NBMAX + j);
            // ---- QR of the column panel --------------------------------------
            const FinArgs fq = fin_of(sgq + 32 * j, Tj, A + (size_t)c * lda + c, lda, 1);
            if (j == 0) {
                e = launch_cqr<T>(A + (size_t)c * lda + c, lda, 1, mr, Lw + (size_t)c * 256, 256, 1, nullptr, 0, 0, Tj,
                                  A + (size_t)c * lda + c, lda, 1, ws, Ly, err, s, false, fq);
            } else {
                PrepArgs p;
                p.A = A; p.lda = lda; p.Lw = Lw; p.RwT = RwT; p.ldr = ldr;
                p.part = ws + Ly.part; p.mp = Ly.mp; p.ksplit = ks_x;
                p.G = ws + Ly.vout; p.Tm = tf + 1024 * (NBMAX + j - 1);
                p.Qp = ws + Ly.qp; p.mq = Ly.mp;
                p.c = c; p.j = j; p.items = mr; p.reduce = 1; p.factor = 1;
                p.sgn = sg_prev;
                launch_k_prep<T>(false, prep_grid(p, target), p, s);
                e = hipGetLastError();
                if (e != hipSuccess) return e;
                e = launch_cqr<T>((const T *)(ws + Ly.qp), 1, Ly.mp, mr, Lw + (size_t)c * 256 + 32 * j, 256, 1, nullptr, 0, 0, Tj,
                                  A + (size_t)c * lda + c, lda, 1, ws, Ly, err, s, false, fq);
            }
            if (e != hipSuccess) return e;
            // ---- Y pass (+ the QR panel's finish) + LQ of the row panel -------
            int ks_y = 1;
            e = launch_rpass<T>(true, A + (size_t)c * lda + c + 32, lda, mr, n2, Lw + (size_t)c * 256 + 32 * j, 256,
                                Lw + (size_t)c * 256, 256, ws, Ly, ctr + 16, err, s, target, &ks_y, &fq,
                                Lw + (size_t)c * 256 + 32 * j, 257, sgq + 32 * j);
            if (e != hipSuccess) return e;
            {
                PrepArgs p;
                p.A = A; p.lda = lda; p.Lw = Lw; p.RwT = RwT; p.ldr = ldr;
                p.part = ws + Ly.part; p.mp = Ly.mp; p.ksplit = ks_y;
                p.G = ws + Ly.vout; p.Tm = Tj;
                p.Qp = ws + Ly.qp; p.mq = Ly.mp;
                p.c = c; p.j = j; p.items = n2; p.reduce = 0; p.factor = 0;
                p.sgn = sgq + 32 * j;
                launch_k_prep<T>(true, prep_grid(p, target), p, s);
                e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            const bool inl = j == NBMAX - 1;
            const FinArgs fl = fin_of(sgl + 32 * j, Sj, A + (size_t)c * lda + c + 32, 1, lda);
            e = launch_cqr<T>((const T *)(ws + Ly.qp), 1, Ly.mp, n2, RwT + (size_t)(128 + 32 * j) * ldr + c + 32, 1, ldr,
                              Ub + (size_t)(c + 32) * 32, 32, 1, Sj, A + (size_t)c * lda + c + 32, 1, lda, ws, Ly, err, s,
                              inl, fl);
            if (e != hipSuccess) return e;
            // ---- X pass (+ the LQ panel's finish) --------------------------------
            e = launch_rpass<T>(false, A + (size_t)(c + 32) * lda + c + 32, lda, n2, m - c - 32,
                                Ub + (size_t)(c + 32) * 32, 32, RwT + c + 32, ldr, ws, Ly, ctr + 16, err, s,
                                target, &ks_x, inl ? nullptr : &fl,
                                inl ? nullptr : RwT + (size_t)(128 + 32 * j) * ldr + c + 32, ldr + 1, sgl + 32 * j);
            if (e != hipSuccess) return e;
            sg_prev = inl ? sg0 : sgl + 32 * j;
        }
        // ---- block end: X_3, then the rank-256 update ---------------------------
        const int k1 = k0 + NBMAX * 32;
        {
            PrepArgs p;
            p.A = A; p.lda = lda; p.Lw = Lw; p.RwT = RwT; p.ldr = ldr;
            p.part = ws + Ly.part; p.mp = Ly.mp; p.ksplit = ks_x;
            p.G = ws + Ly.vout; p.Tm = tf + 1024 * (2 * NBMAX - 1);
            p.Qp = ws + Ly.qp; p.mq = Ly.mp;
            p.c = k1; p.j = NBMAX; p.items = m - k1; p.reduce = 1; p.factor = 0;
            p.sgn = sg_prev;   // the block's last LQ panel finished inline: zeros
            launch_k_prep<T>(false, prep_grid(p, target), p, s);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        {
            GemmArgs g;
            g.C = A + (size_t)k1 * lda + k1; g.ldc = lda;
            g.rows = m - k1; g.cols = n - k1;
            g.Lw = Lw + (size_t)k1 * 256; g.RwT = RwT + k1; g.ldr = ldr;
            g.K = 256;
            g.tiles_c = (g.cols + kGM - 1) / kGM;
            const int tiles_r = (g.rows + kGM - 1) / kGM;
            g.ntiles = tiles_r * g.tiles_c;
            const int grid = g.ntiles;
            // algorithmic: C read and written once, Lw / RwT read once; 2 x 256 flops per element
            const double el = (double)g.rows * g.cols;
            launch_k_blkupd<T>(dim3(grid), g, s, 2.0 * 256 * el, (2.0 * el + 256.0 * (g.rows + g.cols)) * sizeof(T));
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

template hipError_t blk_ge2band<double>(double *, int, int, long, void *, hipStream_t, int, int *);
template hipError_t blk_ge2band<float>(float *, int, int, long, void *, hipStream_t, int, int *);

}  // namespace brd
