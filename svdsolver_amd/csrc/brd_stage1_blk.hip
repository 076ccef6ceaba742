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
#include "brd.h"
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
    size_t lw, rwt, ub, part, vpart, vout, qp, tf, cws, ctr, sg, gpp, total;
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
    L.ctr = take((64 + kCW) * sizeof(int));   // counters; [64, 64 + kCW): prep Gram groups
    L.sg = take((size_t)(2 * NBMAX + 1) * 32 * sizeof(double));   // s_j per panel and side; zeros
    // the prep kernels' Gram partials (PrepArgs::gram): per workgroup of kPI items
    L.gpp = take((size_t)((std::max(m, n) + kPI - 1) / kPI) * kGramRec * sizeof(double));
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
// that grid fits the CUs the stream may use (one workgroup per CU: LDS) and
// nothing runs beside it, else 2 kPI items per workgroup, one K range per
// wave.  The two forms round the K1 sums differently, so a matrix's band
// depends on whether it ran in a stream -- as the read passes' split already
// does.  BRD_PREP_SPLIT=0 / 1 forces either form for A/B.
// cus: the CUs the stream may use (api_apply_target: fewer beside a stage-2
// reservation).  Sizing the split on the device's CUs instead (round 5,
// ADVICE r4) made the prep kernels' rounding independent of the overlap, but
// the read passes' K split already depends on it, and the
// 8-lane stream measured 24.07 against 24.26 TFLOP/s (N = 8192 fp64, same
// box): so the target, as in round 4.
// Beside a stage-2 reservation (a stream of reductions) at N <= 12288 the
// prep kernels do not split K and the read passes are sized for half the
// target (prep_grid, launch_rpass): at 8192 the 8-lane stream went 24.4 ->
// 25.2 TFLOP/s; at 16384 the same sizing took it from 33.4 to 25.9 (30.3 with
// the halving on passes <= 12288 wide only), so larger matrices keep the
// one-at-a-time sizing.
//
// The sizing of one call's launches is fixed when the call starts and passed
// to every launcher (no hidden per-thread state):
//   target  workgroups a bandwidth launch may fill (api_apply_target: the
//           device's CUs, less a stage-2 reservation);
//   lean    beside a stage-2 reservation and max(m, n) <= kLeanMaxN: no prep
//           K split, read passes sized for target / 2 (the measured rule above).
static constexpr int kLeanMaxN = 12288;
struct S1Launch {
    int target;
    bool lean;
};
static S1Launch s1_launch(int m, int n, int target) {
    return S1Launch{target, api_overlap_active() && std::max(m, n) <= kLeanMaxN};
}
static dim3 prep_grid(PrepArgs &p, const S1Launch &lc) {
    const int items = std::max(p.items, p.zfill);
    const int n1 = (items + kPI - 1) / kPI;
    const int mode = getenv("BRD_PREP_SPLIT") ? atoi(getenv("BRD_PREP_SPLIT")) : -1;   // A/B: 0 never, 1 always
    // beside other work (a stage-2 reservation: a stream of reductions) never
    // split: half the workgroups, each holding a whole CU (LDS) for the same
    // ~20 us, leave CUs to the other lanes' passes (8-lane stream, N = 8192
    // fp64, same box: 24.36 / 24.39 -> 24.82 / 24.55 TFLOP/s)
    p.split = mode == 0 ? 0 : (mode == 1 || (n1 <= lc.target && !lc.lean)) ? 1 : 0;
    return dim3(std::max(1, p.split ? n1 : (items + 2 * kPI - 1) / (2 * kPI)));
}

template <typename T>
static hipError_t launch_rpass(bool yp, const T *src, long ld, int K, int M, const T *bsrc, long bld, const T *vsrc,
                               long vld, char *ws, const BlkLayout &Ly, int *counter, int *err, hipStream_t s,
                               const S1Launch &lc, int *ksplit_out, const FinArgs *fin, T *pbase, long pstride,
                               const double *psgn, void *vout = nullptr, bool *vfolded = nullptr, int va = 0,
                               int vb = 0) {
    RpArgs a;
    a.src = src; a.ld = ld; a.vsrc = vsrc; a.vld = vld; a.bsrc = bsrc; a.bld = bld;
    a.K = K; a.M = M;
    a.mtiles = (M + kMT - 1) / kMT;
    // Beside a stage-2 reservation (a stream of reductions) a pass is sized for
    // half the CUs: the other lanes' kernels run on the rest (8-lane stream,
    // N = 8192 fp64, same box: target x 1 / 0.75 / 0.5 / 0.375 / 0.25 ->
    // 24.73-24.84 / 24.94 / 25.05-25.15 / 24.78 / 24.10-24.23 TFLOP/s).
    // BRD_BLK_RPX scales the target further (A/B).
    static const double rpx = getenv("BRD_BLK_RPX") ? std::max(0.125, atof(getenv("BRD_BLK_RPX"))) : 1.0;
    int target = lc.lean ? std::max(1, lc.target / 2) : lc.target;
    target = std::max(1, (int)(target * rpx));
    int ks, nwg;
    a.tiles = a.ns = a.wst = 0;
    if (rpass_dma_ok(yp, K, M, sizeof(T), src, ld, vsrc, vld, bsrc, bld) && K > 0) {
        // k_rpass_d: the tiles' stages (32 KB of a 256-wide tile each) laid end
        // to end and dealt in equal runs of wst stages, one run per workgroup
        a.tiles = a.mtiles + (vsrc ? 1 : 0);
        const int krk = rpass_stage_k(sizeof(T));
        a.ns = (K + krk - 1) / krk;
        const long tot = (long)a.tiles * a.ns;
        int wst = (int)((tot + target - 1) / std::max(1, target));
        wst = std::max(wst, std::max(1, 64 / krk));   // >= 64 k per workgroup
        wst = std::max(wst, (a.ns + Ly.ksmax - 2) / (Ly.ksmax - 1));   // <= ksmax slots per tile
        a.wst = wst;
        nwg = (int)((tot + wst - 1) / wst);
        ks = 1;
        for (int t = 0; t < a.tiles; ++t)
            ks = std::max(ks, (int)(((long)(t + 1) * a.ns - 1) / wst - ((long)t * a.ns) / wst + 1));
        a.kper = 0;
    } else {
        ks = std::max(1, target / std::max(1, a.mtiles + 1));
        ks = std::min(ks, std::max(1, K / 64));
        ks = std::min(ks, Ly.ksmax);
        a.kper = ((K + ks - 1) / ks + 7) / 8 * 8;
        ks = (K + a.kper - 1) / a.kper;
        nwg = (vsrc ? ks : 0) + a.mtiles * ks;
    }
    a.ksplit = ks;
    a.nvirt = vsrc ? ks : 0;
    a.part = ws + Ly.part; a.mp = Ly.mp;
    a.vpart = ws + Ly.vpart; a.vout = vout ? vout : ws + Ly.vout;
    a.counter = counter;
    a.err = err;
    a.has_fin = fin ? 1 : 0;
    const FinArgs fa = fin ? *fin : FinArgs{};
    *ksplit_out = ks;
    dim3 grid(a.has_fin + nwg);
    // algorithmic: the K x M source read once, 2 x 32 flops per element
    const double fl = 2.0 * 32 * K * M, by = (double)K * M * sizeof(T);
    // the virtual tile's partials summed inside k_rpass_d (the last of its
    // contributors to arrive; only the entries the consumer reads) when the
    // caller's consumers patch V's / U's top block themselves (vfolded) --
    // beside other work only (brd_set_overlap: a stream of reductions), where
    // one fewer launch per pass is worth more than the pass's longer tail:
    // N = 8192 fp64 stream 23.6 -> 25.0 TFLOP/s, one at a time stage 1
    // 73.4 -> 75.6 ms.  The sum's order and the patch are k_vsum's, so the
    // band is bitwise the same either way.  BRD_VSUM_FOLD=0 / 1 forces it.
    const char *vfe = getenv("BRD_VSUM_FOLD");
    const bool want = vfe ? atoi(vfe) != 0 : api_overlap_active();
    a.vfold = (vfolded && want && a.wst > 0 && a.nvirt > 0) ? 1 : 0;
    a.va = va; a.vb = vb;
    if (vfolded) *vfolded = a.vfold != 0;
    launch_k_rpass<T>(yp, grid, a, fa, s, fl, by);
    if (a.nvirt > 0 && !a.vfold) launch_k_vsum<T>((const T *)a.vpart, (T *)a.vout, a.nvirt, pbase, pstride, psgn, s);
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_cqr(const T *src, long si, long st, int M, T *vdst, long vsi, long vst, T *vdst2, long vsi2,
                             long vst2, T *tout, T *apan, long asi, long ast, char *ws, const BlkLayout &Ly, int *err,
                             hipStream_t s, bool inl, const FinArgs &fin, int azero = 1, double *qcopy = nullptr,
                             bool gram_done = false) {
    CqrArgs a;
    a.rec = nullptr; a.nrec = 1; a.rme = 0; a.rctr = nullptr;
    a.Mg = M; a.goff = 0; a.top = 1;
    a.src = src; a.si = si; a.st = st; a.M = M;
    a.vdst = vdst; a.vsi = vsi; a.vst = vst;
    a.vdst2 = vdst2; a.vsi2 = vsi2; a.vst2 = vst2;
    a.tout = tout; a.apan = apan; a.asi = asi; a.ast = ast;
    const int nwg = (M + kCT - 1) / kCT;
    if (nwg > Ly.cwg) return hipErrorInvalidValue;
    a.ws = (double *)(ws + Ly.cws);
    a.err = err;
    a.azero = azero;
    a.qcopy = qcopy;
    if (!gram_done) launch_k_cqr<T>(kCqrGram, nwg, a, fin, s);   // else the prep kernel formed gp1 / ew
    launch_k_cqr<T>(kCqrQ1, nwg, a, fin, s);
    launch_k_cqr<T>(inl ? kCqrVInline : kCqrV, nwg, a, fin, s);
    return hipGetLastError();
}

// Blocked stage 1 over columns [0, kend) (kend = blk_columns(m, n, 32) > 0);
// the caller finishes the remaining panels with the per-panel path.
template <typename T>
hipError_t blk_ge2band(T *A, int m, int n, long lda, void *wsv, hipStream_t s, int target, int *err) {
    const S1Launch lc = s1_launch(m, n, target);
    char *ws = (char *)wsv;
    const BlkLayout Ly = blk_layout(m, n, sizeof(T));
    const int kend = blk_columns(m, n, 32);
    T *Lw = (T *)(ws + Ly.lw), *RwT = (T *)(ws + Ly.rwt), *Ub = (T *)(ws + Ly.ub);
    T *tf = (T *)(ws + Ly.tf);   // T_j at tf + 1024 j, S_j at tf + 1024 (4 + j)
    int *ctr = (int *)(ws + Ly.ctr);
    const long ldr = Ly.ldr;
    hipError_t e = hipMemsetAsync(ctr, 0, (64 + kCW) * sizeof(int), s);
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
    bool x_patch = false;          // the previous X pass left U's top block for prep_qr to patch
    const double *sg_prev = sg0;   // s of the previous LQ panel (prep_qr's correction)
    // the prep kernels form the next panel QR's first Gram partials (no
    // k_cqr_gram launch) unless BRD_PREP_GRAM=0 (A/B)
    // (BRD_PREP_GRAM: bit 0 the QR side, bit 1 the LQ side; default both)
    const int foldm = getenv("BRD_PREP_GRAM") ? atoi(getenv("BRD_PREP_GRAM")) : 3;   // read per call (tests)
    const bool fold_qr = foldm & 1, fold_lq = foldm & 2;
    auto gram_into = [&](PrepArgs &p, bool on) {
        if (!on) return;
        double *cw = (double *)(ws + Ly.cws);
        p.gram = 1;
        p.gpp = (double *)(ws + Ly.gpp);   // records [wg][kGramRec]
        p.gout = cw;                    // CqrWs::gp1
        p.gew = cw + 3072 * kCW;        // CqrWs::ew
        p.gcnt = ctr + 64;
    };
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
                p.cc = c; p.zfill = 0;
                p.upatch = x_patch ? 1 : 0;
                gram_into(p, fold_qr);
                launch_k_prep<T>(false, prep_grid(p, lc), p, s);
                e = hipGetLastError();
                if (e != hipSuccess) return e;
                e = launch_cqr<T>((const T *)(ws + Ly.qp), 1, Ly.mp, mr, Lw + (size_t)c * 256 + 32 * j, 256, 1, nullptr, 0, 0, Tj,
                                  A + (size_t)c * lda + c, lda, 1, ws, Ly, err, s, false, fq, 1, nullptr, fold_qr);
            }
            if (e != hipSuccess) return e;
            // ---- Y pass (+ the QR panel's finish) + LQ of the row panel -------
            int ks_y = 1;
            bool yfold = false;
            e = launch_rpass<T>(true, A + (size_t)c * lda + c + 32, lda, mr, n2, Lw + (size_t)c * 256 + 32 * j, 256,
                                Lw + (size_t)c * 256, 256, ws, Ly, ctr + 16, err, s, lc, &ks_y, &fq,
                                Lw + (size_t)c * 256 + 32 * j, 257, sgq + 32 * j, nullptr, &yfold, 32 * j, 32 * j);
            if (e != hipSuccess) return e;
            {
                PrepArgs p;
                p.A = A; p.lda = lda; p.Lw = Lw; p.RwT = RwT; p.ldr = ldr;
                p.part = ws + Ly.part; p.mp = Ly.mp; p.ksplit = ks_y;
                p.G = ws + Ly.vout; p.Tm = Tj;
                p.Qp = ws + Ly.qp; p.mq = Ly.mp;
                p.c = c; p.j = j; p.items = n2; p.reduce = 0; p.factor = 0;
                p.sgn = sgq + 32 * j;
                p.cc = c + 32; p.zfill = 0;
                p.vpatch = yfold ? 1 : 0;
                gram_into(p, fold_lq);
                launch_k_prep<T>(true, prep_grid(p, lc), p, s);
                e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            const bool inl = j == NBMAX - 1;
            const FinArgs fl = fin_of(sgl + 32 * j, Sj, A + (size_t)c * lda + c + 32, 1, lda);
            e = launch_cqr<T>((const T *)(ws + Ly.qp), 1, Ly.mp, n2, RwT + (size_t)(128 + 32 * j) * ldr + c + 32, 1, ldr,
                              Ub + (size_t)(c + 32) * 32, 32, 1, Sj, A + (size_t)c * lda + c + 32, 1, lda, ws, Ly, err, s,
                              inl, fl, 1, nullptr, fold_lq);
            if (e != hipSuccess) return e;
            // ---- X pass (+ the LQ panel's finish) --------------------------------
            bool xfold = false;
            e = launch_rpass<T>(false, A + (size_t)(c + 32) * lda + c + 32, lda, n2, m - c - 32,
                                Ub + (size_t)(c + 32) * 32, 32, RwT + c + 32, ldr, ws, Ly, ctr + 16, err, s,
                                lc, &ks_x, inl ? nullptr : &fl,
                                inl ? nullptr : RwT + (size_t)(128 + 32 * j) * ldr + c + 32, ldr + 1, sgl + 32 * j,
                                nullptr, &xfold, 32 * (j + 1), 32 * j);   // prep_qr(j + 1) / the block end read these
            x_patch = !inl && xfold;   // prep_qr of the next panel patches U_j's top block
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
            p.cc = k1; p.zfill = 0;
            launch_k_prep<T>(false, prep_grid(p, lc), p, s);
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

// ==========================================================================
// The blocked path sharded over P GPUs (brd_dist.hip's
// layout: global column panel p on rank p mod P).  Lw = [V | X] (m x 256) is
// replicated, RwT = [Y | U] and Ub hold this rank's columns; the block update
// k_blkupd is local to each rank's columns.  Per panel j (global panel p,
// column c), five collectives:
//   QR   the owner of panel p forms the corrected column panel (k_prep_qr,
//        after every rank has added X_{j-1} to its Lw from the all-reduced
//        X partials) and runs its CholeskyQR; V' = Q (m - c rows), Q_t and
//        the zero flag are BROADCAST; every rank finishes the reconstruction
//        (modified LU, T_j, signs) beside its own Y pass, which is local:
//        Y_j = A^T V_j T_j needs only this rank's columns (svd_cuda_2.cu:1184,
//        qr_apply_cuda's column loop, sharded by columns).
//   LQ   every rank corrects its columns of the row panel (k_prep_lq) and
//        factors its rows of the panel's transpose by a SHARDED CholeskyQR
//        (lq_cuda, svd_cuda_2.cu:959, does the same QR on
//        one device): per pass a local 32 x 32 Gram (k_cqr_gram / k_cqr_q1 /
//        k_cqr_mid: the kernel's last workgroup sums its partials into this
//        rank's record), an ALL-GATHER of the P records (8 KB each), summed
//        in rank order by every rank -- the same R on every rank, bit for bit
//        -- and the local Q = P R^-1; three all-gathers per panel (G1, G2 and
//        sCQR3's middle Gram).  The rank holding panel p+1 (the band block's
//        columns: the panel's top block) finishes the basis-kernel
//        reconstruction inline (LU of Q_t - S, S_j, the band block), S_j
//        straight into its slot of the X all-reduce below (the other ranks
//        zero it, so the sum is S_j exactly; round 5 broadcast it on its
//        own).  U_j's rows stay where they were formed.
//   X    X_j = A U_j S_j sums over columns: each rank's split-K partials
//        (and its part of G = Rw^T U_j) are summed locally (k_dist_psum) and
//        ALL-REDUCED (m - c - 32 + 256 rows of 32, and S_j).
// Message sizes per panel: m x 32 (broadcast), 3 x P x 8 KB (all-gathers),
// (m + 256) x 32 + 1024 (all-reduce) -- against the
// per-panel path's m x b broadcast + P b^2 gather + b x m all-reduce, but 2.5
// passes over the trailing matrix per 32 columns instead of 4, the update on
// the matrix cores.  With one rank every collective is the identity and the
// path is the one-GPU blk_ge2band, launch for launch.
// ==========================================================================
namespace {
struct DistBlk {
    size_t bc, rec, ar, total;
};
DistBlk dist_blk_layout(int m, int n, int P, int rank, size_t elem) {
    const BlkLayout Ly = blk_layout(m, std::max(dist_local_cols(n, 32, P, rank), 1), elem);
    DistBlk D;
    size_t off = Ly.total;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    D.bc = take((size_t)m * 32 * elem + 1032 * sizeof(double));   // V' rows, then Q_t + zero flag
    D.rec = take((size_t)3 * P * kCqrRec * sizeof(double));       // the row panel QR's Gram records
    D.ar = take(((size_t)m * 32 + 256 * 32 + 1024) * elem);       // G (256 x 32), X rows, then S_j
    D.total = off;
    return D;
}
}  // namespace

size_t blk_dist_ws_bytes(int m, int n, int P, int rank, size_t elem) { return dist_blk_layout(m, n, P, rank, elem).total; }
bool blk_dist_fits(int n, int P) {
    return P >= 1 && P <= kBlkMaxRanks && dist_local_cols(n, 32, P, 0) <= kCW * kCT;   // rank 0 holds the most
}

#define BD_HIP(expr)                                                                          \
    do {                                                                                      \
        const hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                               \
            char m_[256];                                                                     \
            snprintf(m_, sizeof m_, "blocked distributed stage 1: %s (%s:%d)", hipGetErrorString(e_), \
                     __FILE__, __LINE__);                                                     \
            return api_fail(BRD_EHIP, m_);                                                    \
        }                                                                                     \
    } while (0)
#define BD_TRY(expr)             \
    do {                         \
        const int rc_ = (expr);  \
        if (rc_) return rc_;     \
    } while (0)

template <typename T>
int blk_ge2band_dist(T *A, int m, int n, long lda, Comm &C, void *wsv, hipStream_t s, int target, int *err) {
    const int P = C.nranks, me = C.rank;
    if (P == 1) {
        // one rank: every collective below is the identity and every rank-local
        // piece is the whole panel -- the one-GPU blocked path is this path
        // (its workspace is the head of this one's), launch for launch
        BD_HIP(blk_ge2band<T>(A, m, n, lda, wsv, s, target, err));
        return BRD_OK;
    }
    const int n_loc = dist_local_cols(n, 32, P, me);
    const int kend = blk_columns(m, n, 32);
    const S1Launch lc = s1_launch(m, n, target);
    char *ws = (char *)wsv;
    const BlkLayout Ly = blk_layout(m, std::max(n_loc, 1), sizeof(T));
    const DistBlk D = dist_blk_layout(m, n, P, me, sizeof(T));
    T *Lw = (T *)(ws + Ly.lw), *RwT = (T *)(ws + Ly.rwt), *Ub = (T *)(ws + Ly.ub);
    T *tf = (T *)(ws + Ly.tf);
    int *ctr = (int *)(ws + Ly.ctr);
    const long ldr = Ly.ldr;
    T *bc = (T *)(ws + D.bc), *ar = (T *)(ws + D.ar);
    double *rec = (double *)(ws + D.rec);
    const int dt = sizeof(T) == 8 ? BRD_DT_F64 : BRD_DT_F32;
    // every counter, the prep Gram groups' [64, 64 + kCW) included: the workspace
    // is shared with the per-panel tail and the band gather, and a nonzero
    // group counter would hold back the last-arriver's Gram sum
    BD_HIP(hipMemsetAsync(ctr, 0, (64 + kCW) * sizeof(int), s));
    double *sgq = (double *)(ws + Ly.sg), *sgl = sgq + NBMAX * 32, *sg0 = sgq + 2 * NBMAX * 32;
    BD_HIP(hipMemsetAsync(sg0, 0, 32 * sizeof(double), s));
    const double *cws = (const double *)(ws + Ly.cws);
    auto prep = [&](int c, int j, int items, int reduce, int factor, const void *part, long mp, int ks, const void *G,
                    const T *Tm, const double *sgn, long cc) {
        PrepArgs p;
        p.A = A; p.lda = lda; p.Lw = Lw; p.RwT = RwT; p.ldr = ldr;
        p.part = part; p.mp = mp; p.ksplit = ks; p.G = G; p.Tm = Tm;
        p.Qp = ws + Ly.qp; p.mq = Ly.mp;
        p.c = c; p.j = j; p.items = items; p.reduce = reduce; p.factor = factor;
        p.sgn = sgn; p.cc = cc; p.zfill = 0;
        return p;
    };
    // the panel QR's first Gram partials formed by the prep kernel that
    // writes the panel (no k_cqr_gram launch), as on one GPU (BRD_PREP_GRAM)
    const int foldm = getenv("BRD_PREP_GRAM") ? atoi(getenv("BRD_PREP_GRAM")) : 3;
    auto gram_into = [&](PrepArgs &pa) {
        double *cw = (double *)(ws + Ly.cws);
        pa.gram = 1;
        pa.gpp = (double *)(ws + Ly.gpp);
        pa.gout = cw;                    // CqrWs::gp1
        pa.gew = cw + 3072 * kCW;        // CqrWs::ew
        pa.gcnt = ctr + 64;
    };
    const T *s_prev = nullptr;   // S_{j-1}: the previous panel's all-reduced slot
    for (int k0 = 0; k0 < kend; k0 += NBMAX * 32) {
        for (int j = 0; j < NBMAX; ++j) {
            const int p = k0 / 32 + j, c = 32 * p, mr = m - c, mx = m - c - 32;
            const int o = p % P, o2 = (p + 1) % P;          // owners of panel p and of panel p + 1
            const bool own = me == o, own2 = me == o2;
            const long lco = (long)(p / P) * 32;            // panel p's column on its owner
            const long lcs = (long)dist_panels_before(p + 1, P, me) * 32;   // first local trailing column
            const int nc = n_loc - (int)lcs;                 // local trailing columns
            T *Tj = tf + 1024 * j, *Sj = tf + 1024 * (NBMAX + j);
            T *sj_ar = ar + (size_t)mx * 32 + 256 * 32;   // S_j's slot at the tail of the X all-reduce
            double *qt = (double *)((char *)bc + (size_t)mr * 32 * sizeof(T));   // Q_t, zero flag
            // ---- X_{j-1} (every rank) + the column panel's QR (its owner) ----------
            const bool fold_qr = own && j > 0 && (foldm & 1);
            if (j > 0) {
                PrepArgs pa = prep(c, j, mr, 1, own ? 1 : 0, ar + 256 * 32, 0, 1, ar, s_prev, sg0, lco);
                if (fold_qr) gram_into(pa);
                launch_k_prep<T>(false, prep_grid(pa, lc), pa, s);
                BD_HIP(hipGetLastError());
            }
            const FinArgs fq{qt, qt + 1024, sgq + 32 * j, Tj, own ? (void *)(A + (size_t)c * lda + lco) : nullptr, lda, 1};
            if (own) {
                const T *src = j == 0 ? A + (size_t)c * lda + lco : (const T *)(ws + Ly.qp);
                const long si = j == 0 ? lda : 1, st = j == 0 ? 1 : Ly.mp;
                BD_HIP(launch_cqr<T>(src, si, st, mr, Lw + (size_t)c * 256 + 32 * j, 256, 1, bc, 32, 1, Tj,
                                     A + (size_t)c * lda + lco, lda, 1, ws, Ly, err, s, false, fq, 1, qt, fold_qr));
            }
            {
                BD_TRY(C.bcast(bc, (size_t)mr * 32 * sizeof(T) + 1025 * sizeof(double), o, s));
                if (!own) launch_dist_unpack_v<T>(bc, Lw + (size_t)c * 256 + 32 * j, mr, s);
            }
            // ---- Y pass (local columns; every rank finishes the QR panel) -----------
            int ks_y = 1;
            BD_HIP(launch_rpass<T>(true, A + (size_t)c * lda + lcs, lda, mr, nc, Lw + (size_t)c * 256 + 32 * j, 256,
                                   Lw + (size_t)c * 256, 256, ws, Ly, ctr + 16, err, s, lc, &ks_y, &fq,
                                   Lw + (size_t)c * 256 + 32 * j, 257, sgq + 32 * j));
            // ---- the row panel: corrected locally, factored by a sharded CholeskyQR --
            {
                PrepArgs pa = prep(c, j, nc, 0, 0, ws + Ly.part, Ly.mp, ks_y, ws + Ly.vout, Tj, sgq + 32 * j, lcs);
                launch_k_prep<T>(true, prep_grid(pa, lc), pa, s);
                BD_HIP(hipGetLastError());
            }
            {
                CqrArgs a;
                a.src = ws + Ly.qp; a.si = 1; a.st = Ly.mp; a.M = std::max(nc, 0);
                a.vdst = RwT + (size_t)(128 + 32 * j) * ldr + lcs; a.vsi = 1; a.vst = ldr;
                a.vdst2 = Ub + (size_t)lcs * 32; a.vsi2 = 32; a.vst2 = 1;
                a.tout = Sj;
                a.apan = A + (size_t)c * lda + lcs; a.asi = 1; a.ast = lda;
                a.ws = (double *)(ws + Ly.cws);
                a.err = err;
                a.azero = 1;
                a.qcopy = nullptr;
                a.rec = rec; a.nrec = P; a.rme = me; a.rctr = ctr + 40;
                a.Mg = n - c - 32;
                a.goff = (long)((me - o2 + P) % P) * kCW * kCT;
                a.top = own2 ? 1 : 0;
                const int nwg = std::max(1, (a.M + kCT - 1) / kCT);
                // S_j straight into its slot of the X all-reduce (the other
                // ranks add exact zeros: the sum is S_j bit for bit), which
                // replaces a broadcast of its own
                const FinArgs fl{cws + cqr_ws_qt(), cws + cqr_ws_zero(), sgl + 32 * j, own2 ? sj_ar : Sj,
                                 own2 ? (void *)(A + (size_t)c * lda + lcs) : nullptr, 1, lda};
                if (!own2) BD_HIP(hipMemsetAsync(sj_ar, 0, 1024 * sizeof(T), s));
                const size_t rb = (size_t)kCqrRec * sizeof(double);
                launch_k_cqr<T>(kCqrGram, nwg, a, fl, s);   // -> record bank 0: this rank's G1, exponent
                BD_TRY(C.allgather(rec + (size_t)me * kCqrRec, rec, rb, s));
                launch_k_cqr<T>(kCqrQ1, nwg, a, fl, s);     // R1 (every rank, the same), Q1 rows -> bank 1
                BD_TRY(C.allgather(rec + (size_t)(P + me) * kCqrRec, rec + (size_t)P * kCqrRec, rb, s));
                launch_k_cqr<T>(kCqrMid, nwg, a, fl, s);    // sCQR3's middle pass (shifted panels) -> bank 2
                BD_TRY(C.allgather(rec + (size_t)(2 * P + me) * kCqrRec, rec + (size_t)2 * P * kCqrRec, rb, s));
                // V rows into RwT and Ub; the top block's owner finishes inline (LU, S_j, the band block)
                launch_k_cqr<T>(own2 ? kCqrVInline : kCqrV, nwg, a, fl, s);
                BD_HIP(hipGetLastError());
            }
            // ---- X pass (local columns), partials summed and all-reduced ------------
            if (nc > 0) {
                int ks_x = 1;
                BD_HIP(launch_rpass<T>(false, A + (size_t)(c + 32) * lda + lcs, lda, nc, mx, Ub + lcs * 32, 32,
                                       RwT + lcs, ldr, ws, Ly, ctr + 16, err, s, lc, &ks_x, nullptr, nullptr, 0,
                                       nullptr, ar));
                launch_dist_psum<T>((const T *)(ws + Ly.part), ks_x, Ly.mp, mx, ar + 256 * 32, s);
            } else {
                BD_HIP(hipMemsetAsync(ar, 0, ((size_t)mx * 32 + 256 * 32) * sizeof(T), s));
            }
            BD_TRY(C.allreduce_sum(ar, (size_t)mx * 32 + 256 * 32 + 1024, dt, s));
            s_prev = sj_ar;   // read by the next prep_qr / the block end, before the next X pass writes ar
        }
        // ---- block end: X_3 (every rank), the rank-256 update of my columns ---------
        const int k1 = k0 + NBMAX * 32;
        {
            PrepArgs pa = prep(k1, NBMAX, m - k1, 1, 0, ar + 256 * 32, 0, 1, ar, s_prev, sg0, 0);
            launch_k_prep<T>(false, prep_grid(pa, lc), pa, s);
            BD_HIP(hipGetLastError());
        }
        const long lck = (long)dist_panels_before(k1 / 32, P, me) * 32;
        const int cols = n_loc - (int)lck;
        if (cols > 0) {
            GemmArgs g;
            g.C = A + (size_t)k1 * lda + lck; g.ldc = lda;
            g.rows = m - k1; g.cols = cols;
            g.Lw = Lw + (size_t)k1 * 256; g.RwT = RwT + lck; g.ldr = ldr;
            g.K = 256;
            g.tiles_c = (g.cols + kGM - 1) / kGM;
            g.ntiles = ((g.rows + kGM - 1) / kGM) * g.tiles_c;
            const double el = (double)g.rows * g.cols;
            launch_k_blkupd<T>(dim3(g.ntiles), g, s, 2.0 * 256 * el, (2.0 * el + 256.0 * (g.rows + g.cols)) * sizeof(T));
            BD_HIP(hipGetLastError());
        }
    }
    return BRD_OK;
}
template int blk_ge2band_dist<double>(double *, int, int, long, Comm &, void *, hipStream_t, int, int *);
template int blk_ge2band_dist<float>(float *, int, int, long, Comm &, void *, hipStream_t, int, int *);

}  // namespace brd
