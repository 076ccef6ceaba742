/*
 * TEST INFRASTRUCTURE ONLY -- the CPU oracle for the two-stage bidiagonal
 * reduction.  Nothing in svdsolver_amd/ links or calls this; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / CPU baseline.
 *
 * Generic body, instantiated twice by brd_oracle.c with
 *   OT   = element type (float | double)
 *   OSFX = symbol suffix (f32 | f64)
 *
 * This is a restatement, in plain C on flat row-major arrays, of the
 * reference's CPU tiled algorithm (the algorithm that generated the
 * reference's data/band_* and data/bidiagonal_* fixtures).
 * Every arithmetic operation is performed in the same order and the same
 * precision as the reference's std::vector-of-rows code, so that compiled
 * without FMA contraction (-ffp-contract=off, no -march=native) the results
 * are bit-identical to the fixtures.  Each function cites the reference
 * code it restates.
 */

#define OCAT_(a, b) a##_##b
#define OCAT(a, b) OCAT_(a, b)
#define OFN(name) OCAT(name, OSFX)

/* ------------------------------------------------------------------------ */
/* Dense helpers.  mm() restates csc586::Matrix::mm (matrix.h:234-246):      */
/* result[i][j] starts at 0 and accumulates a[i][k]*b[k][j] for k = 0..q-1.  */
/* ------------------------------------------------------------------------ */
static void OFN(o_mm)(const OT *a, const OT *b, OT *c, int p, int q, int r)
{
    for (int i = 0; i < p; ++i)
        for (int j = 0; j < r; ++j) {
            OT acc = (OT)0;
            for (int k = 0; k < q; ++k)
                acc += a[i * q + k] * b[k * r + j];
            c[i * r + j] = acc;
        }
}

/* Householder reflector: restates csc586::serial::householder
 * (svd_serial.h:189-218).  x has length L; on return w (length L) and *tau.
 * Note the mixed precision of the reference: s = -copysign(1, x0) is a
 * double (integer first argument promotes to double), so u1, 1/u1 and tau
 * are formed in double and rounded to OT. */
static void OFN(o_householder)(const OT *x, int L, OT *w, OT *tau)
{
    double s = -copysign(1.0, (double)x[0]);
    OT acc = (OT)0;                        /* std::inner_product, matrix.h:64 */
    for (int r = 0; r < L; ++r)
        acc = acc + x[r] * x[r];
    OT norm_x = (OT)sqrt((double)acc);     /* std::sqrt: correctly rounded   */
    double u1 = (double)x[0] - s * (double)norm_x;
    OT alpha = (OT)(1. / u1);              /* w *= 1./u1 -> operator*=(T)    */
    for (int r = 0; r < L; ++r)
        w[r] = x[r] * alpha;
    w[0] = (OT)1.;
    *tau = (OT)(-s * u1 / (double)norm_x);
}

/* Explicit H = I - tau w w^T (svd_serial.h:205-214): H = (0 + w_i w_j)*(-tau),
 * then 1 + H_dd on the diagonal. */
static void OFN(o_hh_matrix)(const OT *w, OT tau, int L, OT *H)
{
    OT mt = -tau;
    for (int i = 0; i < L; ++i)
        for (int j = 0; j < L; ++j) {
            OT v = (OT)0 + w[i] * w[j];
            H[i * L + j] = v * mt;
        }
    for (int d = 0; d < L; ++d)
        H[d * L + d] = 1 + H[d * L + d];
}

/* ------------------------------------------------------------------------ */
/* Scratch: every buffer the tile kernels need, sized for tiles t <= TMAX    */
/* ------------------------------------------------------------------------ */
typedef struct {
    int cap;       /* max of (2t) */
    OT *R, *Y, *tmp, *tmp2, *Q1, *Q2, *x, *w, *y, *z, *z2, *X, *UT;
} OFN(o_scratch);

static void OFN(o_scratch_init)(OFN(o_scratch) *s, int t)
{
    int c = 2 * t;
    size_t sq = (size_t)c * c;
    s->cap = c;
    s->R = calloc(sq, sizeof(OT));   s->Y = calloc(sq, sizeof(OT));
    s->tmp = calloc(sq, sizeof(OT)); s->tmp2 = calloc(sq, sizeof(OT));
    s->Q1 = calloc(sq, sizeof(OT));  s->Q2 = calloc(sq, sizeof(OT));
    s->x = calloc(c, sizeof(OT));    s->w = calloc(c, sizeof(OT));
    s->y = calloc(c, sizeof(OT));    s->z = calloc(c, sizeof(OT));
    s->z2 = calloc(c, sizeof(OT));   s->X = calloc(sq, sizeof(OT));
    s->UT = calloc(sq, sizeof(OT));
}

static void OFN(o_scratch_free)(OFN(o_scratch) *s)
{
    free(s->R); free(s->Y); free(s->tmp); free(s->tmp2); free(s->Q1);
    free(s->Q2); free(s->x); free(s->w); free(s->y); free(s->z);
    free(s->z2); free(s->X); free(s->UT);
}

/* Compact WY T-factor column j: restates parallel::hholder_compact
 * (svd_parallel.h:97-114).  V is mv x nv (all rows used), S is t x t. */
static void OFN(o_hholder_compact)(OFN(o_scratch) *s, int j, OT tau, OT *S, int t,
                                   const OT *V, int mv, int nv)
{
    if (j == 0) {
        S[0] = -tau;
        return;
    }
    for (int a = 0; a < j; ++a) {          /* z = V_k^T v  */
        OT acc = (OT)0;
        for (int r = 0; r < mv; ++r)
            acc += V[r * nv + a] * V[r * nv + j];
        s->z[a] = acc;
    }
    for (int a = 0; a < j; ++a) {          /* z = S_k z    */
        OT acc = (OT)0;
        for (int c = 0; c < j; ++c)
            acc += S[a * t + c] * s->z[c];
        s->z2[a] = acc;
    }
    OT mt = -tau;
    for (int a = 0; a < j; ++a)
        S[a * t + j] = s->z2[a] * mt;
    S[j * t + j] = -tau;
}

/* Panel QR in compact form: restates parallel::qr (svd_parallel.h:133-179).
 * A is m x n (in place), S is n x n, V is m x n (persistent across calls). */
static void OFN(o_qr)(OFN(o_scratch) *s, OT *A, int m, int n, OT *S, OT *V)
{
    OT *Y = s->Y, *R = s->R, *VY = s->tmp;
    memset(Y, 0, sizeof(OT) * n * n);
    int jn = n < m ? n : m;
    for (int j = 0; j < jn; ++j) {
        OFN(o_mm)(V, Y, VY, m, n, n);                 /* R = A - V Y   */
        for (int i = 0; i < m * n; ++i)
            R[i] = A[i] - VY[i];
        int L = m - j;
        for (int r = 0; r < L; ++r)
            s->x[r] = R[(j + r) * n + j];
        OT tau;
        OFN(o_householder)(s->x, L, s->w, &tau);
        for (int c = 0; c < n - j; ++c) {             /* y = tau R^T w */
            OT acc = (OT)0;
            for (int r = 0; r < L; ++r)
                acc += R[(j + r) * n + (j + c)] * s->w[r];
            s->y[c] = acc * tau;
        }
        for (int r = 0; r < L; ++r)
            V[(j + r) * n + j] = s->w[r];
        for (int c = 0; c < n - j; ++c)
            Y[j * n + (j + c)] = s->y[c];
        OFN(o_hholder_compact)(s, j, tau, S, n, V, m, n);
    }
    OFN(o_mm)(V, Y, VY, m, n, n);                     /* A -= V Y      */
    for (int i = 0; i < m * n; ++i)
        A[i] = A[i] - VY[i];
}

/* Panel LQ in compact form: restates parallel::lq (svd_parallel.h:189-235).
 * A is m x n (in place), S is m x m, U is m x n (persistent across calls). */
static void OFN(o_lq)(OFN(o_scratch) *s, OT *A, int m, int n, OT *S, OT *U)
{
    OT *X = s->X, *L = s->R, *XU = s->tmp, *UT = s->UT;
    memset(X, 0, sizeof(OT) * m * m);
    int in = n < m ? n : m;
    for (int i = 0; i < in; ++i) {
        OFN(o_mm)(X, U, XU, m, m, n);                 /* L = A - X U   */
        for (int q = 0; q < m * n; ++q)
            L[q] = A[q] - XU[q];
        int Ln = n - i;
        for (int c = 0; c < Ln; ++c)
            s->x[c] = L[i * n + (i + c)];
        OT tau;
        OFN(o_householder)(s->x, Ln, s->w, &tau);
        for (int r = 0; r < m - i; ++r) {             /* x = tau L w   */
            OT acc = (OT)0;
            for (int c = 0; c < Ln; ++c)
                acc += L[(i + r) * n + (i + c)] * s->w[c];
            s->y[r] = acc * tau;
        }
        for (int r = 0; r < m - i; ++r)
            X[(i + r) * m + i] = s->y[r];
        for (int c = 0; c < Ln; ++c)
            U[i * n + (i + c)] = s->w[c];
        for (int r = 0; r < n; ++r)                   /* U_T = U^T     */
            for (int c = 0; c < m; ++c)
                UT[r * m + c] = U[c * n + r];
        OFN(o_hholder_compact)(s, i, tau, S, m, UT, n, m);
    }
    OFN(o_mm)(X, U, XU, m, m, n);                     /* A -= X U      */
    for (int q = 0; q < m * n; ++q)
        A[q] = A[q] - XU[q];
}

/* A <- A + (V S V^T)^T A : restates parallel::qr_apply (svd_parallel.h:243-255).
 * A is mv x na, V is mv x t, S is t x t. */
static void OFN(o_qr_apply)(OFN(o_scratch) *s, OT *A, int mv, int na,
                            const OT *S, const OT *V, int t)
{
    OT *Q1 = s->Q1, *Q2 = s->Q2, *tmp = s->tmp;
    for (int a = 0; a < t; ++a)                       /* Q1 = S V^T    */
        for (int r = 0; r < mv; ++r) {
            OT acc = (OT)0;
            for (int c = 0; c < t; ++c)
                acc += S[a * t + c] * V[r * t + c];
            Q1[a * mv + r] = acc;
        }
    OFN(o_mm)(V, Q1, Q2, mv, t, mv);                  /* Q2 = V Q1     */
    for (int q = 0; q < mv; ++q)                      /* tmp = Q2^T A  */
        for (int c = 0; c < na; ++c) {
            OT acc = (OT)0;
            for (int r = 0; r < mv; ++r)
                acc += Q2[r * mv + q] * A[r * na + c];
            tmp[q * na + c] = acc;
        }
    for (int i = 0; i < mv * na; ++i)
        A[i] = A[i] + tmp[i];
}

/* A <- A + A (V^T S V) : restates parallel::lq_apply (svd_parallel.h:271-282).
 * A is ma x nv, V is t x nv, S is t x t. */
static void OFN(o_lq_apply)(OFN(o_scratch) *s, OT *A, int ma, int nv,
                            const OT *S, const OT *V, int t)
{
    OT *P1 = s->Q1, *P2 = s->Q2, *tmp = s->tmp;
    OFN(o_mm)(S, V, P1, t, t, nv);                    /* P1 = S V      */
    for (int r = 0; r < nv; ++r)                      /* P2 = V^T P1   */
        for (int c = 0; c < nv; ++c) {
            OT acc = (OT)0;
            for (int a = 0; a < t; ++a)
                acc += V[a * nv + r] * P1[a * nv + c];
            P2[r * nv + c] = acc;
        }
    OFN(o_mm)(A, P2, tmp, ma, nv, nv);                /* tmp = A P2    */
    for (int i = 0; i < ma * nv; ++i)
        A[i] = A[i] + tmp[i];
}

/* ------------------------------------------------------------------------ */
/* Tile plumbing (matrix.h:406-428 get_tile / set_tile)                      */
/* ------------------------------------------------------------------------ */
static void OFN(o_get_tile)(const OT *A, int lda, int t, int ti, int tj, OT *dst, int ldd)
{
    for (int r = 0; r < t; ++r)
        memcpy(dst + (size_t)r * ldd, A + (size_t)(ti * t + r) * lda + (size_t)tj * t,
               sizeof(OT) * t);
}

static void OFN(o_set_tile)(OT *A, int lda, int t, int ti, int tj, const OT *src, int lds)
{
    for (int r = 0; r < t; ++r)
        memcpy(A + (size_t)(ti * t + r) * lda + (size_t)tj * t, src + (size_t)r * lds,
               sizeof(OT) * t);
}

/* Tile-kernel state carried between calls exactly as the reference's
 * brd_p1 locals (svd_parallel.h:416-434). */
typedef struct {
    int t;
    OT *S_kk, *V_kk, *S_ik, *V_ik, *S_ki, *V_ki, *S_kk1, *V_kk1, *R_kk, *R_kk1;
    OT *buf;  /* 2t*2t work tile */
} OFN(o_tiles);

/* factor_1tile (svd_parallel.h:296-308) for transform = qr (is_qr) or lq */
static void OFN(o_factor_1tile)(OFN(o_scratch) *s, int is_qr, OT *A, int lda, int t,
                                int i, int j, OT *R, OT *S, OT *V)
{
    OFN(o_get_tile)(A, lda, t, i, j, R, t);
    if (is_qr) OFN(o_qr)(s, R, t, t, S, V);
    else       OFN(o_lq)(s, R, t, t, S, V);
    OFN(o_set_tile)(A, lda, t, i, j, R, t);
}

/* factor_2tile (svd_parallel.h:311-340): concatenate the carried R with tile
 * (i2,j2) row-wise (QR) or column-wise (LQ), factor, split back. */
static void OFN(o_factor_2tile)(OFN(o_scratch) *s, int is_qr, OT *A, int lda, int t,
                                int i1, int j1, int i2, int j2, OT *R, OT *S, OT *V,
                                OT *buf)
{
    if (is_qr) {                              /* [R; A_i2j2]  (2t x t) */
        memcpy(buf, R, sizeof(OT) * t * t);
        OFN(o_get_tile)(A, lda, t, i2, j2, buf + t * t, t);
        OFN(o_qr)(s, buf, 2 * t, t, S, V);
        memcpy(R, buf, sizeof(OT) * t * t);
        OFN(o_set_tile)(A, lda, t, i1, j1, R, t);
        OFN(o_set_tile)(A, lda, t, i2, j2, buf + t * t, t);
    } else {                                  /* [R | A_i2j2] (t x 2t) */
        for (int r = 0; r < t; ++r)
            memcpy(buf + r * 2 * t, R + r * t, sizeof(OT) * t);
        OFN(o_get_tile)(A, lda, t, i2, j2, buf + t, 2 * t);
        OFN(o_lq)(s, buf, t, 2 * t, S, V);
        for (int r = 0; r < t; ++r)
            memcpy(R + r * t, buf + r * 2 * t, sizeof(OT) * t);
        OFN(o_set_tile)(A, lda, t, i1, j1, R, t);
        OFN(o_set_tile)(A, lda, t, i2, j2, buf + t, 2 * t);
    }
}

/* apply_1tile (svd_parallel.h:347-360) */
static void OFN(o_apply_1tile)(OFN(o_scratch) *s, int is_qr, OT *A, int lda, int t,
                               int i, int j, const OT *S, const OT *V, OT *buf)
{
    OFN(o_get_tile)(A, lda, t, i, j, buf, t);
    if (is_qr) OFN(o_qr_apply)(s, buf, t, t, S, V, t);
    else       OFN(o_lq_apply)(s, buf, t, t, S, V, t);
    OFN(o_set_tile)(A, lda, t, i, j, buf, t);
}

/* apply_2tile (svd_parallel.h:363-394) */
static void OFN(o_apply_2tile)(OFN(o_scratch) *s, int is_qr, OT *A, int lda, int t,
                               int i1, int j1, int i2, int j2, const OT *S, const OT *V,
                               OT *buf)
{
    if (is_qr) {
        OFN(o_get_tile)(A, lda, t, i1, j1, buf, t);
        OFN(o_get_tile)(A, lda, t, i2, j2, buf + t * t, t);
        OFN(o_qr_apply)(s, buf, 2 * t, t, S, V, t);
        OFN(o_set_tile)(A, lda, t, i2, j2, buf + t * t, t);
        OFN(o_set_tile)(A, lda, t, i1, j1, buf, t);
    } else {
        OFN(o_get_tile)(A, lda, t, i1, j1, buf, 2 * t);
        OFN(o_get_tile)(A, lda, t, i2, j2, buf + t, 2 * t);
        OFN(o_lq_apply)(s, buf, t, 2 * t, S, V, t);
        OFN(o_set_tile)(A, lda, t, i2, j2, buf + t, 2 * t);
        OFN(o_set_tile)(A, lda, t, i1, j1, buf, 2 * t);
    }
}

/* ------------------------------------------------------------------------ */
/* Stage 1: dense -> band.  Restates parallel::brd_p1 (svd_parallel.h:411-533)
 * in its serial order (the OpenMP loops run disjoint tiles; the result does
 * not depend on the thread count).  A is n x n row-major,
 * lda >= n, t | n.  Returns 0, or -1 on bad arguments.                      */
/* ------------------------------------------------------------------------ */
int OFN(oracle_brd_p1)(OT *A, int n, int lda, int t)
{
    if (t <= 0 || n <= 0 || n % t != 0 || lda < n)
        return -1;
    const int nbt = n / t;
    OFN(o_scratch) s;
    OFN(o_scratch_init)(&s, t);
    size_t tt = (size_t)t * t;
    OT *S_kk = calloc(tt, sizeof(OT)),  *V_kk = calloc(tt, sizeof(OT));
    OT *S_ik = calloc(tt, sizeof(OT)),  *V_ik = calloc(2 * tt, sizeof(OT));
    OT *S_ki = calloc(tt, sizeof(OT)),  *V_ki = calloc(2 * tt, sizeof(OT));
    OT *S_kk1 = calloc(tt, sizeof(OT)), *V_kk1 = calloc(tt, sizeof(OT));
    OT *R_kk = calloc(tt, sizeof(OT)),  *R_kk1 = calloc(tt, sizeof(OT));
    OT *buf = calloc(4 * tt, sizeof(OT));

    for (int k = 0; k < nbt; ++k) {
        /* QR step 1 */
        if (k == 0 || k == nbt - 1)
            OFN(o_factor_1tile)(&s, 1, A, lda, t, k, k, R_kk, S_kk, V_kk);
        /* QR step 2 */
        for (int j = k + 1; j < nbt; ++j) {
            OFN(o_apply_1tile)(&s, 1, A, lda, t, k, j, S_kk, V_kk, buf);
            if (j == k + 1)
                OFN(o_factor_2tile)(&s, 1, A, lda, t, k, k, j, k, R_kk, S_ik, V_ik, buf);
        }
        /* QR steps 3 + 4 */
        for (int i = k + 1; i < nbt; ++i) {
            if (i > k + 1)
                OFN(o_factor_2tile)(&s, 1, A, lda, t, k, k, i, k, R_kk, S_ik, V_ik, buf);
            for (int j = k + 1; j < nbt; ++j) {
                OFN(o_apply_2tile)(&s, 1, A, lda, t, k, j, i, j, S_ik, V_ik, buf);
                if (j == k + 1 && i == nbt - 1 && k < nbt - 1)
                    OFN(o_factor_1tile)(&s, 0, A, lda, t, k, k + 1, R_kk1, S_kk1, V_kk1);
            }
        }
        if (k < nbt - 1) {
            /* LQ step 2 */
            for (int j = k + 1; j < nbt; ++j) {
                OFN(o_apply_1tile)(&s, 0, A, lda, t, j, k + 1, S_kk1, V_kk1, buf);
                if (j == k + 1 && k + 2 < nbt)
                    OFN(o_factor_2tile)(&s, 0, A, lda, t, k, k + 1, k, k + 2, R_kk1, S_ki,
                                        V_ki, buf);
            }
            /* LQ steps 3 + 4 */
            for (int i = k + 2; i < nbt; ++i) {
                if (i > k + 2)
                    OFN(o_factor_2tile)(&s, 0, A, lda, t, k, k + 1, k, i, R_kk1, S_ki, V_ki,
                                        buf);
                for (int j = k + 1; j < nbt; ++j) {
                    OFN(o_apply_2tile)(&s, 0, A, lda, t, j, k + 1, j, i, S_ki, V_ki, buf);
                    if (j == k + 1 && i == nbt - 1)
                        OFN(o_factor_1tile)(&s, 1, A, lda, t, j, j, R_kk, S_kk, V_kk);
                }
            }
        }
    }
    free(S_kk); free(V_kk); free(S_ik); free(V_ik); free(S_ki); free(V_ki);
    free(S_kk1); free(V_kk1); free(R_kk); free(R_kk1); free(buf);
    OFN(o_scratch_free)(&s);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Stage 2: band -> bidiagonal, the reference's windowed sweep.              */
/* ------------------------------------------------------------------------ */

/* Right window (band_rd_right, svd_parallel.h:600-609; first half of
 * band_rd_top :569-580): reflector from the window's first row, A_t <- A_t H,
 * applied only inside rows [i1,i2) x cols [j1,j2). */
static int OFN(o_win_right)(OT *A, int lda, int i1, int i2, int j1, int j2,
                            OT *x, OT *w, OT *H, OT *tmp)
{
    int R = i2 - i1, L = j2 - j1;
    if (R <= 0 || L <= 0)
        return R <= 0 && L > 0 ? -2 : 0;  /* reference would read row 0 of an empty slice */
    for (int c = 0; c < L; ++c)
        x[c] = A[(size_t)i1 * lda + j1 + c];
    OT tau;
    OFN(o_householder)(x, L, w, &tau);
    OFN(o_hh_matrix)(w, tau, L, H);
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < L; ++c) {
            OT acc = (OT)0;
            const OT *row = A + (size_t)(i1 + r) * lda + j1;
            for (int k = 0; k < L; ++k)
                acc += row[k] * H[k * L + c];
            tmp[r * L + c] = acc;
        }
    for (int r = 0; r < R; ++r)
        memcpy(A + (size_t)(i1 + r) * lda + j1, tmp + r * L, sizeof(OT) * L);
    return 0;
}

/* Left window (band_rd_left, svd_parallel.h:617-626; second half of
 * band_rd_top :582-595): reflector from the window's first column,
 * A_t <- H A_t, inside the window only. */
static int OFN(o_win_left)(OT *A, int lda, int i1, int i2, int j1, int j2,
                           OT *x, OT *w, OT *H, OT *tmp)
{
    int R = i2 - i1, L = j2 - j1;
    if (R <= 0 || L <= 0)
        return L <= 0 ? 0 : -2;
    for (int r = 0; r < R; ++r)
        x[r] = A[(size_t)(i1 + r) * lda + j1];
    OT tau;
    OFN(o_householder)(x, R, w, &tau);
    OFN(o_hh_matrix)(w, tau, R, H);
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < L; ++c) {
            OT acc = (OT)0;
            for (int k = 0; k < R; ++k)
                acc += H[r * R + k] * A[(size_t)(i1 + k) * lda + j1 + c];
            tmp[r * L + c] = acc;
        }
    for (int r = 0; r < R; ++r)
        memcpy(A + (size_t)(i1 + r) * lda + j1, tmp + r * L, sizeof(OT) * L);
    return 0;
}

#ifndef O_IMIN_DEFINED
#define O_IMIN_DEFINED
static int o_imin(int a, int b) { return a < b ? a : b; }
#endif

/* Restates parallel::brd_p2 (svd_parallel.h:640-695): A is m x n row-major,
 * band width b (b super-diagonals).  In place; d (n) and e (n-1) receive the
 * diagonal and super-diagonal.  Returns 0, or -2 where the reference would
 * index an empty slice.
 *
 * sigma = 1: the sigma-preserving variant (not in the reference; SURVEY 8(f)
 * rank 1).  The reference's window count nbtx = floor((n - j2) / (b' - 1))
 * stops one window pair short of the matrix edge on most sweeps, so the last
 * bulge is dropped and the result is not orthogonally equivalent to the band.
 * With one more (clipped) pair per sweep, and empty windows skipped instead
 * of failing, every reflector's fill is chased off the matrix and the
 * bidiagonal has the band's singular values (tests/test_oracle.py checks
 * this against numpy's SVD). */
int OFN(oracle_brd_p2x)(OT *A, int m, int n, int lda, int b, OT *d, OT *e, int sigma)
{
    if (b < 1 || m < 1 || n < 2 || lda < n)
        return -1;
    const int bs = b + 1;                      /* b_size += 1  (:648)   */
    int cap = 2 * bs + 2;
    OT *x = calloc(cap, sizeof(OT)), *w = calloc(cap, sizeof(OT));
    OT *H = calloc((size_t)cap * cap, sizeof(OT));
    OT *tmp = calloc((size_t)cap * cap, sizeof(OT));
    int rc = 0;
    for (int i = 0; i < n - 1 && rc == 0; ++i) {
        /* Task 1: band_rd_top (:569-596) */
        int li1 = i, li2 = o_imin(i + bs, m), lj1 = i + 1, lj2 = o_imin(i + bs, n);
        rc = OFN(o_win_right)(A, lda, li1, li2, lj1, lj2, x, w, H, tmp);
        if (rc) break;
        lj2 = o_imin(i + bs + bs - 1, n);
        li1 = li1 + 1;
        lj1 = i + 1;
        rc = OFN(o_win_left)(A, lda, li1, li2, lj1, lj2, x, w, H, tmp);
        if (rc) break;
        /* nbtx = size_t(ceil((n - j2) / (b_size - 1))): integer division first (:664) */
        int nbtx = (n - lj2) / (bs - 1) + (sigma ? 1 : 0);
        for (int k = 0; k < nbtx + 1; ++k) {
            int end_i = o_imin(li2 + bs - 1, m);
            int start_j = o_imin(lj1 + bs - 1, n);
            int end_j3 = o_imin(lj2 + bs - 1, n);
            int ri1 = li1, ri2 = end_i, rj1 = start_j, rj2 = lj2;
            li1 = li2; li2 = end_i; lj1 = start_j; lj2 = end_j3;
            if (rj2 > rj1 && (!sigma || ri2 > ri1)) {   /* Task 2 */
                rc = OFN(o_win_right)(A, lda, ri1, ri2, rj1, rj2, x, w, H, tmp);
                if (rc) break;
            }
            if (lj2 > lj1 && (!sigma || li2 > li1)) {   /* Task 3 */
                rc = OFN(o_win_left)(A, lda, li1, li2, lj1, lj2, x, w, H, tmp);
                if (rc) break;
            }
        }
    }
    if (rc == 0) {
        if (d) for (int q = 0; q < n && q < m; ++q) d[q] = A[(size_t)q * lda + q];
        if (e) for (int q = 0; q < n - 1 && q < m; ++q) e[q] = A[(size_t)q * lda + q + 1];
    }
    free(x); free(w); free(H); free(tmp);
    return rc;
}

int OFN(oracle_brd_p2)(OT *A, int m, int n, int lda, int b, OT *d, OT *e)
{
    return OFN(oracle_brd_p2x)(A, m, n, lda, b, d, e, 0);
}

#undef OFN
#undef OCAT
#undef OCAT_
