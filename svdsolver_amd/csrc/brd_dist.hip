// Distributed stage 1 (dense -> band) over P GPUs, one process per GPU.
//
// Layout: 1-D block-cyclic over column panels of width b.  Global panel p
// (columns [pb, pb + b)) lives on rank p mod P as its local panel p / P; a
// rank's local matrix is m x n_loc, row-major, leading dimension lda_loc.
//
// Panel k (columns [kb, kb + bk)), owner o = k mod P:
//   1. o packs the panel (rows kb.., bk columns) and broadcasts it; every
//      rank factors it with the same Householder tree (identical inputs ->
//      identical V, T), o writes R back.
//   2. left update Q^T A on each rank's own trailing columns (no traffic).
//   3. LQ of the row panel (rows kb..kb+bk, trailing columns, spread over the
//      ranks): each rank runs the tree on its local columns (TSQR leaves),
//      the local b x b R factors are all-gathered and stacked starting with
//      rank (k+1) mod P (who owns the next panel), and every rank factors the
//      stack (the tree root) redundantly.
//   4. right update A Q: the local tree levels on each rank's columns; the
//      root mixes the stacked rows, i.e. the first b local trailing columns
//      of every rank: W = V_root^T X is summed over ranks (all-reduce, b x m2)
//      and each rank updates its own block.
// Traffic per panel: one broadcast of m x b, one all-gather of P b^2, one
// all-reduce of b x m.  The collectives go to RCCL (over xGMI) or, for tests
// and non-RCCL transports, to host callbacks (brd_dist_init_host).
//
// Replaces nothing in the reference (no multi-GPU path there);
// the math per panel is that of brd_api.cpp's single-GPU loop.
#include "brd.h"
#include "brd_internal.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace brd {

// ==========================================================================
// kernels
// ==========================================================================
// Local R of the row-panel tree, TR view (element (r, c) = A[c*ld + r]) ->
// row-major bk x bk, rows >= nrow zero.
template <typename T>
__global__ void k_get_R(T *__restrict__ R, const T *__restrict__ A, long ld, int bk, int nrow) {
    const int r = threadIdx.x, c = threadIdx.y;
    if (r < bk && c < bk) R[r * bk + c] = r < nrow ? A[(long)c * ld + r] : (T)0;
}
template <typename T>
__global__ void k_put_R(T *__restrict__ A, long ld, const T *__restrict__ R, int bk, int nrow) {
    const int r = threadIdx.x, c = threadIdx.y;
    if (r < nrow && c < bk) A[(long)c * ld + r] = R[r * bk + c];
}

// W[col][a] = sum_{r < nrow} Vb[r][a] X(r, col), X in the TR view (X(r, col) =
// X[col*ld + r]); Vb = this rank's rows of the root's V (row-major, 32 cols).
// 256 threads = 8 columns x 32.
template <typename T>
__global__ void __launch_bounds__(256) k_root_w(T *__restrict__ W, const T *__restrict__ X, long ld, int ncols,
                                                 const T *__restrict__ Vb, int nrow, int bk) {
    __shared__ T sV[32][33];
    __shared__ T sX[8][33];
    const int t32 = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int e = threadIdx.x; e < 32 * 32; e += 256) {
        const int r = e >> 5, a = e & 31;
        sV[r][a] = r < nrow ? Vb[r * 32 + a] : (T)0;
    }
    const int col = blockIdx.x * 8 + ty;
    sX[ty][t32] = (col < ncols && t32 < nrow) ? X[(long)col * ld + t32] : (T)0;
    __syncthreads();
    if (col < ncols) {
        T s = (T)0;
        for (int r = 0; r < nrow; ++r) s = fma(sV[r][t32], sX[ty][r], s);
        W[(long)col * 32 + t32] = t32 < bk ? s : (T)0;
    }
}

// X(r, col) += sum_a Vb[r][a] W2[a][col], W2 = -T^T W (the root's Q^T on this
// rank's block of stacked rows).
template <typename T>
__global__ void __launch_bounds__(256) k_root_upd(T *__restrict__ X, long ld, int ncols, const T *__restrict__ Vb,
                                                   const T *__restrict__ Tm, const T *__restrict__ W, int nrow,
                                                   int bk) {
    __shared__ T sV[32][33];
    __shared__ T sT[32][33];
    __shared__ T sW[8][33];
    __shared__ T sW2[8][33];
    const int t32 = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int e = threadIdx.x; e < 32 * 32; e += 256) {
        const int r = e >> 5, a = e & 31;
        sV[r][a] = r < nrow ? Vb[r * 32 + a] : (T)0;
        sT[r][a] = Tm[r * 32 + a];
    }
    const int col = blockIdx.x * 8 + ty;
    sW[ty][t32] = col < ncols ? W[(long)col * 32 + t32] : (T)0;
    __syncthreads();
    T w2 = (T)0;
    for (int b2 = 0; b2 < bk; ++b2) w2 = fma(-sT[b2][t32], sW[ty][b2], w2);
    sW2[ty][t32] = t32 < bk ? w2 : (T)0;
    __syncthreads();
    if (col < ncols && t32 < nrow) {
        T x = X[(long)col * ld + t32];
        for (int a = 0; a < bk; ++a) x = fma(sV[t32][a], sW2[ty][a], x);
        X[(long)col * ld + t32] = x;
    }
}

// Band blocks of this rank's panels: for local panel lp (global p = lp P + me)
// rows [pb - b, pb + b) x its b columns, zero outside the band / matrix.
template <typename T>
__global__ void k_pack_band(T *__restrict__ out, const T *__restrict__ A, long lda, int m, int n, int b, int P,
                            int me, int npl) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long per = 2L * b * b;
    if (e >= per * npl) return;
    const int lp = (int)(e / per), rem = (int)(e % per), rr = rem / b, cc = rem % b;
    const int p = lp * P + me;
    const int row = p * b - b + rr, col = p * b + cc;
    T v = (T)0;
    if (p * b < n && row >= 0 && row < m && col < n && col - row >= 0 && col - row <= b)
        v = A[(long)row * lda + lp * b + cc];
    out[e] = v;
}
template <typename T>
__global__ void k_unpack_band(T *__restrict__ B, long ldb, const T *__restrict__ all, int m, int n, int b, int P,
                              int npl) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long per = 2L * b * b;
    if (e >= per * npl * P) return;
    const int q = (int)(e / (per * npl));
    const long e2 = e % (per * npl);
    const int lp = (int)(e2 / per), rem = (int)(e2 % per), rr = rem / b, cc = rem % b;
    const int p = lp * P + q;
    const int row = p * b - b + rr, col = p * b + cc;
    if (p * b < n && row >= 0 && row < m && col < n && col - row >= 0 && col - row <= b)
        B[(long)row * ldb + col] = all[e];
}

namespace {

// ==========================================================================
// communicators
// ==========================================================================
int rccl_fail(ncclResult_t r, const char *what) {
    std::string m = std::string(what) + ": " + ncclGetErrorString(r);
    return api_fail(BRD_ERCCL, m.c_str());
}

struct RcclComm : Comm {
    ncclComm_t comm = nullptr;
    ~RcclComm() override {
        if (comm) ncclCommDestroy(comm);
    }
    int bcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        ncclResult_t r = ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm, s);
        return r == ncclSuccess ? BRD_OK : rccl_fail(r, "ncclBroadcast");
    }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        ncclResult_t r = ncclAllGather(send, recv, bytes, ncclUint8, comm, s);
        return r == ncclSuccess ? BRD_OK : rccl_fail(r, "ncclAllGather");
    }
    int allreduce_sum(void *buf, size_t count, int dtype, hipStream_t s) override {
        ncclResult_t r = ncclAllReduce(buf, buf, count, dtype == BRD_DT_F64 ? ncclFloat64 : ncclFloat32, ncclSum,
                                       comm, s);
        return r == ncclSuccess ? BRD_OK : rccl_fail(r, "ncclAllReduce");
    }
};

// Host-driven collectives: the library drains its stream, then the callback
// performs the collective on the device buffers and returns when it is done.
struct HostComm : Comm {
    brd_coll_fn fn = nullptr;
    void *user = nullptr;
    int call(int op, const void *send, void *recv, size_t count, int dtype, int root, hipStream_t s) {
        if (hipStreamSynchronize(s) != hipSuccess) return api_fail(BRD_EHIP, "stream sync before a collective");
        const int rc = fn(op, send, recv, count, dtype, root, user);
        return rc == 0 ? BRD_OK : api_fail(BRD_ERCCL, "host collective callback failed");
    }
    int bcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        return call(BRD_COLL_BCAST, buf, buf, bytes, BRD_DT_BYTE, root, s);
    }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        return call(BRD_COLL_ALLGATHER, send, recv, bytes, BRD_DT_BYTE, 0, s);
    }
    int allreduce_sum(void *buf, size_t count, int dtype, hipStream_t s) override {
        return call(BRD_COLL_ALLREDUCE_SUM, buf, buf, count, dtype, 0, s);
    }
};

// Communicators per launch stream.  brd_dist_init / brd_dist_init_host
// register the new communicator for the library's current stream; the first
// one is also the default for streams without a communicator of their own.
// Several streams with their own communicators (and workspaces) let several
// matrices' distributed panel loops run at once: the collectives of one
// communicator are issued in the same order on every rank, those of different
// communicators are independent.
struct CommReg {
    std::vector<std::pair<hipStream_t, std::unique_ptr<Comm>>> v;
    Comm *find(hipStream_t s) const {
        for (auto &e : v)
            if (e.first == s) return e.second.get();
        return v.empty() ? nullptr : v.front().second.get();
    }
    void add(hipStream_t s, std::unique_ptr<Comm> c) {
        for (auto &e : v)
            if (e.first == s) {
                e.second = std::move(c);
                return;
            }
        v.emplace_back(s, std::move(c));
    }
};
CommReg g_comms;

// ==========================================================================
// layout helpers
// ==========================================================================
int npanels(int n, int b) { return (n + b - 1) / b; }
int panels_before(int g, int P, int r) { return dist_panels_before(g, P, r); }
int local_cols(int n, int b, int P, int r) { return dist_local_cols(n, b, P, r); }

// ==========================================================================
// workspace
// ==========================================================================
struct DistWs {
    void *mem = nullptr;
    size_t bytes = 0;
    ~DistWs() {
        if (mem) hipFree(mem);
    }
    int ensure(size_t need, hipStream_t s) {
        if (need <= bytes) return BRD_OK;
        if (mem) {
            hipStreamSynchronize(s);
            hipFree(mem);
            mem = nullptr;
            bytes = 0;
        }
        if (hipMalloc(&mem, need) != hipSuccess) return api_fail(BRD_ENOMEM, "distributed workspace allocation failed");
        bytes = need;
        return BRD_OK;
    }
};
// distributed workspaces per launch stream (std::map: nodes stay put)
std::map<hipStream_t, DistWs> g_dws_by_stream;
DistWs &dist_ws(hipStream_t s) { return g_dws_by_stream[s]; }

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

#define D_HIP(expr)                                                                    \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            std::string m_ = std::string(#expr) + ": " + hipGetErrorString(e_);       \
            return api_fail(BRD_EHIP, m_.c_str());                                     \
        }                                                                              \
    } while (0)
#define D_TRY(expr)              \
    do {                         \
        const int rc_ = (expr);  \
        if (rc_) return rc_;     \
    } while (0)

template <typename T>
int dtype_of() { return sizeof(T) == 8 ? BRD_DT_F64 : BRD_DT_F32; }

// ==========================================================================
// the distributed panel loop
// ==========================================================================
// The blocked form (brd_stage1_blk.hip, blk_ge2band_dist) over the columns
// it covers: b = 32, fp64 (its panel QR computes in fp64 whatever the input,
// as on one GPU), unless BRD_S1_BLOCKED=0; BRD_DIST_BLOCKED=0 keeps the
// per-panel loop throughout (A/B).
template <typename T>
int dist_blocked_columns(int m, int n, int lda, int b, int P, const T *A) {
    const char *e1 = getenv("BRD_S1_BLOCKED"), *e2 = getenv("BRD_DIST_BLOCKED");
    if ((e1 && e1[0] == '0') || (e2 && e2[0] == '0')) return 0;
    if (sizeof(T) != 8 || b != 32 || lda % 2 != 0 || ((uintptr_t)A % 16) != 0) return 0;
    if (!blk_dist_fits(n, P)) return 0;   // the per-panel loop throughout
    return blk_columns(m, n, b);
}

template <typename T>
int ge2band_dist(T *A, int m, int n, int lda, int b, hipStream_t s) {
    Comm &C = *g_comms.find(s);
    DistWs &g_dws = dist_ws(s);
    const int P = C.nranks, me = C.rank;
    const int n_loc = local_cols(n, b, P, me);
    if (lda < std::max(n_loc, 1)) return api_fail(BRD_EINVAL, "lda_loc smaller than the local column count");
    if (P * b > kRmax) return api_fail(BRD_EUNSUPPORTED, "nranks * b must be <= 512 (one-level tree root)");
    const int kend = dist_blocked_columns<T>(m, n, lda, b, P, A);
    if (kend > 0) {
        int *err = api_s1_err();
        if (!err) return api_fail(BRD_ENOMEM, "stage-1 error word allocation failed");
        D_TRY(g_dws.ensure(blk_dist_ws_bytes(m, n, P, me, sizeof(T)), s));
        D_TRY(blk_ge2band_dist<T>(A, m, n, lda, C, g_dws.mem, s, api_apply_target(), err));
    }
    const size_t sz = sizeof(T);
    // workspace: QR / local-LQ tree, root tree, panel, local R, gathered R, stack, W
    const size_t ws_tree = std::max(tree_ws_bytes(make_tree(m, b), sz),
                                    tree_ws_bytes(make_tree(std::max(n_loc, 1), b), sz));
    const size_t ws_root = tree_ws_bytes(make_tree(P * b, b), sz);
    const size_t o_root = align_up(ws_tree), o_pan = o_root + align_up(ws_root);
    const size_t o_rloc = o_pan + align_up((size_t)m * b * sz);
    const size_t o_rall = o_rloc + align_up((size_t)b * b * sz);
    const size_t o_stk = o_rall + align_up((size_t)P * b * b * sz);
    const size_t o_w = o_stk + align_up((size_t)P * b * b * sz);
    const size_t total = o_w + align_up((size_t)32 * m * sz);
    D_TRY(g_dws.ensure(total, s));
    char *base = (char *)g_dws.mem;
    void *wsmain = base, *wsroot = base + o_root;
    T *Pbuf = (T *)(base + o_pan), *Rloc = (T *)(base + o_rloc), *Rall = (T *)(base + o_rall);
    T *Stk = (T *)(base + o_stk), *W = (T *)(base + o_w);

    TreeWs ws, wsr;
    const int np = npanels(n, b);
    for (int k = kend / b; k < np; ++k) {
        const int kb = k * b, bk = std::min(b, n - kb), mp = m - kb, n2 = n - kb - bk;
        const int owner = k % P;
        const int lc_k = (k / P) * b;                       // owner's local column of panel k
        const int lcs = panels_before(k + 1, P, me) * b;   // my first local trailing column
        const int nc = n_loc - lcs;                         // my local trailing columns
        // ---- 1. broadcast + redundant QR of the column panel
        if (me == owner)
            D_HIP(hipMemcpy2DAsync(Pbuf, bk * sz, A + (long)kb * lda + lc_k, lda * sz, bk * sz, mp,
                                   hipMemcpyDeviceToDevice, s));
        D_TRY(C.bcast(Pbuf, (size_t)mp * bk * sz, owner, s));
        const Tree tq = make_tree(mp, bk);
        tree_ws_carve(tq, sz, wsmain, ws);
        // with trailing columns here, the upper tree levels are factored inside
        // the apply launches (k_apply_factor), as in the one-GPU driver
        const bool fuse = n2 > 0 && nc > 0;
        for (int l = 0; l < (fuse ? 1 : tq.nlevels); ++l) {
            void *h = api_prof_begin("s1_factor", 0, 0, s);
            D_HIP(launch_factor<T>(false, Pbuf, bk, tq, l, ws, s));
            api_prof_end(h, s);
        }
        // ---- 2. left update of my trailing columns
        if (fuse) {
            for (int l = 0; l < tq.nlevels; ++l) {
                const double rows = (double)tree_level_rows(tq, l);
                void *h = api_prof_begin("s1_apply", 4.0 * bk * rows * nc, 2.0 * rows * nc * sz, s);
                D_HIP(launch_apply<T>(false, A + (long)kb * lda + lcs, lda, tq, l, nc, ws, s, api_apply_target(), Pbuf, bk));
                api_prof_end(h, s);
            }
        }
        if (me == owner)   // the factored panel (R, zeros below) back into my columns
            D_HIP(hipMemcpy2DAsync(A + (long)kb * lda + lc_k, lda * sz, Pbuf, bk * sz, bk * sz, mp,
                                   hipMemcpyDeviceToDevice, s));
        if (n2 <= 0) continue;
        // ---- 3. LQ of the row panel: local tree, gathered stacked R, root
        T *Q = A + (long)kb * lda + lcs;   // TR view: logical rows = my trailing columns
        Tree tl{};
        if (nc > 0) {
            tl = make_tree(nc, bk);
            tree_ws_carve(tl, sz, wsmain, ws);
            for (int l = 0; l < tl.nlevels; ++l) {
                void *h = api_prof_begin("s1_factor", 0, 0, s);
                D_HIP(launch_factor<T>(true, Q, lda, tl, l, ws, s));
                api_prof_end(h, s);
            }
        }
        const int nrow = std::min(std::max(nc, 0), bk);
        hipLaunchKernelGGL((k_get_R<T>), dim3(1), dim3(32, 32), 0, s, Rloc, Q, (long)lda, bk, nrow);
        D_TRY(C.allgather(Rloc, Rall, (size_t)bk * bk * sz, s));
        const int first = (k + 1) % P;   // the stack starts with the owner of panel k+1
        {   // rank q's block to position (q - first) mod P: a rotation, two copies
            const size_t bb = (size_t)bk * bk;
            D_HIP(hipMemcpyAsync(Stk, Rall + first * bb, (P - first) * bb * sz, hipMemcpyDeviceToDevice, s));
            if (first > 0)
                D_HIP(hipMemcpyAsync(Stk + (P - first) * bb, Rall, first * bb * sz, hipMemcpyDeviceToDevice, s));
        }
        const Tree tr = make_tree(P * bk, bk);
        tree_ws_carve(tr, sz, wsroot, wsr);
        {
            void *h = api_prof_begin("s1_factor", 0, 0, s);
            D_HIP(launch_factor<T>(false, Stk, bk, tr, 0, wsr, s));
            api_prof_end(h, s);
        }
        const int mypos = (me - first + P) % P;
        if (nrow > 0)
            hipLaunchKernelGGL((k_put_R<T>), dim3(1), dim3(32, 32), 0, s, Q, (long)lda,
                               Stk + (size_t)mypos * bk * bk, bk, nrow);
        // ---- 4. right update of rows kb+bk.. on my trailing columns
        const int m2 = m - kb - bk;
        if (m2 <= 0) continue;
        T *X = Q + (long)bk * lda;
        if (nc > 0) {
            for (int l = 0; l < tl.nlevels; ++l) {
                const double rows = (double)tree_level_rows(tl, l);
                void *h = api_prof_begin("s1_apply", 4.0 * bk * rows * m2, 2.0 * rows * m2 * sz, s);
                D_HIP(launch_apply<T>(true, X, lda, tl, l, m2, ws, s, api_apply_target()));
                api_prof_end(h, s);
            }
        }
        const T *Vb = (const T *)wsr.V[0] + (size_t)mypos * bk * 32;
        const T *Troot = (const T *)wsr.T[0];
        if (P > 1) {
            const dim3 grid((m2 + 7) / 8);
            if (nrow > 0)
                hipLaunchKernelGGL((k_root_w<T>), grid, dim3(256), 0, s, W, (const T *)X, (long)lda, m2, Vb, nrow, bk);
            else
                D_HIP(hipMemsetAsync(W, 0, (size_t)32 * m2 * sz, s));
            D_TRY(C.allreduce_sum(W, (size_t)32 * m2, dtype_of<T>(), s));
            if (nrow > 0)
                hipLaunchKernelGGL((k_root_upd<T>), grid, dim3(256), 0, s, X, (long)lda, m2, Vb, Troot,
                                   (const T *)W, nrow, bk);
        }
        // (P == 1: the root factors an upper-triangular R, its reflectors are
        //  the identity and the update is skipped.)
        D_HIP(hipGetLastError());
    }
    return BRD_OK;
}

template <typename T>
int gather_band(const T *A, int m, int n, int lda, int b, T *B, int ldb, int root, hipStream_t s) {
    Comm &C = *g_comms.find(s);
    DistWs &g_dws = dist_ws(s);
    const int P = C.nranks, me = C.rank;
    const int np = npanels(n, b), npl = (np + P - 1) / P;
    const size_t per = 2 * (size_t)b * b, sz = sizeof(T);
    const size_t o_all = align_up(per * npl * sz);
    D_TRY(g_dws.ensure(o_all + align_up(per * npl * P * sz), s));
    T *mine = (T *)g_dws.mem, *all = (T *)((char *)g_dws.mem + o_all);
    const long cnt = (long)per * npl;
    hipLaunchKernelGGL((k_pack_band<T>), dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, mine, A, (long)lda, m,
                       n, b, P, me, npl);
    D_TRY(C.allgather(mine, all, per * npl * sz, s));
    if (me == root) {
        D_HIP(hipMemset2DAsync(B, ldb * sz, 0, n * sz, m, s));
        const long tot = cnt * P;
        hipLaunchKernelGGL((k_unpack_band<T>), dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, B, (long)ldb,
                           (const T *)all, m, n, b, P, npl);
    }
    D_HIP(hipGetLastError());
    return BRD_OK;
}

struct Lock {
    Lock() { api_lock(); }
    ~Lock() { api_unlock(); }
};

template <typename T>
int ge2band_dist_entry(T *A, int m, int n, int lda, int b, unsigned flags) {
    Lock lk;
    hipStream_t s = api_stream();
    const Comm *c = g_comms.find(s);
    if (!c) return api_fail(BRD_EINVAL, "brd_dist_init / brd_dist_init_host has not been called");
    if (!A && local_cols(n, b, c->nranks, c->rank) > 0) return api_fail(BRD_EINVAL, "A_loc is NULL");
    if (n < 1 || m < n) return api_fail(BRD_EINVAL, "need m >= n >= 1");
    if (b < 1 || b > kBmax) return api_fail(BRD_EINVAL, "band width outside [1, 32]");
    if (!(flags & BRD_DEVICE_PTR)) return api_fail(BRD_EINVAL, "distributed stage 1 takes device pointers (BRD_DEVICE_PTR)");
    int rc = ge2band_dist<T>(A, m, n, lda, b, s);
    if (rc == BRD_OK && !(flags & BRD_ASYNC)) {
        D_HIP(hipStreamSynchronize(s));
        int code = 0;
        D_TRY(api_take_s1_error(&code));
        if (code) {
            std::string msg = std::string("distributed stage 1: ") + api_err_text(code);
            return api_fail(BRD_EHIP, msg.c_str());
        }
    }
    return rc;
}

template <typename T>
int gather_band_entry(const T *A, int m, int n, int lda, int b, T *B, int ldb, int root, unsigned flags) {
    Lock lk;
    hipStream_t s = api_stream();
    const Comm *c = g_comms.find(s);
    if (!c) return api_fail(BRD_EINVAL, "brd_dist_init / brd_dist_init_host has not been called");
    if (b < 1 || b > kBmax || n < 1 || m < n) return api_fail(BRD_EINVAL, "bad sizes");
    if (root < 0 || root >= c->nranks) return api_fail(BRD_EINVAL, "bad root rank");
    if (c->rank == root && (!B || ldb < n)) return api_fail(BRD_EINVAL, "root needs B with ldb >= n");
    int rc = gather_band<T>(A, m, n, lda, b, B, ldb, root, s);
    if (rc == BRD_OK && !(flags & BRD_ASYNC)) D_HIP(hipStreamSynchronize(s));
    return rc;
}

}  // namespace
}  // namespace brd

// ==========================================================================
// extern "C"
// ==========================================================================
extern "C" {

int brd_dist_unique_id(void *id_out, int id_bytes) {
    if (!id_out || id_bytes < (int)sizeof(ncclUniqueId)) return brd::api_fail(BRD_EINVAL, "id buffer too small (128 bytes)");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return brd::rccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof id);
    return BRD_OK;
}

int brd_dist_init(int rank, int nranks, const void *id, int id_bytes) {
    brd::Lock lk;
    if (!id || id_bytes < (int)sizeof(ncclUniqueId)) return brd::api_fail(BRD_EINVAL, "id buffer too small (128 bytes)");
    if (nranks < 1 || rank < 0 || rank >= nranks) return brd::api_fail(BRD_EINVAL, "bad rank / nranks");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    auto c = std::make_unique<brd::RcclComm>();
    // Several communicators run at once (one per launch stream: several
    // matrices in flight), each collective a kernel that waits for its peers
    // on the other GPUs.  Capped at a few blocks per collective, the kernels
    // of all communicators fit on the CUs together, so no GPU can fill up
    // with collectives whose peers are still queued behind it (the
    // multi-communicator hang); the per-panel messages are <= b x m elements,
    // latency-bound, so the cap costs little bandwidth.  BRD_RCCL_MAX_CTAS
    // overrides (0 = RCCL's default).
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    static const char *cenv = getenv("BRD_RCCL_MAX_CTAS");
    const int max_ctas = cenv ? atoi(cenv) : 8;
    if (max_ctas > 0) {
        cfg.minCTAs = 1;
        cfg.maxCTAs = max_ctas;
    }
    ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, uid, rank, &cfg);
    if (r != ncclSuccess) return brd::rccl_fail(r, "ncclCommInitRankConfig");
    c->rank = rank;
    c->nranks = nranks;
    brd::g_comms.add(brd::api_stream(), std::move(c));
    return BRD_OK;
}

int brd_dist_init_host(int rank, int nranks, brd_coll_fn fn, void *user) {
    brd::Lock lk;
    if (!fn) return brd::api_fail(BRD_EINVAL, "callback is NULL");
    if (nranks < 1 || rank < 0 || rank >= nranks) return brd::api_fail(BRD_EINVAL, "bad rank / nranks");
    auto c = std::make_unique<brd::HostComm>();
    c->fn = fn;
    c->user = user;
    c->rank = rank;
    c->nranks = nranks;
    brd::g_comms.add(brd::api_stream(), std::move(c));
    return BRD_OK;
}

int brd_dist_finalize(void) {
    brd::Lock lk;
    brd::g_comms.v.clear();
    brd::g_dws_by_stream.clear();
    return BRD_OK;
}

int brd_dist_local_cols(int n, int b, int nranks, int rank) {
    if (n < 1 || b < 1 || nranks < 1 || rank < 0 || rank >= nranks) return brd::api_fail(BRD_EINVAL, "bad layout arguments");
    return brd::local_cols(n, b, nranks, rank);
}

int brd_ge2band_dist_f64(double *A_loc, int m, int n, int lda_loc, int b, unsigned flags) {
    return brd::ge2band_dist_entry<double>(A_loc, m, n, lda_loc, b, flags);
}
int brd_ge2band_dist_f32(float *A_loc, int m, int n, int lda_loc, int b, unsigned flags) {
    return brd::ge2band_dist_entry<float>(A_loc, m, n, lda_loc, b, flags);
}
int brd_dist_gather_band_f64(const double *A_loc, int m, int n, int lda_loc, int b, double *B, int ldb, int root,
                             unsigned flags) {
    return brd::gather_band_entry<double>(A_loc, m, n, lda_loc, b, B, ldb, root, flags);
}
int brd_dist_gather_band_f32(const float *A_loc, int m, int n, int lda_loc, int b, float *B, int ldb, int root,
                             unsigned flags) {
    return brd::gather_band_entry<float>(A_loc, m, n, lda_loc, b, B, ldb, root, flags);
}

}  // extern "C"
