// Internal declarations shared by the stage-1 / stage-2 HIP translation units
// and the C-ABI layer (brd_api.cpp).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace brd {

// Largest logical tile (rows) held in LDS by one workgroup.  A Householder
// tree level groups consecutive rows into chunks of at most kRmax rows
// (leaf level) or stacks of at most kRmax/bk R-factors (inner levels).
constexpr int kRmax = 512;
// Widest panel (= band width b) the kernels support.
constexpr int kBmax = 32;

// One level of the Householder reduction tree of a panel with M logical rows
// and bk logical columns (see DESIGN.md "Stage 1").
struct TreeLevel {
    int level;      // 0 = leaves (chunks of consecutive rows)
    int groups;     // workgroups at this level
    int stride;     // leaves per child at this level (F^(level-1)); 1 for level 0
    int nchild;     // children of the previous level (level >= 1)
};

struct Tree {
    int M;          // logical rows of the panel
    int bk;         // logical columns (reflectors per leaf)
    int G0;         // leaf chunks
    int F;          // fan-in of inner levels = kRmax / bk
    int nlevels;
    TreeLevel lv[8];
};

Tree make_tree(int M, int bk);

// Device workspace layout of one tree: per level, per group: V (kRmax x 32),
// VT (32 x kRmax), T (32 x 32).
struct TreeWs {
    void *V[8];
    void *VT[8];
    void *T[8];
};
size_t tree_ws_bytes(const Tree &t, size_t elem);
void tree_ws_carve(const Tree &t, size_t elem, void *base, TreeWs &ws);

// Stage-1 launchers (brd_stage1.hip).  view base/ld: logical element (r,c) is
// base[r*ld + c] (trans = false) or base[c*ld + r] (trans = true).
template <typename T>
hipError_t launch_factor(bool trans, T *base, long ld, const Tree &t, int level,
                         const TreeWs &ws, hipStream_t s);
// target: workgroups to aim for (about one per CU).  fuse_panel / fuse_ld:
// the panel (factor view base, leading dimension; 0 = ld) whose level+1
// factor runs in the same launch (k_apply_factor), when the tree has that level.
template <typename T>
hipError_t launch_apply(bool trans, T *base, long ld, const Tree &t, int level,
                        int ncols, const TreeWs &ws, hipStream_t s, int target = 256,
                        T *fuse_panel = nullptr, long fuse_ld = 0);

// Blocked stage 1 (brd_stage1_blk.hip): panels of width 32 grouped in blocks
// of 4 with a delayed two-sided update.  blk_columns: columns [0, kend) the
// blocked path reduces (0 when it does not apply); the caller finishes the
// remaining panels with the per-panel path.  err: the stage-1 device error
// word (3: CholeskyQR breakdown -- a non-finite panel; rank deficiency is
// handled, cqr_shifted_pass).
size_t blk_ws_bytes(int m, int n, size_t elem);
int blk_columns(int m, int n, int b);
template <typename T>
hipError_t blk_ge2band(T *A, int m, int n, long lda, void *ws, hipStream_t s, int target, int *err);

// ---- multi-GPU (brd_dist.hip) -------------------------------------------------
// Collectives on device buffers, enqueued on (or drained from) stream s:
// RCCL over xGMI, or host callbacks (tests).  Return BRD_OK or a brd_status
// with brd_last_error set.
struct Comm {
    int rank = 0, nranks = 1;
    virtual ~Comm() {}
    virtual int bcast(void *buf, size_t bytes, int root, hipStream_t s) = 0;
    virtual int allgather(const void *send, void *recv, size_t bytes, hipStream_t s) = 0;
    virtual int allreduce_sum(void *buf, size_t count, int dtype, hipStream_t s) = 0;
};
// 1-D block-cyclic layout over column panels of width b: global panel p on
// rank p mod P.  Panels p' < g on rank r, and rank r's column count.
inline int dist_panels_before(int g, int P, int r) { return g > r ? (g - r + P - 1) / P : 0; }
inline int dist_local_cols(int n, int b, int P, int r) {
    const int np = (n + b - 1) / b;
    const int cnt = dist_panels_before(np, P, r);
    if (cnt == 0) return 0;
    const int last = (cnt - 1) * P + r;
    return (cnt - 1) * b + (n - last * b < b ? n - last * b : b);
}

// Blocked stage 1 sharded over the ranks of C (b = 32, fp64): columns [0,
// blk_columns(m, n, 32)) of the global matrix; A is this rank's m x n_loc
// shard.  ws: blk_dist_ws_bytes.  The caller finishes the remaining panels
// with the per-panel distributed loop.
size_t blk_dist_ws_bytes(int m, int n, int P, int rank, size_t elem);
// whether the blocked distributed form can run at all: its gathered row panel
// (P slots of dist_slot_rows rows) fits one panel QR (kCW kCT rows) and P fits
// the panel QR's per-block row counts
bool blk_dist_fits(int n, int P);
template <typename T>
int blk_ge2band_dist(T *A, int m, int n, long lda, Comm &C, void *ws, hipStream_t s, int target, int *err);

// Stage-2 launchers (brd_stage2.hip).
template <typename T>
hipError_t launch_band2bd(T *A, int n, long lda, int b, bool exact_order, bool sigma_geom, int *prog, int *err,
                          int nwaves, hipStream_t s);
template <typename T>
hipError_t launch_extract_bidiag(const T *A, int n, long lda, T *d, T *e, hipStream_t s);

// Bidiagonal singular values on the GPU (brd_bdsvd_dev.hip); ws >= 2n + 1 elements.
template <typename T>
hipError_t launch_bdsvd_dev(const T *d, const T *e, int n, T *sv, T *ws, hipStream_t s);

// ---- services of the C-ABI layer (brd_api.cpp) used by the distributed
// driver (brd_dist.hip) ------------------------------------------------------
int api_fail(int code, const char *msg);           // sets brd_last_error, returns code
hipStream_t api_stream();                          // the library stream
int api_apply_target();                            // workgroups per stage-1 apply launch
int api_device_cus();                              // CUs of the current device (whatever brd_set_overlap reserves)
int api_min_run(int level);                        // least slabs per apply workgroup at a tree level
bool api_overlap_active();                         // brd_set_overlap reservation in force
void *api_prof_begin(const char *kind, double flops, double bytes, hipStream_t s);
void api_prof_end(void *handle, hipStream_t s);
bool api_prof_launch_events(const char *kind, double flops, double bytes, hipEvent_t *a, hipEvent_t *b, int grid = 0);
// Profiling with kernel-bracketing events: a ProfScope in "launch" mode arms a
// pair of events that the NEXT stage-1 launch takes (hipExtLaunchKernel
// records them at the dispatch's start and end, the timestamps rocprofv3
// reports); false when nothing is armed.
bool api_take_launch_events(hipEvent_t *start, hipEvent_t *stop);
void api_lock();
void api_unlock();
// The current stream's stage-1 device error word (allocated on first use),
// and a synchronous read-and-clear of it (0: no error).
int *api_s1_err();
int api_take_s1_error(int *code);
const char *api_err_text(int code);
// Stage-1 panel helpers shared with the single-GPU loop.
long tree_level_rows(const Tree &t, int level);

}  // namespace brd
