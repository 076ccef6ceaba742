// C ABI of libbrd_hip.so (include/brd.h): argument checking, host<->device
// staging, workspace management, the stage-1 panel loop and the stage-2
// launch.  All GPU work is enqueued on one HIP stream.
#include "brd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "brd_internal.h"

namespace brd {

// --------------------------------------------------------------------------
// error reporting
// --------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// Device error word codes (sticky per launch stream; brd_check_errors).
static const char *err_word_text(int code) {
    switch (code) {
        case 1: return "stage-2 pipeline stalled (spin limit hit)";
        case 3: return "stage-1 CholeskyQR panel breakdown";
        default: return "device error";
    }
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(BRD_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),  \
                        __FILE__, __LINE__);                                              \
    } while (0)

// --------------------------------------------------------------------------
// reduction tree
// --------------------------------------------------------------------------
Tree make_tree(int M, int bk) {
    Tree t;
    t.M = M;
    t.bk = bk;
    t.G0 = std::max(1, (M + kRmax - 1) / kRmax);
    t.F = kRmax / std::max(bk, 1);
    t.nlevels = 1;
    t.lv[0] = {0, t.G0, 1, 0};
    int prev = t.G0, stride = 1;
    while (prev > 1) {
        const int l = t.nlevels;
        const int g = (prev + t.F - 1) / t.F;
        t.lv[l] = {l, g, stride, prev};
        stride *= t.F;
        prev = g;
        ++t.nlevels;
    }
    return t;
}

static size_t group_elems() { return (size_t)kRmax * 32 * 2 + 32 * 32; }

size_t tree_ws_bytes(const Tree &t, size_t elem) {
    size_t e = 0;
    for (int l = 0; l < t.nlevels; ++l) e += (size_t)t.lv[l].groups * group_elems();
    return e * elem;
}

void tree_ws_carve(const Tree &t, size_t elem, void *base, TreeWs &ws) {
    char *p = (char *)base;
    for (int l = 0; l < t.nlevels; ++l) {
        const size_t g = t.lv[l].groups;
        ws.V[l] = p;  p += g * kRmax * 32 * elem;
        ws.VT[l] = p; p += g * 32 * kRmax * elem;
        ws.T[l] = p;  p += g * 32 * 32 * elem;
    }
}

// --------------------------------------------------------------------------
// context: stream, workspace, profiling
// --------------------------------------------------------------------------
struct ProfAcc {
    long long launches = 0;
    double ms = 0, flops = 0, bytes = 0;
};
struct Pending {
    std::string kind;
    hipEvent_t a, b;
    double flops, bytes;
    int grid = 0;   // workgroups (0: unknown), for the launch timeline
};

struct Ctx {
    std::mutex mu;
    bool have_user_stream = false;   // true: use user_stream (NULL = legacy default stream)
    hipStream_t user_stream = nullptr;
    hipStream_t own_stream = nullptr;
    // Device workspaces per launch stream (stage-1 tree V/T, stage-2 progress
    // flags), so reductions on different streams can run at the same time.
    struct Slot {
        hipStream_t s = nullptr;
        void *ws = nullptr;
        size_t ws_bytes = 0;
        int *s2_flags = nullptr;     // stage-2 progress flags (n+1)
        int s2_cap = 0;
        // Stage-2 error word: written by the sweep kernel when a bounded spin
        // gives up, never reset by a launch (an asynchronous call's failure
        // stays visible until a synchronous call or brd_check_errors reads it).
        int *s2_err = nullptr;
        // Stage-1 error word (blocked path: 3 = CholeskyQR breakdown), kept
        // apart from stage 2's so a sync stage-1 call never consumes (and
        // misreports) a code an earlier asynchronous stage 2 left.
        int *s1_err = nullptr;
        void *stage = nullptr;       // host-pointer calls: cached HBM staging buffer
        size_t stage_bytes = 0;
    };
    std::deque<Slot> slots;      // deque: references stay valid as slots are added
    int *s2_err_host = nullptr;  // pinned copy of an error word
    int overlap_cus = 0;         // > 0: stage 2 on this many CUs, stage 1 sized for the rest
    bool prof = false;
    // BRD_PROF_TRACE=<file>: every profiled launch appended as "kind grid
    // start_ms end_ms bytes" relative to the event recorded at brd_profile_enable
    // (developer timeline of a stream: tools/cu_time.py --lib)
    FILE *trace = nullptr;
    hipEvent_t trace_ref = nullptr;
    // events armed for the next launch (ProfScope in launch mode)
    hipEvent_t ext_a = nullptr, ext_b = nullptr;
    bool ext_armed = false, ext_taken = false;
    std::map<std::string, ProfAcc> acc;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
};
static Ctx g_ctx;

static hipStream_t stream() {
    if (g_ctx.have_user_stream) return g_ctx.user_stream;
    if (!g_ctx.own_stream) hipStreamCreateWithFlags(&g_ctx.own_stream, hipStreamNonBlocking);
    return g_ctx.own_stream;
}

static Ctx::Slot &slot() {
    const hipStream_t s = stream();
    for (Ctx::Slot &x : g_ctx.slots)
        if (x.s == s) return x;
    g_ctx.slots.emplace_back();
    g_ctx.slots.back().s = s;
    return g_ctx.slots.back();
}

static int ensure_ws(size_t bytes, void **out) {
    Ctx::Slot &w = slot();
    *out = w.ws;
    if (bytes <= w.ws_bytes) return BRD_OK;
    if (w.ws) {
        hipStreamSynchronize(w.s);
        hipFree(w.ws);
        w.ws = nullptr;
        w.ws_bytes = 0;
    }
    if (hipMalloc(&w.ws, bytes) != hipSuccess)
        return fail(BRD_ENOMEM, "workspace allocation of %zu bytes failed", bytes);
    w.ws_bytes = bytes;
    *out = w.ws;
    return BRD_OK;
}

static int ensure_s2_flags(int n, int **out, int **err) {
    Ctx::Slot &w = slot();
    if (!g_ctx.s2_err_host && hipHostMalloc(&g_ctx.s2_err_host, sizeof(int)) != hipSuccess)
        return fail(BRD_ENOMEM, "pinned allocation failed");
    if (!w.s2_err) {
        if (hipMalloc(&w.s2_err, sizeof(int)) != hipSuccess) return fail(BRD_ENOMEM, "stage-2 error word allocation failed");
        if (hipMemsetAsync(w.s2_err, 0, sizeof(int), w.s) != hipSuccess) return fail(BRD_EHIP, "stage-2 error word reset failed");
    }
    *err = w.s2_err;
    *out = w.s2_flags;
    if (n + 2 <= w.s2_cap) return BRD_OK;
    if (w.s2_flags) {
        hipStreamSynchronize(w.s);
        hipFree(w.s2_flags);
        w.s2_flags = nullptr;
        w.s2_cap = 0;
    }
    if (hipMalloc(&w.s2_flags, sizeof(int) * (size_t)(n + 2)) != hipSuccess)
        return fail(BRD_ENOMEM, "stage-2 flag allocation failed");
    w.s2_cap = n + 2;
    *out = w.s2_flags;
    return BRD_OK;
}

static int ensure_s1_err(int **err) {
    Ctx::Slot &w = slot();
    if (!g_ctx.s2_err_host && hipHostMalloc(&g_ctx.s2_err_host, sizeof(int)) != hipSuccess)
        return fail(BRD_ENOMEM, "pinned allocation failed");
    if (!w.s1_err) {
        if (hipMalloc(&w.s1_err, sizeof(int)) != hipSuccess) return fail(BRD_ENOMEM, "stage-1 error word allocation failed");
        if (hipMemsetAsync(w.s1_err, 0, sizeof(int), w.s) != hipSuccess) return fail(BRD_EHIP, "stage-1 error word reset failed");
    }
    *err = w.s1_err;
    return BRD_OK;
}

// Reads (and clears) one of a slot's error words; the slot's stream is drained.
static int take_err_word(Ctx::Slot &w, int *word, int *code) {
    *code = 0;
    if (!word) return BRD_OK;
    HIP_TRY(hipMemcpyAsync(g_ctx.s2_err_host, word, sizeof(int), hipMemcpyDeviceToHost, w.s));
    HIP_TRY(hipStreamSynchronize(w.s));
    *code = *g_ctx.s2_err_host;
    if (*code) {
        HIP_TRY(hipMemsetAsync(word, 0, sizeof(int), w.s));
        HIP_TRY(hipStreamSynchronize(w.s));
    }
    return BRD_OK;
}
static int take_s2_error(Ctx::Slot &w, int *code) { return take_err_word(w, w.s2_err, code); }
static int take_s1_error(Ctx::Slot &w, int *code) { return take_err_word(w, w.s1_err, code); }

// HBM staging buffer of the host-pointer paths, cached per launch stream (no
// allocation per call, nothing to free on an error return).
static int ensure_stage(size_t bytes, void **out) {
    Ctx::Slot &w = slot();
    if (bytes > w.stage_bytes) {
        if (w.stage) {
            hipStreamSynchronize(w.s);
            hipFree(w.stage);
            w.stage = nullptr;
            w.stage_bytes = 0;
        }
        if (hipMalloc(&w.stage, bytes) != hipSuccess)
            return fail(BRD_ENOMEM, "device staging allocation of %zu bytes failed", bytes);
        w.stage_bytes = bytes;
    }
    *out = w.stage;
    return BRD_OK;
}

// Host-pointer calls stage the matrix in HBM.  The staging buffer is kept for
// the stream's lifetime (brd_release_stream frees it): freeing it after every
// call would make each call pay hipMalloc + hipFree, and hipFree synchronises
// the whole device (other streams' work included).  BRD_STAGE_KEEP_MB caps
// what is kept (a larger buffer is then freed when the call returns).
static void trim_stage(Ctx::Slot &w) {
    static const char *kenv = getenv("BRD_STAGE_KEEP_MB");
    if (!kenv) return;
    const size_t keep = (size_t)std::max(0, atoi(kenv)) << 20;
    if (w.stage && w.stage_bytes > keep) {
        hipStreamSynchronize(w.s);
        hipFree(w.stage);
        w.stage = nullptr;
        w.stage_bytes = 0;
    }
}

int api_device_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        cus = 256;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    }
    return cus;
}

// Workgroups a stage-1 apply launch is sized for: every CU, or the CUs that
// brd_set_overlap leaves to stage 1 (one workgroup per free CU, so no CU
// runs a second round of slabs while the others idle).
int api_apply_target() {
    const int ov = g_ctx.overlap_cus;
    static const char *tenv = getenv("BRD_S1_TARGET");   // tuning: workgroups per apply launch
    if (tenv && atoi(tenv) > 0) return atoi(tenv);
    return ov > 0 ? std::max(32, api_device_cus() - ov) : api_device_cus();
}

// Least slabs per apply workgroup at tree level `level`.  Beside other work
// (brd_set_overlap: a stream of reductions, CU time is what counts) an
// upper-level apply -- one node of stacked R rows, latency-bound, one slab
// per workgroup when the trailing matrix is narrow -- takes at least 8 slabs
// per workgroup so that each workgroup's V-fragment load is spread over more
// than one slab: N = 8192 fp64 stream 20.7-21.0 -> 21.4 TFLOP/s (floor 4:
// 21.4, 16: 21.3; a floor of 3 at level 0: no gain).  One reduction at a
// time (latency) the grid stays as wide as the target.
// BRD_S1_MINRUN0 / BRD_S1_MINRUN1 override (levels 0 / >= 1).
bool api_overlap_active() { return g_ctx.overlap_cus > 0; }

int api_min_run(int level) {
    static const char *mr0 = getenv("BRD_S1_MINRUN0"), *mr1 = getenv("BRD_S1_MINRUN1");
    const char *mr = level == 0 ? mr0 : mr1;
    if (mr) return std::max(1, atoi(mr));
    return (level > 0 && g_ctx.overlap_cus > 0) ? 8 : 1;
}

static int s2_waves() {
    if (g_ctx.overlap_cus > 0) return g_ctx.overlap_cus;
    static int nw = 0;
    if (!nw) {
        nw = api_device_cus();   // launch_band2bd clamps to the co-resident capacity
        // Bundles that can make progress at once are bounded by the chain
        // (~one bundle lifetime / one hand-off, < 64 at N <= 16384): a smaller
        // grid leaves CUs free for work on another stream (tuning override).
        static const char *genv = getenv("BRD_S2_GRID");
        if (genv && atoi(genv) > 0) nw = atoi(genv);
    }
    return nw;
}

static hipEvent_t get_event() {
    if (!g_ctx.event_pool.empty()) {
        hipEvent_t e = g_ctx.event_pool.back();
        g_ctx.event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

// Per-launch timing for brd_profile_*.  Default mode: events recorded on the
// launch stream before and after the launch (they also take in the dispatch
// gap).  Launch mode (the stage-1 apply, the roofline's kernel): the events
// are handed to the launch itself (api_take_launch_events ->
// hipExtLaunchKernel), which stamps the kernel's own start and end.
struct ProfScope {
    bool on, launch_mode;
    Pending p;
    hipStream_t s;
    ProfScope(const char *kind, double flops, double bytes, hipStream_t s_, bool launch = false)
        : on(g_ctx.prof), launch_mode(launch), s(s_) {
        if (!on) return;
        p.kind = kind;
        p.flops = flops;
        p.bytes = bytes;
        p.a = get_event();
        p.b = get_event();
        if (launch_mode) {
            g_ctx.ext_a = p.a;
            g_ctx.ext_b = p.b;
            g_ctx.ext_armed = true;
            g_ctx.ext_taken = false;
        } else {
            hipEventRecord(p.a, s);
        }
    }
    ~ProfScope() {
        if (!on) return;
        if (launch_mode) {
            const bool taken = g_ctx.ext_taken;
            g_ctx.ext_armed = g_ctx.ext_taken = false;
            if (!taken) {   // nothing was launched in the scope
                g_ctx.event_pool.push_back(p.a);
                g_ctx.event_pool.push_back(p.b);
                return;
            }
        } else {
            hipEventRecord(p.b, s);
        }
        g_ctx.pending.push_back(p);
    }
};

bool api_take_launch_events(hipEvent_t *start, hipEvent_t *stop) {
    if (!g_ctx.ext_armed || g_ctx.ext_taken) return false;
    *start = g_ctx.ext_a;
    *stop = g_ctx.ext_b;
    g_ctx.ext_taken = true;
    return true;
}

static void prof_drain() {
    for (auto &p : g_ctx.pending) {
        hipEventSynchronize(p.b);
        float ms = 0;
        hipEventElapsedTime(&ms, p.a, p.b);
        if (g_ctx.trace && g_ctx.trace_ref) {
            float t0 = 0, t1 = 0;
            hipEventElapsedTime(&t0, g_ctx.trace_ref, p.a);
            hipEventElapsedTime(&t1, g_ctx.trace_ref, p.b);
            fprintf(g_ctx.trace, "%s %d %.4f %.4f %.0f\n", p.kind.c_str(), p.grid, t0, t1, p.bytes);
        }
        ProfAcc &a = g_ctx.acc[p.kind];
        a.launches += 1;
        a.ms += ms;
        a.flops += p.flops;
        a.bytes += p.bytes;
        g_ctx.event_pool.push_back(p.a);
        g_ctx.event_pool.push_back(p.b);
    }
    g_ctx.pending.clear();
}

// Runs the stage-2 sweep on a device matrix.  A synchronous call checks (and
// clears) the slot's sticky spin-limit word; asynchronous calls leave it for
// the next synchronous call or brd_check_errors().
template <typename T>
static int band2bd_device(T *A, int n, long lda, int b, bool exact, bool sigma, bool sync, hipStream_t s) {
    int *prog = nullptr, *err = nullptr;
    int rc = ensure_s2_flags(n, &prog, &err);
    if (rc) return rc;
    {
        ProfScope ps("s2_sweep", 0, 0, s);
        HIP_TRY(launch_band2bd<T>(A, n, lda, b, exact, sigma, prog, err, s2_waves(), s));
    }
    if (sync) {
        int code = 0;
        rc = take_s2_error(slot(), &code);
        if (rc) return rc;
        if (code)
            return fail(BRD_EHIP, "%s (code %d) in this or an earlier asynchronous call on this stream",
                        err_word_text(code), code);
    }
    return BRD_OK;
}

// Rows of every group of a tree level, summed (= rows touched by one apply).
long tree_level_rows(const Tree &t, int level) {
    if (level == 0) return t.M;
    long r = 0;
    const int nprev = t.lv[level - 1].groups;
    for (int g = 0; g < t.lv[level].groups; ++g) r += (long)std::min(t.F, nprev - g * t.F) * t.bk;
    return r;
}

// --------------------------------------------------------------------------
// stage 1 panel loop on a device matrix
// --------------------------------------------------------------------------
// One side (QR of a column panel + left update, or LQ of a row panel + right
// update) of panel k.  The reduction tree's upper levels depend only on the
// leaves' R factors (panel columns) and the leaf-level apply only on the
// leaves' V, T (trailing columns), so each apply launch also runs the next
// level's factor (k_apply_factor): factor L0, then [apply L0 + factor L1],
// [apply L1 + factor L2], ... on one stream, with no event hand-offs.
template <typename T>
static int panel_side(bool trans, T *P, long lda, const Tree &t, const TreeWs &ws, T *X, int ncols,
                      hipStream_t s) {
    {
        ProfScope ps("s1_factor", 0, 0, s);
        HIP_TRY(launch_factor<T>(trans, P, lda, t, 0, ws, s));
    }
    static const char *ov = getenv("BRD_S1_OVERLAP");   // tuning: "0" = factors and applies as separate launches
    const bool fuse = ncols > 0 && !(ov && ov[0] == '0');
    if (!fuse) {
        for (int l = 1; l < t.nlevels; ++l) {
            ProfScope ps("s1_factor", 0, 0, s);
            HIP_TRY(launch_factor<T>(trans, P, lda, t, l, ws, s));
        }
    }
    if (ncols <= 0) return BRD_OK;
    for (int l = 0; l < t.nlevels; ++l) {
        const double rows = (double)tree_level_rows(t, l);
        ProfScope ps("s1_apply", 4.0 * t.bk * rows * ncols, 2.0 * rows * ncols * sizeof(T), s, true);
        HIP_TRY(launch_apply<T>(trans, X, lda, t, l, ncols, ws, s, api_apply_target(), fuse ? P : nullptr));
    }
    return BRD_OK;
}

// Blocked stage 1 (brd_stage1_blk.hip) for b = 32 -- the delayed two-sided
// update -- over all but the last panels: the default in both types.  Its
// panel QR computes in fp64 whatever the input type; the read passes and the
// block update run in the input type (fp32 N = 8192, one at a time: stage 1
// 55.2 ms blocked vs 60.0 per-panel; fp64 72.9 vs 86.3).
// BRD_S1_BLOCKED=1 / 0 forces either path (A/B and parity tests).
static bool blocked_enabled(size_t) {
    const char *env = getenv("BRD_S1_BLOCKED");   // read per call: tests switch it between calls
    if (env && env[0] == '0') return false;
    return true;
}

template <typename T>
static int ge2band_device(T *A, int m, int n, long lda, int b, hipStream_t s, bool *used_blocked = nullptr) {
    const bool blk_ok = blocked_enabled(sizeof(T)) && b == 32 && lda % 2 == 0 && ((uintptr_t)A % 16) == 0;
    const int kend = blk_ok ? blk_columns(m, n, b) : 0;
    size_t need = tree_ws_bytes(make_tree(m, std::min(b, n)), sizeof(T));
    need = std::max(need, tree_ws_bytes(make_tree(std::max(n - 1, 1), std::min(b, n)), sizeof(T)));
    if (kend > 0) need = std::max(need, blk_ws_bytes(m, n, sizeof(T)));
    void *wsbase = nullptr;
    int rc = ensure_ws(need, &wsbase);
    if (rc) return rc;
    if (used_blocked) *used_blocked = kend > 0;
    if (kend > 0) {
        int *err = nullptr;
        rc = ensure_s1_err(&err);
        if (rc) return rc;
        HIP_TRY(blk_ge2band<T>(A, m, n, lda, wsbase, s, api_apply_target(), err));
    }
    TreeWs ws;
    for (int k = kend; k < n; k += b) {
        const int bk = std::min(b, n - k);
        const int mp = m - k;
        const int n2 = n - k - bk;
        T *P = A + (long)k * lda + k;
        // QR of the column panel A[k:m, k:k+bk], left update of A[k:m, k+bk:n]
        const Tree tq = make_tree(mp, bk);
        tree_ws_carve(tq, sizeof(T), wsbase, ws);
        rc = panel_side<T>(false, P, lda, tq, ws, P + bk, n2, s);
        if (rc) return rc;
        if (n2 <= 0) continue;
        // LQ of the row panel A[k:k+bk, k+bk:n] (logical transpose), right
        // update of A[k+bk:m, k+bk:n]
        const Tree tl = make_tree(n2, bk);
        tree_ws_carve(tl, sizeof(T), wsbase, ws);
        T *Q = P + bk;
        rc = panel_side<T>(true, Q, lda, tl, ws, Q + (long)bk * lda, m - k - bk, s);
        if (rc) return rc;
    }
    return BRD_OK;
}

// --------------------------------------------------------------------------
// services for the distributed driver (brd_internal.h)
// --------------------------------------------------------------------------
int api_fail(int code, const char *msg) { return fail(code, "%s", msg); }
hipStream_t api_stream() { return stream(); }
void *api_prof_begin(const char *kind, double flops, double bytes, hipStream_t s) {
    if (!g_ctx.prof) return nullptr;
    Pending *p = new Pending{kind, get_event(), get_event(), flops, bytes};
    hipEventRecord(p->a, s);
    return p;
}
void api_prof_end(void *h, hipStream_t s) {
    if (!h) return;
    Pending *p = (Pending *)h;
    hipEventRecord(p->b, s);
    g_ctx.pending.push_back(*p);
    delete p;
}
// Launch-mode profiling for kernels launched outside a ProfScope (the blocked
// stage 1): two events the caller hands to hipExtLaunchKernel, queued for
// prof_drain.  False (no events) when profiling is off.
bool api_prof_launch_events(const char *kind, double flops, double bytes, hipEvent_t *a, hipEvent_t *b, int grid) {
    if (!g_ctx.prof) return false;
    Pending p{kind, get_event(), get_event(), flops, bytes, grid};
    *a = p.a;
    *b = p.b;
    g_ctx.pending.push_back(p);
    return true;
}
void api_lock() { g_ctx.mu.lock(); }
void api_unlock() { g_ctx.mu.unlock(); }
int *api_s1_err() {
    int *e = nullptr;
    return ensure_s1_err(&e) == BRD_OK ? e : nullptr;
}
int api_take_s1_error(int *code) { return take_s1_error(slot(), code); }
const char *api_err_text(int code) { return err_word_text(code); }

// --------------------------------------------------------------------------
// host/device staging shared by both stages
// --------------------------------------------------------------------------
static bool is_device_ptr(const void *p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

template <typename T>
static int ge2band(T *A, int m, int n, int lda, int b, int ngpus, unsigned flags) {
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    if (!A) return fail(BRD_EINVAL, "A is NULL");
    if (n < 1 || m < n) return fail(BRD_EINVAL, "need m >= n >= 1 (m=%d n=%d)", m, n);
    if (lda < n) return fail(BRD_EINVAL, "lda (%d) < n (%d)", lda, n);
    if (b < 1 || b > kBmax) return fail(BRD_EINVAL, "band width b=%d outside [1,%d]", b, kBmax);
    if (ngpus > 1) return fail(BRD_EUNSUPPORTED, "multi-GPU stage 1 goes through the distributed entry points");
    hipStream_t s = stream();
    const bool dev = (flags & BRD_DEVICE_PTR) != 0;
    if (dev && !is_device_ptr(A)) return fail(BRD_EINVAL, "BRD_DEVICE_PTR set but A is not device memory");
    int rc;
    bool blocked = false;
    if (dev) {
        rc = ge2band_device<T>(A, m, n, lda, b, s, &blocked);
        if (rc == BRD_OK && !(flags & BRD_ASYNC)) HIP_TRY(hipStreamSynchronize(s));
    } else {
        void *stage = nullptr;
        rc = ensure_stage(sizeof(T) * (size_t)m * n, &stage);
        if (rc) return rc;
        T *d = (T *)stage;
        HIP_TRY(hipMemcpy2DAsync(d, sizeof(T) * n, A, sizeof(T) * lda, sizeof(T) * n, m,
                                 hipMemcpyHostToDevice, s));
        rc = ge2band_device<T>(d, m, n, n, b, s, &blocked);
        if (rc == BRD_OK)
            HIP_TRY(hipMemcpy2DAsync(A, sizeof(T) * lda, d, sizeof(T) * n, sizeof(T) * n, m,
                                     hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        trim_stage(slot());
    }
    if (rc == BRD_OK) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(BRD_EHIP, "stage 1: %s", hipGetErrorString(e));
        if (blocked && (!dev || !(flags & BRD_ASYNC))) {
            int code = 0;
            rc = take_s1_error(slot(), &code);
            if (rc) return rc;
            if (code) return fail(BRD_EHIP, "stage 1: %s (code %d)", err_word_text(code), code);
        }
    }
    return rc;
}

template <typename T>
static int band2bd(T *A, int n, int lda, int b, T *dd, T *ee, unsigned flags) {
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    if (!A) return fail(BRD_EINVAL, "A is NULL");
    if (n < 1) return fail(BRD_EINVAL, "need n >= 1 (n=%d)", n);
    if (lda < n) return fail(BRD_EINVAL, "lda (%d) < n (%d)", lda, n);
    if (b < 1 || b > kBmax) return fail(BRD_EINVAL, "band width b=%d outside [1,%d]", b, kBmax);
    const bool extract = !(flags & BRD_NO_EXTRACT);
    if (extract && !dd) return fail(BRD_EINVAL, "d is NULL (pass BRD_NO_EXTRACT to skip d and e)");
    if (extract && !ee && n > 1) return fail(BRD_EINVAL, "e is NULL (pass BRD_NO_EXTRACT to skip d and e)");
    if (n == 1) {   // a 1 x 1 band is its own bidiagonal (the reference's sweep loop runs zero times)
        if (!extract) return BRD_OK;
        const hipMemcpyKind k = (flags & BRD_DEVICE_PTR) ? hipMemcpyDeviceToDevice : hipMemcpyHostToHost;
        HIP_TRY(hipMemcpyAsync(dd, A, sizeof(T), k, stream()));
        if (!(flags & BRD_ASYNC) || !(flags & BRD_DEVICE_PTR)) HIP_TRY(hipStreamSynchronize(stream()));
        return BRD_OK;
    }
    const bool exact = (flags & BRD_EXACT_ORDER) != 0;
    const bool sigma = (flags & BRD_SIGMA) != 0;
    hipStream_t s = stream();
    const bool dev = (flags & BRD_DEVICE_PTR) != 0;
    if (dev) {
        if (!is_device_ptr(A)) return fail(BRD_EINVAL, "BRD_DEVICE_PTR set but A is not device memory");
        int rc = band2bd_device<T>(A, n, lda, b, exact, sigma, !(flags & BRD_ASYNC), s);
        if (rc) return rc;
        if (extract) HIP_TRY(launch_extract_bidiag<T>(A, n, lda, dd, ee, s));
        if (!(flags & BRD_ASYNC)) HIP_TRY(hipStreamSynchronize(s));
    } else {
        void *stage = nullptr;
        int rc = ensure_stage(sizeof(T) * ((size_t)n * n + 2 * (size_t)n), &stage);
        if (rc) return rc;
        T *d = (T *)stage, *de = d + (size_t)n * n;
        HIP_TRY(hipMemcpy2DAsync(d, sizeof(T) * n, A, sizeof(T) * lda, sizeof(T) * n, n,
                                 hipMemcpyHostToDevice, s));
        rc = band2bd_device<T>(d, n, n, b, exact, sigma, true, s);
        if (rc) return rc;
        HIP_TRY(launch_extract_bidiag<T>(d, n, n, de, de + n, s));
        HIP_TRY(hipMemcpy2DAsync(A, sizeof(T) * lda, d, sizeof(T) * n, sizeof(T) * n, n,
                                 hipMemcpyDeviceToHost, s));
        if (extract) {
            HIP_TRY(hipMemcpyAsync(dd, de, sizeof(T) * n, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(ee, de + n, sizeof(T) * (n - 1), hipMemcpyDeviceToHost, s));
        }
        HIP_TRY(hipStreamSynchronize(s));
        trim_stage(slot());
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(BRD_EHIP, "stage 2: %s", hipGetErrorString(e));
    return BRD_OK;
}

// Bidiagonal singular values on the GPU (device pointers; brd_bdsvd_dev.hip).
// The workspace (2n + 1 elements: the squared Golub-Kahan off-diagonals, the
// scale and the bound) is the launch stream's cached staging buffer.
template <typename T>
static int bdsvd_dev(const T *d, const T *e, int n, T *sv, unsigned flags) {
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    if (n < 1) return fail(BRD_EINVAL, "need n >= 1 (n=%d)", n);
    if (!d || !sv || (n > 1 && !e)) return fail(BRD_EINVAL, "d, e (n > 1) and sv must be device pointers");
    if (!is_device_ptr(d) || !is_device_ptr(sv) || (n > 1 && !is_device_ptr(e)))
        return fail(BRD_EINVAL, "brd_bdsvd_dev: d, e and sv must be device memory");
    void *ws = nullptr;
    int rc = ensure_stage(sizeof(T) * (2 * (size_t)n + 1), &ws);
    if (rc) return rc;
    hipStream_t s = stream();
    HIP_TRY(launch_bdsvd_dev<T>(d, n > 1 ? e : d, n, sv, (T *)ws, s));
    if (!(flags & BRD_ASYNC)) HIP_TRY(hipStreamSynchronize(s));
    return BRD_OK;
}

}  // namespace brd

// ==========================================================================
// extern "C" entry points
// ==========================================================================
extern "C" {

int brd_ge2band_f64(double *A, int m, int n, int lda, int b, int ngpus, unsigned flags) {
    return brd::ge2band<double>(A, m, n, lda, b, ngpus, flags);
}
int brd_ge2band_f32(float *A, int m, int n, int lda, int b, int ngpus, unsigned flags) {
    return brd::ge2band<float>(A, m, n, lda, b, ngpus, flags);
}
int brd_band2bd_f64(double *A, int n, int lda, int b, double *d, double *e, unsigned flags) {
    return brd::band2bd<double>(A, n, lda, b, d, e, flags);
}
int brd_band2bd_f32(float *A, int n, int lda, int b, float *d, float *e, unsigned flags) {
    return brd::band2bd<float>(A, n, lda, b, d, e, flags);
}

int brd_bdsvd_dev_f64(const double *d, const double *e, int n, double *sv, unsigned flags) {
    return brd::bdsvd_dev<double>(d, e, n, sv, flags);
}
int brd_bdsvd_dev_f32(const float *d, const float *e, int n, float *sv, unsigned flags) {
    return brd::bdsvd_dev<float>(d, e, n, sv, flags);
}

int brd_set_stream(void *hip_stream) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    brd::g_ctx.user_stream = (hipStream_t)hip_stream;
    brd::g_ctx.have_user_stream = true;
    return BRD_OK;
}

int brd_set_overlap(int s2_cus) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    const int cus = brd::api_device_cus();
    if (s2_cus < 0 || s2_cus >= cus)
        return brd::fail(BRD_EINVAL, "brd_set_overlap: s2_cus=%d outside [0,%d) (device CUs)", s2_cus, cus);
    brd::g_ctx.overlap_cus = s2_cus;
    return BRD_OK;
}

int brd_check_errors(void) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    std::string bad;
    for (brd::Ctx::Slot &w : brd::g_ctx.slots) {
        for (int which = 0; which < 2; ++which) {
            int code = 0;
            const int rc = which ? brd::take_s1_error(w, &code) : brd::take_s2_error(w, &code);
            if (rc) return rc;
            if (code) bad += (bad.empty() ? "" : ", ") + std::to_string(code);
        }
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return brd::fail(BRD_EHIP, "HIP error: %s", hipGetErrorString(e));
    if (!bad.empty())
        return brd::fail(BRD_EHIP, "device error word set in an asynchronous call (1: stage-2 spin limit, "
                                    "3: stage-1 panel breakdown; codes %s)", bad.c_str());
    return BRD_OK;
}

int brd_release_stream(void *hip_stream) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    const hipStream_t s = hip_stream ? (hipStream_t)hip_stream : brd::stream();
    auto &slots = brd::g_ctx.slots;
    for (auto it = slots.begin(); it != slots.end(); ++it) {
        if (it->s != s) continue;
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return brd::fail(BRD_EHIP, "brd_release_stream: %s", hipGetErrorString(e));
        int code = 0;
        int h = 0;
        if (it->s2_err && hipMemcpy(&h, it->s2_err, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess) code = h;
        if (!code && it->s1_err && hipMemcpy(&h, it->s1_err, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess) code = h;
        if (it->ws) hipFree(it->ws);
        if (it->s2_flags) hipFree(it->s2_flags);
        if (it->s2_err) hipFree(it->s2_err);
        if (it->s1_err) hipFree(it->s1_err);
        if (it->stage) hipFree(it->stage);
        slots.erase(it);
        if (code)
            return brd::fail(BRD_EHIP, "brd_release_stream: the stream's device error word was set (code %d)", code);
        return BRD_OK;
    }
    return BRD_OK;   // the library never launched on it
}

int brd_use_own_stream(void) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    brd::g_ctx.have_user_stream = false;
    return BRD_OK;
}

int brd_profile_enable(int enable) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    brd::g_ctx.prof = enable != 0;
    const char *tp = getenv("BRD_PROF_TRACE");
    if (enable && tp && !brd::g_ctx.trace) {
        brd::g_ctx.trace = fopen(tp, "w");
        if (!brd::g_ctx.trace_ref) hipEventCreate(&brd::g_ctx.trace_ref);
        hipDeviceSynchronize();
        hipEventRecord(brd::g_ctx.trace_ref, nullptr);
    }
    if (!enable && brd::g_ctx.trace) {
        brd::prof_drain();
        fclose(brd::g_ctx.trace);
        brd::g_ctx.trace = nullptr;
    }
    return BRD_OK;
}

int brd_profile_reset(void) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    brd::prof_drain();
    brd::g_ctx.acc.clear();
    return BRD_OK;
}

int brd_profile_query(const char *kernel, long long *launches, double *total_ms, double *flops,
                      double *bytes) {
    std::lock_guard<std::mutex> lk(brd::g_ctx.mu);
    if (!kernel) return brd::fail(BRD_EINVAL, "kernel name is NULL");
    brd::prof_drain();
    auto it = brd::g_ctx.acc.find(kernel);
    brd::ProfAcc a;
    if (it != brd::g_ctx.acc.end()) a = it->second;
    if (launches) *launches = a.launches;
    if (total_ms) *total_ms = a.ms;
    if (flops) *flops = a.flops;
    if (bytes) *bytes = a.bytes;
    return BRD_OK;
}

const char *brd_last_error(void) { return brd::g_err.c_str(); }
int brd_version(void) { return 1; }

}  // extern "C"
