// Stage 2 (band -> bidiagonal) kernels for gfx950.
//
// Replaces csc586::parallel::brd_p2 (reference svd_parallel.h:640-695) and its
// window kernels band_rd_top (:569), band_rd_right (:600), band_rd_left (:617).
// The window geometry is the reference's ("compat" semantics):
// every Householder is formed from a window's first row (right windows) or
// first column (left windows) and applied only inside that window, with the
// reference's b_size += 1 and floor-then-ceil window count.
//
// One wave executes one window: a right window (<= 2b rows x b cols) holds one
// row per lane, a left window (<= b rows x 2b cols) one column per lane, so the
// reflector's application is a per-lane dot product + axpy and the reflector
// itself comes from one LDS broadcast.  Two arithmetic modes:
//   fast         w^T x / rank-1 update with FMAs (the production path);
//   exact order  the reference's explicit H = I - tau w w^T and naive product
//                in its operation order with fp contraction off -- the output
//                is bit-identical to the reference's CPU code on the same
//                input (used to pin the geometry in tests).
//
// Three kernels (DESIGN.md "Stage 2"):
//   k_sweeps          fast mode, b = 32 (production): bundles of S sweeps per
//                     workgroup on an LDS ring, one straight-line wave per
//                     window (brd_s2win.h), loader / writer / poller waves.
//   k_band2bd_bundle  exact order, and fast mode for b != 32: the same bundle
//                     scheme with the generic (predicated) one-wave windows.
//   k_band2bd_pipe    bands too small for a ring (n < 64): one wave per sweep
//                     straight on HBM (sc1 hand-offs).
#include "brd_internal.h"

#include <algorithm>
#include <cstdlib>

namespace brd {

template <typename T>
__device__ __forceinline__ T ld_c(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_c(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void wave_sync2() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Reflector of csc586::serial::householder (svd_serial.h:189-218), including
// its mixed precision (s, u1 and tau are doubles, rounded to T).
template <typename T>
struct Refl {
    T alpha;   // 1/u1 rounded to T (the scale applied to x)
    T tau;
};

// Reflector of the vector held in the calling lane's registers (lane 0 holds
// the window's first row / column), computed in the reference's operation order
// in exact mode (fp contraction off).
template <typename T, bool EXACT>
__device__ __forceinline__ Refl<T> refl_regs(const T (&x)[32], int L) {
    T acc = (T)0;
    double s;
    T nrm;
    if constexpr (EXACT) {
#pragma clang fp contract(off)
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (r < L) acc = acc + x[r] * x[r];
        nrm = (T)sqrt((double)acc);
        s = -copysign(1.0, (double)x[0]);
    } else {
        T acc1 = (T)0;   // two chains: fast mode does not keep the serial order
#pragma unroll
        for (int r = 0; r < 32; r += 2) {
            if (r < L) acc = fma(x[r], x[r], acc);
            if (r + 1 < L) acc1 = fma(x[r + 1], x[r + 1], acc1);
        }
        nrm = sqrt(acc + acc1);
        s = x[0] >= (T)0 ? -1.0 : 1.0;   // -copysign(1, x0) (x0 = -0 -> treated as +0)
    }
    const double u1 = (double)x[0] - s * (double)nrm;
    Refl<T> h;
    h.alpha = (T)(1. / u1);
    h.tau = (T)(-s * u1 / (double)nrm);
    return h;
}

// Per-wave LDS scratch.  Fast mode needs only the broadcast reflector w and
// tau; exact mode also holds x, the explicit H (<= 32 x 32) and the lane's
// row/column.
template <typename T, bool EXACT>
struct WaveLds {
    T w[64];
    T h[2];
};
template <typename T>
struct WaveLds<T, true> {
    T w[64];          // reflector (w[0] = 1)
    T h[2];           // alpha, tau
    T x[64];          // reflector source vector
    T H[32 * 33];     // explicit H
    T buf[64 * 33];   // the lane's row / column (dynamic indexing)
};

// Element accessors: the band in HBM (agent-coherent sc1 accesses) or a ring
// of band rows in LDS.  row(r) returns a pointer p with p[c] = element (r, c).
template <typename T>
struct HbmAcc {
    T *A;
    long lda;
    __device__ __forceinline__ T *row(int r) const { return A + (long)r * lda; }
    __device__ __forceinline__ T ld(const T *p) const { return ld_c(p); }
    __device__ __forceinline__ void st(T *p, T v) const { st_c(p, v); }
};
// r mod R without an integer division: with magic = ceil(2^32 / R),
// umulhi(r, magic) = floor(r / R) exactly for 0 <= r < 2^32 / R (the rounding
// excess r * (magic - 2^32/R) / 2^32 stays below 1/R); the compare is a guard.
__device__ __forceinline__ int fast_mod(int r, int R, unsigned magic) {
    int s = r - (int)__umulhi((unsigned)r, magic) * R;
    return s >= R ? s - R : s;
}

template <typename T>
struct RingAcc {
    T *d;            // ring rows * P elements
    int P;           // row pitch ring_pitch(b) >= 3b - 1 (diagonals -(b-1) .. 2b-1)
    int R;           // ring rows
    int off;         // b - 1
    unsigned magic;  // ceil(2^32 / R)
    __device__ __forceinline__ int slot(int r) const { return fast_mod(r, R, magic); }
    __device__ __forceinline__ T *row(int r) const { return d + slot(r) * P + off - r; }
    __device__ __forceinline__ T ld(const T *p) const { return *p; }
    __device__ __forceinline__ void st(T *p, T v) const { *p = v; }
};

// Apply the reflector of lane 0's vector to every lane's vector a[0..L) (a
// right window's row or a left window's column).  Lane 0 forms the reflector
// from its registers and broadcasts w (and tau) through LDS once.
template <typename T, bool EXACT>
__device__ __forceinline__ void refl_apply(T (&a)[32], int L, WaveLds<T, EXACT> &S, int lane, bool row_major)
{
    if constexpr (!EXACT) {
        if (lane == 0) {
            const Refl<T> h = refl_regs<T, false>(a, L);
            S.h[1] = h.tau;
#pragma unroll
            for (int c = 1; c < 32; ++c)
                if (c < L) S.w[c] = a[c] * h.alpha;   // w_0 = 1, w_c = x_c * alpha
        }
        wave_sync2();
        const T tau = S.h[1];
        T w[32];
#pragma unroll
        for (int c = 1; c < 32; ++c) w[c] = c < L ? S.w[c] : (T)0;
        T d0 = a[0], d1 = (T)0, d2 = (T)0, d3 = (T)0;
#pragma unroll
        for (int c = 1; c < 32; c += 4) {
            d1 = fma(a[c], w[c], d1);
            if (c + 1 < 32) d2 = fma(a[c + 1], w[c + 1], d2);
            if (c + 2 < 32) d3 = fma(a[c + 2], w[c + 2], d3);
            if (c + 3 < 32) d0 = fma(a[c + 3], w[c + 3], d0);
        }
        const T td = tau * ((d0 + d1) + (d2 + d3));
        a[0] -= td;
#pragma unroll
        for (int c = 1; c < 32; ++c)
            if (c < L) a[c] = fma(-td, w[c], a[c]);
    } else {
#pragma clang fp contract(off)
        if (lane == 0) {
            const Refl<T> h = refl_regs<T, true>(a, L);
            S.h[0] = h.alpha;
            S.h[1] = h.tau;
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (c < L) S.x[c] = a[c];
        }
        wave_sync2();
        const Refl<T> h{S.h[0], S.h[1]};
        // w and explicit H (svd_serial.h:203-214)
        for (int c = lane; c < L; c += 64) S.w[c] = (c == 0) ? (T)1. : S.x[c] * h.alpha;
        wave_sync2();
        const T mt = -h.tau;
        for (int e = lane; e < L * L; e += 64) {
            const int k = e / L, c = e - k * L;
            T v = ((T)0 + S.w[k] * S.w[c]) * mt;
            if (k == c) v = 1 + v;
            S.H[k * 33 + c] = v;
        }
        T *my = S.buf + lane * 33;
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (c < L) my[c] = a[c];
        wave_sync2();
        // right window: A_t <- A_t H, out[c] = sum_k a[k] H[k][c]  (matrix.h:234 order)
        // left window:  A_t <- H A_t, out[r] = sum_k H[r][k] a[k]
        for (int c = 0; c < L; ++c) {
            T acc = (T)0;
            if (row_major)
                for (int k = 0; k < L; ++k) acc += my[k] * S.H[k * 33 + c];
            else
                for (int k = 0; k < L; ++k) acc += S.H[c * 33 + k] * my[k];
#pragma unroll
            for (int cc = 0; cc < 32; ++cc)
                if (cc == c) a[cc] = acc;
        }
    }
}

// ---- right window: rows [i1,i2) x cols [j1,j2); reflector from row i1 ------
template <typename T, bool EXACT, typename Acc>
__device__ void win_right(const Acc &A, int i1, int i2, int j1, int j2, WaveLds<T, EXACT> &S, int lane)
{
    const int R = i2 - i1, L = j2 - j1;   // R <= 64, L <= 32
    T *rowp = A.row(i1 + (lane < R ? lane : 0)) + j1;
    T a[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) a[c] = (lane < R && c < L) ? A.ld(rowp + c) : (T)0;
    refl_apply<T, EXACT>(a, L, S, lane, true);
    if (lane < R) {
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (c < L) A.st(rowp + c, a[c]);
    }
}

// ---- left window: rows [i1,i2) x cols [j1,j2); reflector from column j1 ----
template <typename T, bool EXACT, typename Acc>
__device__ void win_left(const Acc &A, int i1, int i2, int j1, int j2, WaveLds<T, EXACT> &S, int lane)
{
    const int R = i2 - i1, L = j2 - j1;   // R <= 32, L <= 64
    const int col = j1 + (lane < L ? lane : 0);
    T a[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) a[r] = (lane < L && r < R) ? A.ld(A.row(i1 + r) + col) : (T)0;
    refl_apply<T, EXACT>(a, R, S, lane, false);
    if (lane < L) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (r < R) A.st(A.row(i1 + r) + col, a[r]);
    }
}

// 1/sqrt(q) and 1/u: hardware estimate refined by Newton steps to full precision
// The hardware estimates flush denormal inputs and results, so arguments
// near the ends of the exponent range are rescaled by a power of two first
// (exact): a squared norm below 2^-960 (fp64) / 2^-100 (fp32), a reciprocal
// argument outside 2^+-960 / 2^+-100.
__device__ __forceinline__ double rsq_nr(double q) {
    const bool tiny = q < 0x1p-960;
    const double qs = tiny ? q * 0x1p+1000 : q;
    double r = __builtin_amdgcn_rsq(qs);
    const double h = 0.5 * qs;
    r = r * fma(-h * r, r, 1.5);
    r = r * fma(-h * r, r, 1.5);
    return tiny ? r * 0x1p+500 : r;
}
__device__ __forceinline__ float rsq_nr(float q) {
    const bool tiny = q < 0x1p-100f;
    const float qs = tiny ? q * 0x1p+100f : q;
    const float r = __builtin_amdgcn_rsqf(qs);
    const float rr = r * fmaf(-0.5f * qs * r, r, 1.5f);
    return tiny ? rr * 0x1p+50f : rr;
}
__device__ __forceinline__ double rcp_nr(double u) {
    const double au = fabs(u);
    const double sc = au < 0x1p-960 ? 0x1p+960 : (au > 0x1p+960 ? 0x1p-960 : 1.0);
    const double us = u * sc;
    double y = __builtin_amdgcn_rcp(us);
    y = fma(y, fma(-us, y, 1.0), y);
    y = fma(y, fma(-us, y, 1.0), y);
    return y * sc;
}
__device__ __forceinline__ float rcp_nr(float u) {
    const float au = fabsf(u);
    const float sc = au < 0x1p-100f ? 0x1p+100f : (au > 0x1p+100f ? 0x1p-100f : 1.0f);
    const float us = u * sc;
    const float y = __builtin_amdgcn_rcpf(us);
    return fmaf(y, fmaf(-us, y, 1.0f), y) * sc;
}

// ---- the reference's task list of one sweep --------------------------------
// Task 0: top right window, task 1: top left window, then tasks 2+2k / 3+2k:
// right / left windows of iteration k (svd_parallel.h:651-687).  An empty
// window (no columns) is skipped exactly as the reference skips it.
struct Win {
    int i1, i2, j1, j2;
};

struct SweepIter {
    int m, n, bs;       // bs = b + 1  (svd_parallel.h:648)
    int i;              // sweep index
    int ntask;          // 2 + 2*(nbtx+1)
    Win tl;             // running t_left
    // sigma = 1: the sigma-preserving geometry (BRD_SIGMA): one more window
    // pair per sweep, so the last bulge is chased off the matrix instead of
    // dropped (oracle_brd_p2x; empty windows are skipped by the callers)
    __device__ void init(int m_, int n_, int b, int i_, int sigma) {
        m = m_; n = n_; bs = b + 1; i = i_;
        const int tl_j2 = min(i + bs + bs - 1, n);
        const int nbtx = (n - tl_j2) / (bs - 1) + sigma;
        ntask = 2 + 2 * (nbtx + 1);
    }
    // Window of task t (tasks must be requested in order 0,1,2,...).
    __device__ Win task(int t, bool &is_right) {
        Win w;
        if (t == 0) {
            w = {i, min(i + bs, m), i + 1, min(i + bs, n)};
            tl = w;
            is_right = true;
        } else if (t == 1) {
            w = {i + 1, min(i + bs, m), i + 1, min(i + bs + bs - 1, n)};
            tl = w;
            is_right = false;
        } else if ((t & 1) == 0) {
            const int end_i = min(tl.i2 + bs - 1, m);
            const int start_j = min(tl.j1 + bs - 1, n);
            const int end_j3 = min(tl.j2 + bs - 1, n);
            w = {tl.i1, end_i, start_j, tl.j2};
            tl = {tl.i2, end_i, start_j, end_j3};
            is_right = true;
        } else {
            w = tl;
            is_right = false;
        }
        return w;
    }
    // Whether task t+1's window is at least k x k (the state after task t;
    // the lag-2 deferral's condition: the next window hosts the fixup).
    __device__ bool next_at_least(int t, int k) const {
        if (t + 1 >= ntask) return false;
        int nr, nc;
        if (t == 0) {
            nr = min(i + bs, m) - (i + 1);
            nc = min(i + bs + bs - 1, n) - (i + 1);
        } else if (((t + 1) & 1) == 0) {   // a right window from the running t_left
            nr = min(tl.i2 + bs - 1, m) - tl.i1;
            nc = tl.j2 - min(tl.j1 + bs - 1, n);
        } else {                           // the left window is t_left itself
            nr = tl.i2 - tl.i1;
            nc = tl.j2 - tl.j1;
        }
        return nr >= k && nc >= k;
    }
    // Top row of task t+1 given the state after task t (window tops are
    // non-decreasing along a sweep); m once the sweep is finished.
    __device__ int next_top(int t) const {
        if (t + 1 >= ntask) return m;
        return t == 0 ? i + 1 : tl.i1;
    }
};

constexpr int kSpinLimit = 1 << 24;

__device__ __forceinline__ int sweep_ntask(int m, int n, int b, int i, int sigma) {
    SweepIter it;
    it.init(m, n, b, i, sigma);
    return it.ntask;
}

// ==========================================================================
// k_band2bd_pipe: sweep i runs on wave i mod NW of a persistent grid and
// executes its tasks in order; task t of sweep i may start once task t+3 of
// sweep i-1 has finished (or sweep i-1 is complete).  Lag 3 is the smallest
// lag for which every pair of overlapping windows keeps the reference's
// serial order (checked exhaustively in tests/test_stage2_schedule.py).
// Hand-off (MI355X_MICROARCH.md, valid forms, table row 1): every band access
// is an sc1 load/store, the producing wave drains its stores
// (s_waitcnt vmcnt(0)) before its sc1 progress-flag store, and the consuming
// wave polls that flag with sc1 loads before its own sc1 loads.
// ==========================================================================
template <typename T, bool EXACT>
__global__ void __launch_bounds__(64) k_band2bd_pipe(T *A, int m, int n, long lda, int b, int sigma, int *prog,
                                                     int *err)
{
    __shared__ WaveLds<T, EXACT> S;
    const int lane = threadIdx.x;
    const int nw = gridDim.x;
    const HbmAcc<T> acc{A, lda};
    for (int i = blockIdx.x; i < n - 1; i += nw) {
        SweepIter it;
        it.init(m, n, b, i, sigma);
        const int prev_ntask = i > 0 ? sweep_ntask(m, n, b, i - 1, sigma) : 0;
        for (int t = 0; t < it.ntask; ++t) {
            bool right;
            const Win wnd = it.task(t, right);
            if (i > 0) {
                const int need = min(t + 4, prev_ntask);
                if (lane == 0) {
                    int spins = 0;
                    while (__hip_atomic_load(prog + i - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > kSpinLimit) {
                            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (wnd.j2 > wnd.j1 && wnd.i2 > wnd.i1) {
                if (right) win_right<T, EXACT>(acc, wnd.i1, wnd.i2, wnd.j1, wnd.j2, S, lane);
                else       win_left<T, EXACT>(acc, wnd.i1, wnd.i2, wnd.j1, wnd.j2, S, lane);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (lane == 0) __hip_atomic_store(prog + i, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ==========================================================================
// k_band2bd_bundle: workgroup = S compute waves + loader + writer; bundle beta =
// sweeps beta*S .. beta*S+S-1, bundles dealt round-robin to a persistent grid.
//
// LDS ring: band row r (diagonals -(b-1)..2b-1, every element any window can
// touch) lives in slot r % R while the bundle works on it.  Compute wave s runs
// sweep beta*S+s on the ring with the lag-3 rule against wave s-1 (LDS
// progress flags) and publishes the top row of its next window ("front").
// The loader wave fills the ring ahead of the sweeps, 16 rows per batch, as
// far as the ring allows (slot r is free once the writer has read row r-R)
// and as far as bundle beta-1 has finished (its rows_done counter).  The
// writer wave writes back every row below all fronts (no sweep of the bundle
// touches it again) and advances rows_done[beta].
// Bundle beta+1 loads a row only after bundle beta is done with it, so every
// element still sees the reference's serial order.  Row hand-offs between
// bundles use the sc1 protocol of k_band2bd_pipe.
// ==========================================================================
struct BundleFlags {
    int prog[16];    // tasks completed per compute wave
    int front[16];   // top row of each wave's next window (n when done)
    int loaded;      // rows < loaded are in the ring (loader wave)
    int freed;       // ring slots of rows < freed may be reused (writer wave)
    int avail;       // rows < avail have been written back by bundle beta-1 (poller wave)
};

__device__ __forceinline__ int lds_acq(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_rel(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Workgroup = S compute waves (one per sweep) + loader + writer + poller:
// up to 3 (fp64, LDS-limited: the ring also needs slack for the loader, see
// bundle_plan) or 5 (fp32) sweeps.
template <typename T> constexpr int bundle_max_threads() { return 64 * ((sizeof(T) == 8 ? 3 : 5) + 3); }
// (BRD_S2_* macros: developer A/B builds, tools/variant_lib.sh; measured at
// N = 8192 fp64, round 2: 63 rows in flight 87.3 vs 87.6 ms, 4-row loader
// chunks 93.2, 16-row writer batches 89.0, compute waves at s_setprio 2 87.2 --
// and two or three LDS-DMA loader waves dealing the rows in chunks 89.4 /
// 91.5: the loader's rate is not what holds the chain)
#ifndef BRD_S2_WRITE_ROWS
#define BRD_S2_WRITE_ROWS 32
#endif
#ifndef BRD_S2_FLY
#define BRD_S2_FLY 48
#endif
#ifndef BRD_S2_CHUNK
#define BRD_S2_CHUNK 8
#endif
constexpr int kWriteRows = BRD_S2_WRITE_ROWS;  // rows per writer batch (at most)
constexpr int kSubRows = 8;                    // rows per writer sub-chunk (registers)
constexpr int kFly = BRD_S2_FLY;               // loader: rows in flight (LDS-DMA), <= 63
constexpr int kChunk = BRD_S2_CHUNK;           // loader: rows published per wait

// s_waitcnt vmcnt(k) for a run-time k in [0, 63] (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int k) {
    switch (k) {
#define BRD_VMCNT_CASE(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        BRD_VMCNT_CASE(1) BRD_VMCNT_CASE(2) BRD_VMCNT_CASE(3) BRD_VMCNT_CASE(4) BRD_VMCNT_CASE(5)
        BRD_VMCNT_CASE(6) BRD_VMCNT_CASE(7) BRD_VMCNT_CASE(8) BRD_VMCNT_CASE(9) BRD_VMCNT_CASE(10)
        BRD_VMCNT_CASE(11) BRD_VMCNT_CASE(12) BRD_VMCNT_CASE(13) BRD_VMCNT_CASE(14) BRD_VMCNT_CASE(15)
        BRD_VMCNT_CASE(16) BRD_VMCNT_CASE(17) BRD_VMCNT_CASE(18) BRD_VMCNT_CASE(19) BRD_VMCNT_CASE(20)
        BRD_VMCNT_CASE(21) BRD_VMCNT_CASE(22) BRD_VMCNT_CASE(23) BRD_VMCNT_CASE(24) BRD_VMCNT_CASE(25)
        BRD_VMCNT_CASE(26) BRD_VMCNT_CASE(27) BRD_VMCNT_CASE(28) BRD_VMCNT_CASE(29) BRD_VMCNT_CASE(30)
        BRD_VMCNT_CASE(31) BRD_VMCNT_CASE(32) BRD_VMCNT_CASE(33) BRD_VMCNT_CASE(34) BRD_VMCNT_CASE(35)
        BRD_VMCNT_CASE(36) BRD_VMCNT_CASE(37) BRD_VMCNT_CASE(38) BRD_VMCNT_CASE(39) BRD_VMCNT_CASE(40)
        BRD_VMCNT_CASE(41) BRD_VMCNT_CASE(42) BRD_VMCNT_CASE(43) BRD_VMCNT_CASE(44) BRD_VMCNT_CASE(45)
        BRD_VMCNT_CASE(46) BRD_VMCNT_CASE(47) BRD_VMCNT_CASE(48)
        BRD_VMCNT_CASE(49) BRD_VMCNT_CASE(50) BRD_VMCNT_CASE(51) BRD_VMCNT_CASE(52) BRD_VMCNT_CASE(53)
        BRD_VMCNT_CASE(54) BRD_VMCNT_CASE(55) BRD_VMCNT_CASE(56) BRD_VMCNT_CASE(57) BRD_VMCNT_CASE(58)
        BRD_VMCNT_CASE(59) BRD_VMCNT_CASE(60) BRD_VMCNT_CASE(61) BRD_VMCNT_CASE(62) BRD_VMCNT_CASE(63)
#undef BRD_VMCNT_CASE
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}
template <typename T> constexpr int kEpp = 16 / sizeof(T);   // elements per 16-byte piece

// Ring row pitch: diagonals -(b-1) .. 2b-1 (3b-1 elements), rounded up to a
// multiple of 16 bytes (rows move as 16-byte pieces: LDS-DMA in, b128 out),
// which also leaves consecutive rows (a right window's lanes) an odd number
// of elements apart: conflict-free LDS access.
template <typename T>
__host__ __device__ constexpr int ring_pitch(int b) {
    return (3 * b - 1 + (int)(16 / sizeof(T)) - 1) / (int)(16 / sizeof(T)) * (int)(16 / sizeof(T));
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// One 16-byte piece per lane from global memory (sc1) straight into LDS at
// lds_byte + 16 * lane (global_load_lds_dwordx4; M0 = the wave-uniform LDS base,
// saved and restored inside the statement).  Counted by vmcnt; the compiler does
// not see it, so the caller waits explicitly.
__device__ __forceinline__ void dma16_sc1(const void *gsrc, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_byte) : "memory");
}
// Ring image of an edge row (some of its P columns outside the matrix):
// clamped element loads, zeros outside.
template <typename T>
__device__ __forceinline__ void load_edge_row(const T *A, long lda, int n, int b, int r, T *dst, int row_q, int lane) {
    if (lane < row_q) {
        const int c0 = r - (b - 1) + lane * kEpp<T>;
        T e[kEpp<T>];
#pragma unroll
        for (int k = 0; k < kEpp<T>; ++k) {
            const int c = c0 + k;
            e[k] = (c >= 0 && c < n) ? ld_c(A + (long)r * lda + c) : (T)0;
        }
        u32x4 v;
        __builtin_memcpy(&v, e, 16);
        *(u32x4 *)(dst + lane * kEpp<T>) = v;
    }
}
// 16-byte agent-coherent (sc1, write-through) store
__device__ __forceinline__ void st16_sc1(void *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}


template <typename T, bool EXACT>
__global__ void __launch_bounds__((bundle_max_threads<T>()))
k_band2bd_bundle(T *A, int n, long lda, int b, int sigma, int S, int R, unsigned magic, int *rows_done, int *err)
{
    extern __shared__ __align__(16) unsigned char smem[];
    const int P = ring_pitch<T>(b);
    T *ring = (T *)smem;
    const size_t ring_bytes = ((size_t)R * P * sizeof(T) + 15) & ~(size_t)15;
    WaveLds<T, EXACT> *wl = (WaveLds<T, EXACT> *)(smem + ring_bytes);
    BundleFlags *F = (BundleFlags *)(wl + S);
    // readfirstlane: the compiler then keeps all window geometry in SGPRs
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const RingAcc<T> acc{ring, P, R, b - 1, magic};
    const int nbundles = (n - 1 + S - 1) / S;

    for (int beta = blockIdx.x; beta < nbundles; beta += gridDim.x) {
        const int i0 = beta * S;
        const int nsw = min(S, n - 1 - i0);
        if (threadIdx.x < 16) {
            F->prog[threadIdx.x] = 0;
            F->front[threadIdx.x] = (int)threadIdx.x < nsw ? i0 + (int)threadIdx.x : n;
        }
        if (threadIdx.x == 0) { F->loaded = i0; F->freed = i0; F->avail = 0; }
        __syncthreads();

        if (wave < nsw) {
            // ---------------- compute wave: sweep i0 + sw ----------------
            // Before task t the wave waits, by the lag-3 rule, for the previous
            // sweep to finish task t + 3.
            const int sw = wave;
            const int i = i0 + sw;
            SweepIter it;
            it.init(n, n, b, i, sigma);
            const int prev_ntask = sw > 0 ? sweep_ntask(n, n, b, i - 1, sigma) : 0;
            for (int t = 0; t < it.ntask; ++t) {
                bool right;
                const Win wnd = it.task(t, right);
                const bool live = wnd.j2 > wnd.j1 && wnd.i2 > wnd.i1;
                int spins = 0;
                if (sw > 0) {
                    const int need = min(t + 4, prev_ntask);
                    while (lds_acq(F->prog + sw - 1) < need) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 2); break; }
                    }
                }
                if (live) {
                    while (lds_acq(&F->loaded) < wnd.i2) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 3); break; }
                    }
                    if (right) win_right<T, EXACT>(acc, wnd.i1, wnd.i2, wnd.j1, wnd.j2, wl[sw], lane);
                    else       win_left<T, EXACT>(acc, wnd.i1, wnd.i2, wnd.j1, wnd.j2, wl[sw], lane);
                }
                if (lane == 0) {
                    lds_rel(&F->front[wave], it.next_top(t));
                    lds_rel(&F->prog[wave], t + 1);
                }
            }
        } else if (wave == S) {
            // ---------------- loader wave: HBM -> ring by LDS-DMA ----------------
            // An interior row (all P columns inside the matrix) is copied by ONE
            // global_load_lds_dwordx4 (lane q moves 16-byte piece q, sc1) straight
            // into its ring slot as soon as bundle beta-1 has written it back (the
            // poller wave's `avail`) and its slot is free (`freed`).  Up to kFly
            // rows are in flight; they are published (`loaded`) oldest first, at
            // most kChunk at a time, behind counted vmcnt waits.  No vector load
            // of this wave may sit between a DMA and its wait (the in-order vmcnt
            // would drain every DMA in flight), so the flags come through LDS.
            // Edge rows go synchronously through registers (clamped element
            // loads, zeros outside the matrix).
            const int row_q = P * (int)sizeof(T) / 16;
            const unsigned row_bytes = (unsigned)(P * (int)sizeof(T));
            const unsigned ring_lds = (unsigned)(uintptr_t)ring;
            const unsigned ring_end = ring_lds + (unsigned)R * row_bytes;
            // rows [1, dma_hi] read P elements inside [A, A + (n-1) lda + n): DMA-able
            const int dma_hi = (int)(((long)(n - 1) * lda + n + (b - 1) - P) / (lda + 1));
            int ra = i0, rl = i0, spins = 0;
            unsigned dst = ring_lds + (unsigned)acc.slot(i0) * row_bytes;   // slot of row ra
            const char *src = (const char *)(A + (long)i0 * lda + i0 - (b - 1)) + 16 * lane;
            const long rstep = (lda + 1) * (long)sizeof(T);
            const bool dma_lane = lane < row_q;
            while (rl < n) {
                const int av = __hip_atomic_load(&F->avail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int fr = __hip_atomic_load(&F->freed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int lim = __builtin_amdgcn_readfirstlane(min(min(av, fr + R), min(n, rl + kFly)));
                bool moved = false;
                if (ra < lim) {
                    if (ra >= 1 && ra <= dma_hi) {
                        const int k = min(lim, dma_hi + 1) - ra;
                        if (dma_lane) {   // exec set once for the batch; loop control is uniform
                            const char *p = src;
                            unsigned d = dst;
                            for (int i = 0; i < k; ++i) {
                                dma16_sc1(p, d);
                                p += rstep;
                                d += row_bytes;
                                if (d == ring_end) d = ring_lds;
                            }
                        }
                        src += (long)k * rstep;
                        dst += (unsigned)k * row_bytes;
                        if (dst >= ring_end) dst -= ring_end - ring_lds;
                        ra += k;
                        moved = true;
                    } else if (ra == rl) {   // edge row, once the DMAs before it have landed
                        load_edge_row<T>(A, lda, n, b, ra, (T *)((char *)ring + (dst - ring_lds)), row_q, lane);
                        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                        ++ra;
                        rl = ra;
                        src += rstep;
                        dst += row_bytes;
                        if (dst == ring_end) dst = ring_lds;
                        if (lane == 0) lds_rel(&F->loaded, rl);
                        moved = true;
                    }
                }
                if (ra > rl) {
                    const int keep = max(0, ra - rl - kChunk);
                    wait_vmcnt(keep);
                    rl = ra - keep;
                    if (lane == 0) lds_rel(&F->loaded, rl);
                    spins = 0;
                } else if (!moved) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 4); break; }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (wave == S + 2) {
            // ---------------- poller wave: rows bundle beta-1 has written back ----------------
            if (beta == 0) {
                if (lane == 0) lds_rel(&F->avail, n);
            } else {
                const int *done_prev = rows_done + beta - 1;
                int av = 0, spins = 0;
                while (av < n) {
                    const int v = __builtin_amdgcn_readfirstlane(ld_c(done_prev));
                    if (v != av) {
                        av = v;
                        if (lane == 0) lds_rel(&F->avail, v);
                        spins = 0;
                    } else {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 6); break; }
                    }
                }
            }
        } else if (wave == S + 1) {
            // ---------------- writer wave: ring -> HBM ----------------
            // Writes every row below all fronts (no sweep of the bundle touches it
            // again), <= kWriteRows per batch: ring -> registers (the slots are
            // freed at once) -> 16-byte sc1 stores.  A batch is published in
            // rows_done[beta] once its stores have drained, which the writer
            // checks after issuing the next batch (counted vmcnt) or when idle,
            // so the drain of one batch overlaps the next.
            const int row_q = P * (int)sizeof(T) / 16;
            int wb = i0, spins = 0, pend = -1;
            while (wb < n) {
                int fmin = n;
                for (int s = 0; s < nsw; ++s) fmin = min(fmin, lds_acq(&F->front[s]));
                const int wt = __builtin_amdgcn_readfirstlane(min(min(fmin, lds_acq(&F->loaded)), wb + kWriteRows));
                if (wt <= wb) {
                    if (pend >= 0) {   // idle: retire the batch in flight
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        if (lane == 0) st_c(rows_done + beta, pend);
                        pend = -1;
                        continue;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 5); break; }
                    continue;
                }
                spins = 0;
                const int k = wt - wb;
                const bool interior = wb >= b - 1 && wt - 1 - (b - 1) + P <= n;
                // the batch moves in sub-chunks of kSubRows rows (registers: one
                // sub-chunk); each sub-chunk's slots are freed once it is read
                int sl = acc.slot(wb);
                const char *g = (const char *)(A + (long)wb * lda + wb - (b - 1)) + 16 * lane;
                const long gstep = (lda + 1) * (long)sizeof(T);
                for (int c = 0; c < k; c += kSubRows) {
                    const int kc = min(kSubRows, k - c);
                    u32x4 v[kSubRows];
                    const u32x4 *srow = (const u32x4 *)(ring + sl * P) + (lane < row_q ? lane : 0);
                    const int wrap = R - sl;   // rows before the ring wraps
#pragma unroll
                    for (int rr = 0; rr < kSubRows; ++rr)
                        if (rr < kc) v[rr] = srow[(rr < wrap ? rr : rr - R) * (P / kEpp<T>)];
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) lds_rel(&F->freed, wb + c + kc);   // slots reusable once read
                    sl = sl + kc >= R ? sl + kc - R : sl + kc;
                    if (interior) {
                        if (lane < row_q) {
#pragma unroll
                            for (int rr = 0; rr < kSubRows; ++rr) {
                                if (rr < kc) st16_sc1((void *)g, v[rr]);
                                g += gstep;
                            }
                        }
                    } else {
#pragma unroll
                        for (int rr = 0; rr < kSubRows; ++rr) {
                            const int r = wb + c + rr;
                            if (rr < kc && lane < row_q) {
                                T *ge = A + (long)r * lda + r - (b - 1) + lane * kEpp<T>;
                                const int cc0 = r - (b - 1) + lane * kEpp<T>;
                                T e[kEpp<T>];
                                __builtin_memcpy(e, &v[rr], 16);
#pragma unroll
                                for (int kk = 0; kk < kEpp<T>; ++kk)
                                    if (cc0 + kk >= 0 && cc0 + kk < n) st_c(ge + kk, e[kk]);
                            }
                        }
                    }
                }
                if (interior) {
                    if (pend >= 0) {   // everything older than this batch's k stores has drained
                        wait_vmcnt(k);
                        if (lane == 0) st_c(rows_done + beta, pend);
                    }
                    pend = wt;
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0) st_c(rows_done + beta, wt);
                    pend = -1;
                }
                wb = wt;
            }
            if (pend >= 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) st_c(rows_done + beta, pend);
            }
        }
        __syncthreads();
    }
}

}  // namespace brd
#include "brd_s2win.h"
namespace brd {

// ==========================================================================
// k_sweeps: the b = 32 fast-arithmetic bundle kernel (the production stage 2).
// Workgroup = S compute waves (one wave per sweep, brd_s2win.h windows) +
// loader + writer + poller; bundle beta = sweeps beta*S .. beta*S+S-1, dealt
// round-robin to a persistent grid, rows handed between bundles through HBM
// exactly as in k_band2bd_bundle (sc1 stores drained before an sc1 flag,
// sc1 polls, LDS-DMA loads).  What differs from k_band2bd_bundle:
//  * one wave per window (no per-task meeting of a wave pair; the window is
//    straight-line code on 32 elements per lane);
//  * the progress words are plain LDS stores behind the window's ring stores
//    (LDS executes a wave's operations in order), no lgkmcnt drain on the
//    compute waves' critical path;
//  * the writer publishes rows_done per 8-row piece behind counted vmcnt
//    waits, so the next bundle's loader starts on the first piece while the
//    rest drains;
//  * a compact role split (no SGPR spills: one window code path per kind).
// ==========================================================================
constexpr int kSweepWriters = 2;   // writer waves (batches dealt alternately)
// Rows per writer batch, by size (k_sweeps' template argument WR).  Same box,
// N = 8192: 8 / 16 / 24 / 32 rows 102.6 / 73.7 / 77.3 / 72.8-73.2 ms fp64 (16:
// 71.5 beside 72.8 in another pair), 78.9 / 60.1 / 62.2 / 60.8 fp32; N = 16384
// fp64: 16 rows 156.2, 32 rows 146.0.  Between the two sizes (not measured)
// the switch is at the midpoint.  BRD_S2_SWEEP_ROWS=16 / 32 forces either.
constexpr int kSweepRowsSplitN = 12288;
// The shrinking grid's stages (k_sweeps, SweepStages): the grid halves once
// the bundles alive at once, (n - i) / (64 S) + 1, times kStageMargin plus
// kStageSpare fit in half of it; at least kStageMin workgroups stay.
// BRD_S2_STAGES=0 keeps the whole grid to the end (A/B).
constexpr double kStageMargin = 1.25;
constexpr int kStageSpare = 2, kStageMin = 4;
static int sweep_rows_for(int n) {
    const char *e = getenv("BRD_S2_SWEEP_ROWS");   // (read per call: tests switch it)
    if (e && (atoi(e) == 16 || atoi(e) == 32)) return atoi(e);
    return n <= kSweepRowsSplitN ? 16 : 32;
}
#ifndef BRD_S2_LAG2
#define BRD_S2_LAG2 0                 // 1: lag 2 with the deferred corner (A/B; bitwise the same band,
                                      // measured 93 ms against lag 3's 72 ms at N = 8192 fp64: the
                                      // fixup's extra LDS round trip sits on the chain it shortens)
#endif
constexpr bool kS2Lag2 = BRD_S2_LAG2 != 0;
#ifndef BRD_S2_DEFER_LAG2
#define BRD_S2_DEFER_LAG2 1           // 0: deferred windows still wait for lag 3 (A/B of the fixup alone)
#endif
#ifndef BRD_S2_REGLOAD
#define BRD_S2_REGLOAD 1              // 0: LDS-DMA only (A/B: N = 8192 fp64 72.9 vs 72.8 ms, fp32 62.9 vs 61.0)
#endif
template <typename T> constexpr int kRG = 16;   // loader: rows loaded into registers ahead of a full ring
struct SweepFlags {
    int prog[12];    // tasks completed per compute wave
    int front[12];   // top row of each compute wave's next window (n when done)
    int loaded;      // rows < loaded are in the ring (loader wave)
    int freed;       // ring slots of rows < freed may be reused (writer waves, in row order)
    int avail;       // rows < avail have been written back by bundle beta-1 (poller wave)
    int wturn;       // writers: index of the next batch to claim
    int wclaim;      // writers: first row of the next batch
    int wpub;        // writers: rows < wpub published in rows_done[beta] (in row order)
};

#ifdef BRD_S2TRACE
// Diagnostic build only (tools/s2trace.py): per-task and per-publication
// timeline of bundles kTrB0 .. kTrB0 + kTrNB - 1 on the chip-wide 100 MHz clock.
constexpr int kTrB0 = 600, kTrNB = 4, kTrTasks = 600, kTrPub = 1024;
struct S2Trace {
    unsigned long long task[kTrNB][12][kTrTasks][4];   // start, lag done, rows ready, end
    unsigned long long pub[kTrNB][8][kTrPub][2];       // loader / writer / poller / claim / issued / ldissue / freed
    int npub[kTrNB][8];
    unsigned long long bundle[kTrNB][4];               // start, end, block, xcc
    unsigned long long wr[kTrNB][256][8];             // writer batch q: stamps
};
__device__ S2Trace g_s2tr;
#define TRB(beta) ((beta) >= kTrB0 && (beta) < kTrB0 + kTrNB)
#define TRT(beta, w, t, k)                                                                      \
    do {                                                                                        \
        if (TRB(beta) && (t) < kTrTasks && lane == 0)                                           \
            g_s2tr.task[(beta) - kTrB0][w][t][k] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)
#define TRP(beta, kind, val)                                                                    \
    do {                                                                                        \
        if (TRB(beta) && lane == 0) {                                                           \
            const int q_ = g_s2tr.npub[(beta) - kTrB0][kind]++;                                 \
            if (q_ < kTrPub) {                                                                  \
                g_s2tr.pub[(beta) - kTrB0][kind][q_][0] = __builtin_amdgcn_s_memrealtime();     \
                g_s2tr.pub[(beta) - kTrB0][kind][q_][1] = (val);                                \
            }                                                                                   \
        }                                                                                       \
    } while (0)
#define TRW(beta, q, k)                                                                         \
    do {                                                                                        \
        if (TRB(beta) && (q) < 256 && lane == 0)                                                \
            g_s2tr.wr[(beta) - kTrB0][q][k] = __builtin_amdgcn_s_memrealtime();                 \
    } while (0)
#else
#define TRT(beta, w, t, k) do {} while (0)
#define TRP(beta, kind, val) do {} while (0)
#define TRW(beta, q, k) do {} while (0)
#endif

template <typename T> constexpr int sweeps_max_threads() { return sizeof(T) == 8 ? 512 : 768; }

__device__ __forceinline__ int lds_ld(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The grid shrinks with the chain (a stage-2 reservation holds whole CUs, so
// in a stream of reductions the CUs it no longer needs go back to stage 1).
// A bundle of S sweeps starting at row i lives (n - i) / 32 task pairs and
// bundles start 4 S tasks apart, so (n - i) / (64 S) bundles are alive at
// once whatever the task time: ~43 at the top of an 8192 fp64 matrix, a few
// near the bottom.  The host splits the bundles into stages (SweepStages:
// bundles [B_k, B_k+1) on the first G_k workgroups, G_k halving from stage to
// stage); in stage k bundle beta goes to workgroup beta mod G_k.  G_k divides
// G_k-1, so a workgroup's next bundle is always >= G_k bundles after its last
// one (consecutive bundles on different workgroups, as with one stage), and
// workgroups >= G_k leave after stage k - 1.  The dealing is static: no
// atomics on the chain's hand-offs.
struct SweepStages {
    int nst;          // stages (1: the whole chain on the grid)
    int B[5];         // first bundle of each stage (B[0] = 0)
    int G[4];         // workgroups of each stage (G[0] = the grid)
};
__device__ __forceinline__ int sweeps_next(const SweepStages &st, int w, int beta, int nbundles) {
    int k = 0;
    while (k + 1 < st.nst && beta >= st.B[k + 1]) ++k;
    int nx = beta + st.G[k];
    while (k + 1 < st.nst && nx >= st.B[k + 1]) {   // into the next stage
        ++k;
        if (w >= st.G[k]) return nbundles;          // not in it: leave
        const int b0 = st.B[k];
        nx = b0 + (((w - b0) % st.G[k]) + st.G[k]) % st.G[k];   // first beta >= B_k with beta = w mod G_k
    }
    return nx;
}
__device__ __forceinline__ int sweeps_first(const SweepStages &st, int w, int nbundles) {
    for (int k = 0; k < st.nst; ++k) {
        if (w >= st.G[k]) return nbundles;
        const int b0 = st.B[k];
        const int c = b0 + (((w - b0) % st.G[k]) + st.G[k]) % st.G[k];
        if (c < st.B[k + 1]) return c;
    }
    return nbundles;
}
template <typename T, int WR>
__global__ void __launch_bounds__(sweeps_max_threads<T>())
k_sweeps(T *A, int n, long lda, int sigma, int S, int R, unsigned magic, int *rows_done, int *err, SweepStages st)
{
    constexpr int b = 32;
    extern __shared__ __align__(16) unsigned char smem[];
    const int P = ring_pitch<T>(b);
    T *ring = (T *)smem;
    const size_t ring_bytes = ((size_t)R * P * sizeof(T) + 15) & ~(size_t)15;
    SweepFlags *F = (SweepFlags *)(smem + ring_bytes);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const S2Ring<T> rg{ring, P, R, magic};
    const int nbundles = (n - 1 + S - 1) / S;

    for (int beta = sweeps_first(st, (int)blockIdx.x, nbundles); beta < nbundles;
         beta = sweeps_next(st, (int)blockIdx.x, beta, nbundles)) {
        const int i0 = beta * S;
        const int nsw = min(S, n - 1 - i0);
        if (threadIdx.x < 12) {
            F->prog[threadIdx.x] = 0;
            F->front[threadIdx.x] = (int)threadIdx.x < nsw ? i0 + (int)threadIdx.x : n;
        }
        if (threadIdx.x == 0) {
            F->loaded = i0; F->freed = i0; F->avail = 0;
            F->wturn = 0; F->wclaim = i0; F->wpub = i0;
        }
#ifdef BRD_S2TRACE
        if (threadIdx.x == 0 && TRB(beta)) {
            g_s2tr.bundle[beta - kTrB0][0] = __builtin_amdgcn_s_memrealtime();
            g_s2tr.bundle[beta - kTrB0][2] = blockIdx.x;
            g_s2tr.bundle[beta - kTrB0][3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
        }
#endif
        __syncthreads();

        if (wave < nsw) {
            // ---------------- compute wave: sweep i0 + wave ----------------
            // Lag 2 with the deferred corner (brd_s2win.h): a full window whose
            // next window can host the fixup starts once the previous sweep has
            // finished window t+2 and defers its last lane; any other window
            // keeps lag 3.  prog[wave] = t means windows < t are complete,
            // deferred parts included (published after the fixup).
            const int i = i0 + wave;
            SweepIter it;
            it.init(n, n, b, i, sigma);
            const int prev_ntask = wave > 0 ? sweep_ntask(n, n, b, i - 1, sigma) : 0;
            S2Fix<T> fx{(T)0, (T)0, (T)0, (T)0, (T)0};
            bool pend = false;
            for (int t = 0; t < it.ntask; ++t) {
                bool right;
                const Win w = it.task(t, right);
                const int nr = w.i2 - w.i1, nc = w.j2 - w.j1;
                const bool live = nr > 0 && nc > 0;
                const bool full = live && (right ? (nr == 2 * b && nc == b) : (nr == b && nc == 2 * b));
                const bool defer = kS2Lag2 && full && it.next_at_least(t, b);
                int spins = 0;
                TRT(beta, wave, t, 0);
                if (wave > 0) {
                    const int need = min(t + (defer ? 4 - BRD_S2_DEFER_LAG2 : 4), prev_ntask);
                    while (lds_ld(&F->prog[wave - 1]) < need) {
                        __builtin_amdgcn_s_sleep(0);
                        if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 12); break; }
                    }
                }
                TRT(beta, wave, t, 1);
                if (live) {
                    while (lds_ld(&F->loaded) < w.i2) {
                        __builtin_amdgcn_s_sleep(0);
                        if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 13); break; }
                    }
                    TRT(beta, wave, t, 2);
                    asm volatile("" ::: "memory");
                    const S2Pub pub{&F->prog[wave], &F->front[wave], t, w.i1};
                    S2Fix<T> fo;
                    if (right) {
                        if (full) s2_right_w1<T, true, kS2Lag2>(rg, w.i1, w.j1, nr, nc, lane, pend, fx, defer, fo, pub);
                        else      s2_right_w1<T, false, kS2Lag2>(rg, w.i1, w.j1, nr, nc, lane, pend, fx, defer, fo, pub);
                    } else {
                        if (full) s2_left_w1<T, true, kS2Lag2>(rg, w.i1, w.j1, nr, nc, lane, pend, fx, defer, fo, pub);
                        else      s2_left_w1<T, false, kS2Lag2>(rg, w.i1, w.j1, nr, nc, lane, pend, fx, defer, fo, pub);
                    }
                    if (defer) fx = fo;
                    asm volatile("" ::: "memory");
                }
                pend = defer;
                TRT(beta, wave, t, 3);
                if (lane == 0) {   // LDS in order: the window's ring stores land first
                    // (a deferring window's front too: its deferred lane lies in
                    // the next window's rows; its progress waits for the fixup)
                    lds_st(&F->front[wave], it.next_top(t));
                    if (!defer) lds_st(&F->prog[wave], t + 1);
                }
            }
        } else if (wave == S) {
            // ---------------- loader wave: HBM -> ring ----------------
            // Rows whose ring slots are free go in by LDS-DMA (one
            // global_load_lds_dwordx4 per interior row, up to kFly rows in
            // flight, published oldest first in chunks of kChunk behind counted
            // vmcnt waits).  When the ring is full (the writers have not freed
            // the next row's slot) and the previous bundle has already written
            // rows back, the next kRG of them are loaded into registers ahead of
            // their slots and stored into the ring (one 16-byte LDS store per
            // lane) the moment each slot is freed: the ring recycle loop -- the
            // trail releases a row, a writer frees its slot, the loader fills it
            // -- is what paces a bundle (the ring was full before 98 % of the
            // DMA issues), and this takes the HBM latency out of it.  Edge rows
            // through registers.
            const int row_q = P * (int)sizeof(T) / 16;
            const bool ql = lane < row_q;
            const unsigned row_bytes = (unsigned)(P * (int)sizeof(T));
            const unsigned ring_lds = (unsigned)(uintptr_t)ring;
            const unsigned ring_end = ring_lds + (unsigned)R * row_bytes;
            const int dma_hi = (int)(((long)(n - 1) * lda + n + (b - 1) - P) / (lda + 1));
            int ra = i0, rl = i0, spins = 0;
            unsigned dst = ring_lds + (unsigned)rg.slot(i0) * row_bytes;
            const char *src = (const char *)(A + (long)i0 * lda + i0 - (b - 1)) + 16 * lane;
            const long rstep = (lda + 1) * (long)sizeof(T);
            const bool dma_lane = lane < row_q;
            while (rl < n) {
                const int av = lds_ld(&F->avail);
                const int fr = lds_ld(&F->freed);
                const int lim = __builtin_amdgcn_readfirstlane(min(min(av, fr + R), min(n, rl + kFly)));
                bool moved = false;
                if (ra < lim) {
                    if (ra >= 1 && ra <= dma_hi) {
                        const int k = min(lim, dma_hi + 1) - ra;
                        if (dma_lane) {
                            const char *p = src;
                            unsigned d = dst;
                            for (int q = 0; q < k; ++q) {
                                dma16_sc1(p, d);
                                p += rstep;
                                d += row_bytes;
                                if (d == ring_end) d = ring_lds;
                            }
                        }
                        src += (long)k * rstep;
                        dst += (unsigned)k * row_bytes;
                        if (dst >= ring_end) dst -= ring_end - ring_lds;
                        ra += k;
                        moved = true;
                        TRP(beta, 5, ra);
                        TRP(beta, 7, (av <= fr + R ? 0 : 1) + (lim == rl + kFly ? 2 : 0));
                    } else if (ra == rl) {   // edge row, once the DMAs before it have landed
                        load_edge_row<T>(A, lda, n, b, ra, (T *)((char *)ring + (dst - ring_lds)), row_q, lane);
                        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                        ++ra;
                        rl = ra;
                        src += rstep;
                        dst += row_bytes;
                        if (dst == ring_end) dst = ring_lds;
                        if (lane == 0) lds_st(&F->loaded, rl);
                        moved = true;
                    }
                }
                if (ra > rl) {
                    const int keep = max(0, ra - rl - kChunk);
                    wait_vmcnt(keep);
                    rl = ra - keep;
                    if (lane == 0) lds_st(&F->loaded, rl);
                    TRP(beta, 0, rl);
                    spins = 0;
                } else if (BRD_S2_REGLOAD && !moved && ra < av && fr + R <= ra && ra >= 1 && ra <= dma_hi) {
                    // the ring is full and rows are waiting upstream: the next
                    // rows into registers, then into their slots as they free
                    const int k = __builtin_amdgcn_readfirstlane(min(min(kRG<T>, av - ra), dma_hi + 1 - ra));
                    u32x4 g[kRG<T>];
                    {
                        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                            (void *)(A + (long)ra * lda + ra - (b - 1)), (short)0, 0x7fffffff, 0x00020000);
                        const int vo = 16 * (ql ? lane : 0);
#pragma unroll
                        for (int kk = 0; kk < kRG<T>; ++kk)   // (past k: row ra again, a fixed count)
                            g[kk] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (unsigned)((kk < k ? kk : 0) * rstep), 16);
                    }
                    const int sl0 = (int)((dst - ring_lds) / row_bytes);
                    int fl = fr + R;   // rows < fl have free slots
#pragma unroll
                    for (int kk = 0; kk < kRG<T>; ++kk) {
                        if (kk < k) {
                            const int r = ra + kk;
                            if (r >= fl) {
                                if (kk > 0 && lane == 0) lds_st(&F->loaded, r);
                                int f2 = __builtin_amdgcn_readfirstlane(lds_ld(&F->freed));
                                while (f2 + R <= r) {
                                    __builtin_amdgcn_s_sleep(0);
                                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 14); break; }
                                    f2 = __builtin_amdgcn_readfirstlane(lds_ld(&F->freed));
                                }
                                fl = f2 + R;
                            }
                            const int sl = sl0 + kk >= R ? sl0 + kk - R : sl0 + kk;
                            if (ql) *((u32x4 *)(ring + sl * P) + lane) = g[kk];
                        }
                    }
                    ra += k;
                    rl = ra;
                    src += (long)k * rstep;
                    dst += (unsigned)k * row_bytes;
                    if (dst >= ring_end) dst -= ring_end - ring_lds;
                    if (lane == 0) lds_st(&F->loaded, rl);   // LDS in order: after the rows
                    TRP(beta, 0, rl);
                    spins = 0;
                } else if (!moved) {
                    __builtin_amdgcn_s_sleep(0);
                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 14); break; }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (wave == S + 1 + kSweepWriters) {
            // ---------------- poller wave: rows bundle beta-1 has written back ----------------
            if (beta == 0) {
                if (lane == 0) lds_st(&F->avail, n);
            } else {
                const int *done_prev = rows_done + beta - 1;
                int av = 0, spins = 0;
                while (av < n) {
                    const int v = __builtin_amdgcn_readfirstlane(ld_c(done_prev));
                    if (v != av) {
                        av = v;
                        if (lane == 0) lds_st(&F->avail, v);
                        TRP(beta, 2, v);
                        spins = 0;
                    } else {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 16); break; }
                    }
                }
            }
        } else if (wave > S && wave <= S + kSweepWriters) {
            // ---------------- writer waves: ring -> HBM ----------------
            // Batches of at most WR rows below all fronts (no sweep of
            // the bundle touches them again), dealt alternately to the writer
            // waves so that one batch's drain overlaps the next batch's stores
            // (a single writer that drains each batch before taking the next
            // held the whole chain to one batch per drain latency).  Per batch:
            // claim its rows (in turn), ring -> registers, free the slots (in
            // row order), 16-byte sc1 stores, drain, publish rows_done[beta]
            // (in row order).
            const int wi = wave - S - 1;
            const int row_q = P * (int)sizeof(T) / 16;
            const long gstep = (lda + 1) * (long)sizeof(T);
            for (int q = wi;; q += kSweepWriters) {
                int spins = 0;
                while (lds_ld(&F->wturn) != q) {   // the previous batch is claimed
                    __builtin_amdgcn_s_sleep(0);
                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 15); break; }
                }
                const int wb = __builtin_amdgcn_readfirstlane(lds_ld(&F->wclaim));
                if (wb >= n) {   // all rows claimed: let the other writer see it too
                    if (lane == 0) lds_st(&F->wturn, q + 1);
                    break;
                }
                int wt = wb;
                spins = 0;
                for (;;) {
                    int fmin = n;
                    for (int s = 0; s < nsw; ++s) fmin = min(fmin, lds_ld(&F->front[s]));
                    wt = __builtin_amdgcn_readfirstlane(min(min(fmin, lds_ld(&F->loaded)), wb + WR));
                    if (wt > wb) break;
                    __builtin_amdgcn_s_sleep(0);
                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 15); break; }
                }
                if (wt <= wb) break;
                if (lane == 0) {
                    lds_st(&F->wclaim, wt);
                    lds_st(&F->wturn, q + 1);
                }
                TRP(beta, 3, wb);
                TRW(beta, q, 0);
                const int k = wt - wb;
                // ring -> registers -> HBM in halves of kH rows (registers); each
                // half's slots are freed (in row order) once it is read.  A full
                // interior half that does not wrap the ring is straight-line code
                // (immediate LDS offsets, buffer stores with the row offset in
                // soffset); anything else goes row by row.
                constexpr int kH = WR / 2;
                const int sl0 = rg.slot(wb);
                const unsigned rstride = (unsigned)gstep;
                for (int r0 = 0; r0 < k; r0 += kH) {
                    const int kh = min(kH, k - r0);
                    const int sl = sl0 + r0 >= R ? sl0 + r0 - R : sl0 + r0;
                    const int rb = wb + r0;
                    const bool fast = kh == kH && sl + kH <= R && rb >= b - 1 && rb + kH - 1 - (b - 1) + P <= n;
                    if (fast) {
                        u32x4 v[kH];
                        const u32x4 *srow = (const u32x4 *)(ring + sl * P) + (lane < row_q ? lane : 0);
#pragma unroll
                        for (int rr = 0; rr < kH; ++rr) v[rr] = srow[rr * (P / kEpp<T>)];
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        TRW(beta, q, 1 + 3 * (r0 / kH));
                        spins = 0;
                        while (lds_ld(&F->freed) != rb) {   // slots are freed in row order
                            __builtin_amdgcn_s_sleep(0);
                            if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 15); break; }
                        }
                        if (lane == 0) lds_st(&F->freed, rb + kH);
                        TRP(beta, 6, rb + kH);
                        TRW(beta, q, 2 + 3 * (r0 / kH));
                        if (lane < row_q) {
                            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                                (void *)(A + (long)rb * lda + rb - (b - 1)), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
                            for (int rr = 0; rr < kH; ++rr)
                                __builtin_amdgcn_raw_buffer_store_b128(v[rr], rs, 16 * lane, rr * rstride, 16);   // sc1
                        }
                        TRW(beta, q, 3 + 3 * (r0 / kH));
                    } else {
                        for (int rr = 0; rr < kh; ++rr) {
                            const int r = rb + rr;
                            const int sk = sl + rr >= R ? sl + rr - R : sl + rr;
                            const u32x4 vr = ((const u32x4 *)(ring + sk * P))[lane < row_q ? lane : 0];
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            if (lane < row_q) {
                                if (r >= b - 1 && r - (b - 1) + P <= n) {
                                    st16_sc1((void *)((const char *)(A + (long)r * lda + r - (b - 1)) + 16 * lane), vr);
                                } else {
                                    T *ge = A + (long)r * lda + r - (b - 1) + lane * kEpp<T>;
                                    const int cc0 = r - (b - 1) + lane * kEpp<T>;
                                    T e[kEpp<T>];
                                    __builtin_memcpy(e, &vr, 16);
#pragma unroll
                                    for (int kk = 0; kk < kEpp<T>; ++kk)
                                        if (cc0 + kk >= 0 && cc0 + kk < n) st_c(ge + kk, e[kk]);
                                }
                            }
                        }
                        spins = 0;
                        while (lds_ld(&F->freed) != rb) {
                            __builtin_amdgcn_s_sleep(0);
                            if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 15); break; }
                        }
                        if (lane == 0) lds_st(&F->freed, rb + kh);
                        TRP(beta, 6, rb + kh);
                    }
                }
                TRP(beta, 4, wt);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                TRW(beta, q, 7);
                spins = 0;
                while (lds_ld(&F->wpub) != wb) {   // rows_done advances in row order
                    __builtin_amdgcn_s_sleep(0);
                    if (++spins > kSpinLimit) { if (lane == 0) st_c(err, 15); break; }
                }
                if (lane == 0) {
                    st_c(rows_done + beta, wt);
                    lds_st(&F->wpub, wt);
                }
                TRP(beta, 1, wt);
            }
        }
        __syncthreads();
#ifdef BRD_S2TRACE
        if (threadIdx.x == 0 && TRB(beta)) g_s2tr.bundle[beta - kTrB0][1] = __builtin_amdgcn_s_memrealtime();
#endif
    }
}

#ifdef BRD_S2TRACE
extern "C" int brd_dbg_s2trace(void *dst, size_t bytes, int reset) {
    if (reset) {
        static S2Trace z;
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_s2tr), &z, sizeof(S2Trace));
    }
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_s2tr), bytes < sizeof(S2Trace) ? bytes : sizeof(S2Trace));
}
#endif

template <typename T>
__global__ void k_extract(const T *A, int n, long lda, T *d, T *e)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = A[(long)i * lda + i];
    if (i < n - 1) e[i] = A[(long)i * lda + i + 1];
}

// ---- bundle geometry ---------------------------------------------------------
// Ring rows needed for S sweeps to make progress: the leading sweep may have to
// run 3(S-1) tasks (1.5(S-1) window pairs of b rows) ahead of the trailing one,
// plus a 2b-row window, plus S rows of sweep shift; checked against the exact
// geometry in tests/test_stage2_schedule.py.
int ring_min_rows(int b, int S) { return ((3 * (S - 1)) / 2 + 2) * b + S + 8; }

template <typename T, bool EXACT>
static size_t bundle_lds_bytes(int b, int S, int R) {
    const size_t ring = ((size_t)R * ring_pitch<T>(b) * sizeof(T) + 15) & ~(size_t)15;
    return ring + (size_t)S * sizeof(WaveLds<T, EXACT>) + sizeof(BundleFlags);
}

template <typename T, bool EXACT>
static bool bundle_plan(int n, int b, int &S, int &R) {
    const size_t budget = 160 * 1024 - 512;
    static const char *senv = getenv("BRD_S2_SWEEPS");   // tuning: cap on sweeps per bundle
    int smax = EXACT ? 2 : bundle_max_threads<T>() / 64 - 3;
    if (senv && atoi(senv) > 0) smax = std::min(smax, atoi(senv));
    // Prefer the most sweeps whose ring keeps 16 rows of slack beyond the
    // minimum (the loader's run-ahead; more sweeps per bundle amortise the
    // inter-bundle hand-off, which dominates -- measured at N = 8192 fp64:
    // S = 2 106 ms, S = 3 95 ms, S = 4 95 ms); else the most that fit at all.
    const bool forced = senv && atoi(senv) > 0;   // a requested S only needs to fit
    for (int slack : {forced ? 8 : 16, 8}) {
        for (S = std::min(smax, std::max(1, n - 1)); S >= 1; --S) {
            const int rmin = ring_min_rows(b, S) + slack;
            if (bundle_lds_bytes<T, EXACT>(b, S, rmin) <= budget) {
                // largest ring that fits, but no more than n rows
                static const char *renv = getenv("BRD_S2_RING");   // tuning: cap on ring rows
                const int rcap = renv && atoi(renv) > 0 ? std::max(rmin, atoi(renv)) : 1 << 30;
                R = rmin;
                while (R < n + 1 && R + 8 <= rcap && bundle_lds_bytes<T, EXACT>(b, S, R + 8) <= budget) R += 8;
                return true;
            }
        }
    }
    return false;
}

// k_sweeps geometry: S sweeps per bundle (one compute wave each) and a ring of
// R rows.  The most sweeps whose ring keeps kSweepSlack rows beyond
// ring_min_rows (the loader's run-ahead: one 32-row release of the trailing
// sweep in flight), then the largest ring that fits.  BRD_S2_SWEEPS caps S
// (tuning).
constexpr int kSweepSlack = 40;
template <typename T>
static size_t sweeps_lds_bytes(int R, int S) {
    (void)S;
    return (((size_t)R * ring_pitch<T>(32) * sizeof(T) + 15) & ~(size_t)15) + ((sizeof(SweepFlags) + 15) & ~(size_t)15);
}
template <typename T>
static bool sweeps_plan(int n, int &S, int &R) {
    const size_t budget = 160 * 1024;
    static const char *senv = getenv("BRD_S2_SWEEPS");
    int smax = sweeps_max_threads<T>() / 64 - 2 - kSweepWriters;
    if (smax > 12) smax = 12;
    if (senv && atoi(senv) > 0) smax = std::min(smax, atoi(senv));
    for (S = std::min(smax, std::max(1, n - 1)); S >= 1; --S) {
        const int rmin = ring_min_rows(32, S) + kSweepSlack;
        if (sweeps_lds_bytes<T>(rmin, S) <= budget) {
            R = rmin;
            while (R < n + 1 && sweeps_lds_bytes<T>(R + 1, S) <= budget) ++R;
            return true;
        }
    }
    return false;
}

// Workgroups of `fn` (block threads, dynamic LDS bytes) that can be resident
// at once on the device: the persistent sweep kernels hand bundles / sweeps
// round-robin and wait on their predecessors, so every workgroup of the grid
// must be able to run at the same time.
static int coresident_limit(const void *fn, int threads, size_t lds) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds) != hipSuccess) return 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return per_cu * cus;
}

static SweepStages sweep_stages(int n, int S, int nbundles, int grid) {
    SweepStages st{};
    st.nst = 1;
    st.B[0] = 0;
    st.G[0] = grid;
    st.B[1] = nbundles;
    const char *e = getenv("BRD_S2_STAGES");   // (read per call: tests switch it)
    if (e && atoi(e) == 0) return st;
    int g = grid;
    for (int beta = 0; beta < nbundles && st.nst < 4; ++beta) {
        const double alive = (double)(n - beta * S) / (64.0 * S) + 1.0;
        const int half = g / 2;
        // (each stage at least one round of its workgroups)
        if (half >= kStageMin && g % 2 == 0 && beta >= st.B[st.nst - 1] + g &&
            alive * kStageMargin + kStageSpare <= half) {
            st.B[st.nst] = beta;
            st.G[st.nst] = half;
            ++st.nst;
            g = half;
        }
    }
    st.B[st.nst] = nbundles;
    return st;
}

// prog: n+1 ints (zeroed here); err: the caller's sticky error word (never
// reset here: a nonzero value from an earlier launch stays visible).
template <typename T>
hipError_t launch_band2bd(T *A, int n, long lda, int b, bool exact_order, bool sigma_geom, int *prog, int *err,
                          int nwaves, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(prog, 0, sizeof(int) * (size_t)(n + 1), s);
    if (e != hipSuccess) return e;
    const int sg = sigma_geom ? 1 : 0;
    static const char *sel = getenv("BRD_S2_SCHEDULE");   // "pipe" selects the HBM-only schedule
    const bool pipe = sel && sel[0] == 'p';
    int S = 0, R = 0;
    const bool fast32 = !exact_order && b == 32;
    if (!pipe && fast32 && n >= 64 && sweeps_plan<T>(n, S, R)) {
        const int nbundles = (n - 1 + S - 1) / S;
        const dim3 block(64 * (S + 2 + kSweepWriters));
        const unsigned magic = (unsigned)((0x100000000ull + R - 1) / R);
        const bool w32 = sweep_rows_for(n) == 32;
        const void *fn = w32 ? (const void *)k_sweeps<T, 32> : (const void *)k_sweeps<T, 16>;
        const size_t lds = sweeps_lds_bytes<T>(R, S);
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        const int cap = coresident_limit(fn, (int)block.x, lds);
        if (cap < 1) return hipErrorInvalidConfiguration;
        const int grid = std::max(1, std::min(std::min(nwaves, cap), nbundles));
        const SweepStages st = sweep_stages(n, S, nbundles, grid);
        if (w32) hipLaunchKernelGGL((k_sweeps<T, 32>), dim3(grid), block, lds, s, A, n, lda, sg, S, R, magic, prog, err, st);
        else     hipLaunchKernelGGL((k_sweeps<T, 16>), dim3(grid), block, lds, s, A, n, lda, sg, S, R, magic, prog, err, st);
        return hipGetLastError();
    }
    // exact order, and fast mode for b != 32: the one-wave-per-sweep bundle
    // kernel (k_band2bd_bundle); tiny bands: the pipe schedule
    const bool ok = exact_order ? bundle_plan<T, true>(n, b, S, R) : bundle_plan<T, false>(n, b, S, R);
    if (!pipe && ok && n >= 64) {
        const int nbundles = (n - 1 + S - 1) / S;
        const dim3 block(64 * (S + 3));
        const unsigned magic = (unsigned)((0x100000000ull + R - 1) / R);
        const void *fn = exact_order ? (const void *)k_band2bd_bundle<T, true> : (const void *)k_band2bd_bundle<T, false>;
        const size_t lds = exact_order ? bundle_lds_bytes<T, true>(b, S, R) : bundle_lds_bytes<T, false>(b, S, R);
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        const int cap = coresident_limit(fn, (int)block.x, lds);
        if (cap < 1) return hipErrorInvalidConfiguration;
        const int grid = std::max(1, std::min(std::min(nwaves, cap), nbundles));
        if (exact_order)
            hipLaunchKernelGGL((k_band2bd_bundle<T, true>), dim3(grid), block, lds, s, A, n, lda, b, sg, S, R, magic, prog, err);
        else
            hipLaunchKernelGGL((k_band2bd_bundle<T, false>), dim3(grid), block, lds, s, A, n, lda, b, sg, S, R, magic, prog, err);
        return hipGetLastError();
    }
    const void *pfn = exact_order ? (const void *)k_band2bd_pipe<T, true> : (const void *)k_band2bd_pipe<T, false>;
    const int cap = coresident_limit(pfn, 64, 0);
    if (cap < 1) return hipErrorInvalidConfiguration;
    const int grid = std::max(1, std::min(std::min(nwaves, cap), n - 1));
    if (exact_order)
        hipLaunchKernelGGL((k_band2bd_pipe<T, true>), dim3(grid), dim3(64), 0, s, A, n, n, lda, b, sg, prog, err);
    else
        hipLaunchKernelGGL((k_band2bd_pipe<T, false>), dim3(grid), dim3(64), 0, s, A, n, n, lda, b, sg, prog, err);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_extract_bidiag(const T *A, int n, long lda, T *d, T *e, hipStream_t s)
{
    hipLaunchKernelGGL((k_extract<T>), dim3((n + 255) / 256), dim3(256), 0, s, A, n, lda, d, e);
    return hipGetLastError();
}

template hipError_t launch_band2bd<double>(double *, int, long, int, bool, bool, int *, int *, int, hipStream_t);
template hipError_t launch_band2bd<float>(float *, int, long, int, bool, bool, int *, int *, int, hipStream_t);
template hipError_t launch_extract_bidiag<double>(const double *, int, long, double *, double *, hipStream_t);
template hipError_t launch_extract_bidiag<float>(const float *, int, long, float *, float *, hipStream_t);

}  // namespace brd
