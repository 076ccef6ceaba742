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
// Band data are read and written with agent-coherent (sc1) accesses, so the
// same code is correct when the sweeps of one launch run on several CUs.
#include "brd_internal.h"

#include <algorithm>

namespace brd {

template <typename T>
__device__ __forceinline__ T ld_c(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_c(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Reflector of csc586::serial::householder (svd_serial.h:189-218), including
// its mixed precision (s, u1 and tau are doubles, rounded to T).
template <typename T>
struct Refl {
    T alpha;   // 1/u1 rounded to T (the scale applied to x)
    T tau;
};

template <typename T>
__device__ __forceinline__ Refl<T> refl_fast(const T *x, int L) {
    T acc = (T)0;
    for (int r = 0; r < L; ++r) acc = fma(x[r], x[r], acc);
    const T nrm = sqrt(acc);
    const double s = x[0] >= (T)0 ? -1.0 : 1.0;   // -copysign(1, x0) (x0 = -0 -> treated as +0)
    const double u1 = (double)x[0] - s * (double)nrm;
    Refl<T> h;
    h.alpha = (T)(1. / u1);
    h.tau = (T)(-s * u1 / (double)nrm);
    return h;
}

template <typename T>
__device__ __forceinline__ Refl<T> refl_exact(const T *x, int L) {
#pragma clang fp contract(off)
    T acc = (T)0;
    for (int r = 0; r < L; ++r) acc = acc + x[r] * x[r];
    const T nrm = (T)sqrt((double)acc);
    const double s = -copysign(1.0, (double)x[0]);
    const double u1 = (double)x[0] - s * (double)nrm;
    Refl<T> h;
    h.alpha = (T)(1. / u1);
    h.tau = (T)(-s * u1 / (double)nrm);
    return h;
}

// Per-wave LDS scratch.  Fast mode needs only the broadcast vector x; exact
// mode also holds w, the explicit H (<= 32 x 32) and the lane's row/column.
template <typename T, bool EXACT>
struct WaveLds {
    T x[64];
};
template <typename T>
struct WaveLds<T, true> {
    T x[64];          // reflector source vector (broadcast)
    T w[64];          // reflector (w[0] = 1)
    T H[32 * 33];     // explicit H
    T buf[64 * 33];   // the lane's row / column (dynamic indexing)
};

// ---- right window: rows [i1,i2) x cols [j1,j2); reflector from row i1 ------
template <typename T, bool EXACT>
__device__ void win_right(T *A, long lda, int i1, int i2, int j1, int j2, WaveLds<T, EXACT> &S, int lane)
{
    const int R = i2 - i1, L = j2 - j1;   // R <= 64, L <= 32
    T *rowp = A + (long)(i1 + lane) * lda + j1;
    T a[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) a[c] = (lane < R && c < L) ? ld_c(rowp + c) : (T)0;
    if (lane == 0) {
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (c < L) S.x[c] = a[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (!EXACT) {
        const Refl<T> h = refl_fast(S.x, L);
        // w_0 = 1, w_c = x_c * alpha
        T dot = a[0];
#pragma unroll
        for (int c = 1; c < 32; ++c)
            if (c < L) dot = fma(a[c], S.x[c] * h.alpha, dot);
        const T td = h.tau * dot;
        a[0] -= td;
#pragma unroll
        for (int c = 1; c < 32; ++c)
            if (c < L) a[c] = fma(-td, S.x[c] * h.alpha, a[c]);
    } else {
#pragma clang fp contract(off)
        const Refl<T> h = refl_exact(S.x, L);
        // w and explicit H (svd_serial.h:203-214), one entry per lane at a time
        for (int c = lane; c < L; c += 64) S.w[c] = (c == 0) ? (T)1. : S.x[c] * h.alpha;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // A_t <- A_t H : out[c] = sum_k a[k] H[k][c]   (matrix.h:234 order)
        for (int c = 0; c < L; ++c) {
            T acc = (T)0;
            for (int k = 0; k < L; ++k) acc += my[k] * S.H[k * 33 + c];
#pragma unroll
            for (int cc = 0; cc < 32; ++cc)
                if (cc == c) a[cc] = acc;
        }
    }
    if (lane < R) {
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (c < L) st_c(rowp + c, a[c]);
    }
}

// ---- left window: rows [i1,i2) x cols [j1,j2); reflector from column j1 ----
template <typename T, bool EXACT>
__device__ void win_left(T *A, long lda, int i1, int i2, int j1, int j2, WaveLds<T, EXACT> &S, int lane)
{
    const int R = i2 - i1, L = j2 - j1;   // R <= 32, L <= 64
    T *colp = A + (long)i1 * lda + j1 + lane;
    T a[32];
#pragma unroll
    for (int r = 0; r < 32; ++r) a[r] = (lane < L && r < R) ? ld_c(colp + (long)r * lda) : (T)0;
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (r < R) S.x[r] = a[r];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (!EXACT) {
        const Refl<T> h = refl_fast(S.x, R);
        T dot = a[0];
#pragma unroll
        for (int r = 1; r < 32; ++r)
            if (r < R) dot = fma(a[r], S.x[r] * h.alpha, dot);
        const T td = h.tau * dot;
        a[0] -= td;
#pragma unroll
        for (int r = 1; r < 32; ++r)
            if (r < R) a[r] = fma(-td, S.x[r] * h.alpha, a[r]);
    } else {
#pragma clang fp contract(off)
        const Refl<T> h = refl_exact(S.x, R);
        for (int r = lane; r < R; r += 64) S.w[r] = (r == 0) ? (T)1. : S.x[r] * h.alpha;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const T mt = -h.tau;
        for (int e = lane; e < R * R; e += 64) {
            const int r = e / R, k = e - r * R;
            T v = ((T)0 + S.w[r] * S.w[k]) * mt;
            if (r == k) v = 1 + v;
            S.H[r * 33 + k] = v;
        }
        T *my = S.buf + lane * 33;
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (r < R) my[r] = a[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // A_t <- H A_t : out[r] = sum_k H[r][k] a[k]
        for (int r = 0; r < R; ++r) {
            T acc = (T)0;
            for (int k = 0; k < R; ++k) acc += S.H[r * 33 + k] * my[k];
#pragma unroll
            for (int rr = 0; rr < 32; ++rr)
                if (rr == r) a[rr] = acc;
        }
    }
    if (lane < L) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
            if (r < R) st_c(colp + (long)r * lda, a[r]);
    }
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
    __device__ void init(int m_, int n_, int b, int i_) {
        m = m_; n = n_; bs = b + 1; i = i_;
        const int tl_j2 = min(i + bs + bs - 1, n);
        const int nbtx = (n - tl_j2) / (bs - 1);
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
};

// Pipelined sweeps.  Sweep i runs on wave i mod NW of a persistent grid and
// executes its tasks in order; task t of sweep i may start once task t+3 of
// sweep i-1 has finished (or sweep i-1 is complete).  Lag 3 is the smallest
// lag for which every pair of overlapping windows keeps the reference's
// serial order (checked exhaustively over the geometry in
// tests/test_stage2_schedule.py), so the result equals the serial sweep's --
// bit for bit in exact-order mode.
// Hand-off (MI355X_MICROARCH.md, valid forms, table row 1): every band access
// is an sc1 load/store, the producing wave drains its stores
// (s_waitcnt vmcnt(0)) before its sc1 progress-flag store, and the consuming
// wave polls that flag with sc1 loads before its own sc1 loads.
constexpr int kSpinLimit = 1 << 24;

__device__ __forceinline__ int sweep_ntask(int m, int n, int b, int i) {
    SweepIter it;
    it.init(m, n, b, i);
    return it.ntask;
}

template <typename T, bool EXACT>
__global__ void __launch_bounds__(64) k_band2bd_pipe(T *A, int m, int n, long lda, int b, int *prog,
                                                     int *err)
{
    __shared__ WaveLds<T, EXACT> S;
    const int lane = threadIdx.x;
    const int nw = gridDim.x;
    for (int i = blockIdx.x; i < n - 1; i += nw) {
        SweepIter it;
        it.init(m, n, b, i);
        const int prev_ntask = i > 0 ? sweep_ntask(m, n, b, i - 1) : 0;
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
                if (right) win_right<T, EXACT>(A, lda, wnd.i1, wnd.i2, wnd.j1, wnd.j2, S, lane);
                else       win_left<T, EXACT>(A, lda, wnd.i1, wnd.i2, wnd.j1, wnd.j2, S, lane);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (lane == 0) __hip_atomic_store(prog + i, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <typename T>
__global__ void k_extract(const T *A, int n, long lda, T *d, T *e)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = A[(long)i * lda + i];
    if (i < n - 1) e[i] = A[(long)i * lda + i + 1];
}

// prog: n ints, err: 1 int (device workspace, zeroed here).
template <typename T>
hipError_t launch_band2bd(T *A, int n, long lda, int b, bool exact_order, int *prog, int *err,
                          int nwaves, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(prog, 0, sizeof(int) * (size_t)(n + 1), s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(err, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    const int grid = std::max(1, std::min(nwaves, n - 1));
    if (exact_order)
        hipLaunchKernelGGL((k_band2bd_pipe<T, true>), dim3(grid), dim3(64), 0, s, A, n, n, lda, b, prog, err);
    else
        hipLaunchKernelGGL((k_band2bd_pipe<T, false>), dim3(grid), dim3(64), 0, s, A, n, n, lda, b, prog, err);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_extract_bidiag(const T *A, int n, long lda, T *d, T *e, hipStream_t s)
{
    hipLaunchKernelGGL((k_extract<T>), dim3((n + 255) / 256), dim3(256), 0, s, A, n, lda, d, e);
    return hipGetLastError();
}

template hipError_t launch_band2bd<double>(double *, int, long, int, bool, int *, int *, int, hipStream_t);
template hipError_t launch_band2bd<float>(float *, int, long, int, bool, int *, int *, int, hipStream_t);
template hipError_t launch_extract_bidiag<double>(const double *, int, long, double *, double *, hipStream_t);
template hipError_t launch_extract_bidiag<float>(const float *, int, long, float *, float *, hipStream_t);

}  // namespace brd
