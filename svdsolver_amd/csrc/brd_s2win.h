// Stage-2 windows on the LDS ring, b = 32, fast arithmetic (the bundle
// kernel's hot path; included by brd_stage2.hip after rsq_nr / rcp_nr /
// fast_mod).
//
// Reference: band_rd_right (svd_parallel.h:600) and band_rd_left (:617) --
// a Householder reflector formed from the window's first row (right window)
// or first column (left window), applied to the whole window only.
//
// Ring: band row r lives in slot r mod R; element (r, c) at
// d[slot(r) * P + 31 + c - r] (diagonals -31 .. 2b - 1 = 63 of row r).
//
// One wave per window.  Right window: lane q holds row i1 + q (32 elements,
// registers); left window: lane q holds column i1 + q.  Every lane reads the
// source vector as an LDS broadcast and forms the reflector's scalars itself,
// so the window is straight-line code: loads, two 32-term sums (the source's
// squared norm and a_q . x), the scalars, the rank-1 update, stores.
#pragma once

namespace brd {

template <typename T>
struct S2Ring {
    T *d;
    int P;           // row pitch (elements)
    int R;           // rows
    unsigned magic;  // ceil(2^32 / R)
    __device__ __forceinline__ int slot(int r) const { return fast_mod(r, R, magic); }
    // pointer p with p[c] = element (r, c)
    __device__ __forceinline__ T *row(int r) const { return d + slot(r) * P + 31 - r; }
};

// ---- lag-2 schedule: the deferred corner (k_sweeps) --------------------------
// Window t of sweep i+1 may start once sweep i has finished window t+2: the
// only element it shares with window t+3 of sweep i is its own bottom-right
// corner, which is never in its source row / column
// (tests/test_stage2_schedule.py::test_lag2_corner_rule_preserves_serial_order).
// So a full window defers its LAST lane (right window: its last row; left
// window: its last column), whose dot product involves the corner: that lane
// neither updates nor stores, and keeps sigma' (its a . x without the corner
// term) for the next window of the same sweep.  The next window holds the
// deferred vector as element 31 of its lanes 0..31 (right -> left: row
// r + 63 is the left window's last row; left -> right: column r' + 63 is the
// right window's last column), the deferred vector's pivot as lane 0's
// element 31 and the corner as lane 31's; once sweep i has finished window
// t+3 (the next window's own lag-2 condition) it completes the update there
// (s2_fixup) before its own reflector, in the same arithmetic as an
// undeferred lane (bitwise the result the lag-3 order gives).
template <typename T>
struct S2Fix {
    T sig;     // sigma' of the deferred lane (sum over j = 1 .. 30 of a_j x_j)
    T alpha;   // the deferring window's reflector: w_j = alpha x_j (j >= 1), w_0 = 1
    T tau;
    T x31;     // x_31 (the corner's factor)
    T xl;      // per lane l < 32: x_l of the deferring window (read with its source vector)
};

__device__ __forceinline__ double s2_readlane(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ float s2_readlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Apply the reflector of x (x[0] the pivot, every lane holds all N = 32) to
// the lane's vector a (the same arithmetic for both window kinds):
//   |x|^2 and sigma' = sum_{j=1..30} a_j x_j in four chains each,
//   sigma = sigma' + a_31 x_31, rn = 1/|x|, u1 = x0 - s |x|, alpha = 1/u1,
//   tau = -s u1 / |x|, dot = a0 + alpha sigma, a0 -= tau dot,
//   a_j -= tau dot alpha x_j.
// Returns sigma' (and the scalars in f) for a deferred lane.
// The two halves of the reflector: the partial sums over j = 0 .. 30 (they
// start as the loads land), then -- after a deferred lane's fixup has
// completed element 31 -- the rest.
template <typename T>
struct S2Sums {
    T q0, q1, q2, q3, g0, g1, g2, g3;
};
// the sums materialised here, in program order: the compiler would otherwise
// sink them below a fixup branch and wait for every load before the first FMA
// (fp32 only: N = 8192 stage 2 60.0 -> 58.0 ms; fp64 measured 73.7 -> 74.2, so
// fp64 leaves the schedule to the compiler)
template <typename T>
__device__ __forceinline__ void s2_pin(S2Sums<T> &u) {
    if constexpr (sizeof(T) == 4)
        asm volatile("" : "+v"(u.q0), "+v"(u.q1), "+v"(u.q2), "+v"(u.q3), "+v"(u.g0), "+v"(u.g1), "+v"(u.g2), "+v"(u.g3));
}
template <typename T, int N>
__device__ __forceinline__ S2Sums<T> s2_sums(const T (&a)[N], const T (&x)[N]) {
    static_assert(N == 32, "b = 32 windows");
    S2Sums<T> u{x[0] * x[0], (T)0, (T)0, (T)0, (T)0, (T)0, (T)0, (T)0};
#pragma unroll
    for (int j = 1; j < N - 1; j += 4) {
        u.q1 = fma(x[j], x[j], u.q1);
        u.g1 = fma(a[j], x[j], u.g1);
        if (j + 1 < N - 1) { u.q2 = fma(x[j + 1], x[j + 1], u.q2); u.g2 = fma(a[j + 1], x[j + 1], u.g2); }
        if (j + 2 < N - 1) { u.q3 = fma(x[j + 2], x[j + 2], u.q3); u.g3 = fma(a[j + 2], x[j + 2], u.g3); }
        if (j + 3 < N - 1) { u.q0 = fma(x[j + 3], x[j + 3], u.q0); u.g0 = fma(a[j + 3], x[j + 3], u.g0); }
    }
    return u;
}
template <typename T, int N>
__device__ __forceinline__ T s2_apply(T (&a)[N], const T (&x)[N], S2Sums<T> u, S2Fix<T> &f) {
    u.q0 = fma(x[N - 1], x[N - 1], u.q0);
    const T qq = (u.q0 + u.q1) + (u.q2 + u.q3);
    const T sigp = (u.g0 + u.g1) + (u.g2 + u.g3);
    const T sig = fma(a[N - 1], x[N - 1], sigp);
    const T rn = rsq_nr(qq);
    const T nrm = qq * rn;
    const T sgn = x[0] >= (T)0 ? (T)-1 : (T)1;
    const T u1 = fma(-sgn, nrm, x[0]);
    const T alpha = rcp_nr(u1);
    const T tau = -sgn * u1 * rn;
    // (explicit fma everywhere: s2_fixup repeats this arithmetic for a
    // deferred lane and must round exactly alike -- a contraction the compiler
    // chose differently in the two places would change the result)
    const T dot = fma(alpha, sig, a[0]);
    const T tda = (tau * dot) * alpha;
    a[0] = fma(-tau, dot, a[0]);
#pragma unroll
    for (int j = 1; j < N; ++j) a[j] = fma(-tda, x[j], a[j]);
    f.alpha = alpha;
    f.tau = tau;
    f.x31 = x[N - 1];
    return sigp;
}
template <typename T, int N>
__device__ __forceinline__ T s2_refl(T (&a)[N], const T (&x)[N], S2Fix<T> &f) {
    return s2_apply<T, N>(a, x, s2_sums<T, N>(a, x), f);
}

// Complete the previous window's deferred vector: element 31 of lanes 0..31
// (lane 0: its pivot, lane 31: the corner, now final).  The pivot is this
// window's x[31] as loaded and the corner comes from its own broadcast load,
// so the reflector scalars and x[31]'s new value (the pivot's) need no
// cross-lane reads of the window's data; f.xl: lane l's element of the
// deferring window's source vector (registers, no LDS round trip).
template <typename T, int N>
__device__ __forceinline__ void s2_fixup(T (&a)[N], T (&x)[N], const S2Fix<T> &f, T corner, int lane) {
    const T a0 = x[N - 1];
    const T dot = fma(f.alpha, fma(corner, f.x31, f.sig), a0);
    const T tda = (f.tau * dot) * f.alpha;
    const T p = fma(-f.tau, dot, a0);   // the pivot's new value (lane 0's element 31)
    if (lane < 32) a[N - 1] = lane == 0 ? p : fma(-tda, f.xl, a[N - 1]);
    x[N - 1] = p;
}

// What a window does around its reflector (k_sweeps):
//   fix   the previous window was deferred: complete it (s2_fixup) and store
//         its 32 elements, then publish the sweep's progress (prog = t, front)
//   defer this window is deferred: its last lane keeps its vector (no
//         update, no store), fo receives the fixup data, xs the source vector
struct S2Pub {
    int *prog, *front;
    int prog_v, front_v;
    __device__ __forceinline__ void publish(int lane) const {
        asm volatile("" ::: "memory");   // LDS executes a wave's operations in order
        if (lane == 0) {
            __hip_atomic_store(front, front_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(prog, prog_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
};

// The fixup on element 31 alone (s2_fixup's arithmetic): a31 = this lane's
// element 31, x31 = the source's, before the bulk of the window -- so the
// previous window's completion is published as early as the window allows.
template <typename T>
__device__ __forceinline__ void s2_fixup1(T &a31, T &x31, const S2Fix<T> &f, T corner, int lane) {
    const T dot = fma(f.alpha, fma(corner, f.x31, f.sig), x31);
    const T tda = (f.tau * dot) * f.alpha;
    const T p = fma(-f.tau, dot, x31);
    if (lane < 32) a31 = lane == 0 ? p : fma(-tda, f.xl, a31);
    x31 = p;
}

// Right window rows [i1, i1 + nr) x cols [j1, j1 + nc) (interior: 64 x 32 at
// j1 = i1 + 32; a sweep's first window: 33 x 32 at j1 = i1 + 1); the
// reflector comes from row i1.  Lane q holds row i1 + q.  FULL: nr = 64,
// nc = 32 (no predicates).
template <typename T, bool FULL, bool LAG2>
__device__ __forceinline__ void s2_right_w1(const S2Ring<T> &rg, int i1, int j1, int nr, int nc, int lane,
                                            bool fix, const S2Fix<T> &fi, bool defer, S2Fix<T> &fo,
                                            const S2Pub &pub) {
    constexpr int N = 32;
    const bool rok = FULL || lane < nr;
    const T *px = rg.row(i1) + j1;
    T *pa = rg.row(i1 + (rok ? lane : 0)) + j1;
    T a[N], x[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const bool cok = FULL || j < nc;
        x[j] = cok ? px[j] : (T)0;
        a[j] = (cok && rok) ? pa[j] : (T)0;
    }
    if (LAG2) fo.xl = px[lane & 31];                  // (loads without branches: see s2_pin)
    const T corner = LAG2 ? rg.row(i1 + 31)[j1 + 31] : (T)0;
    S2Sums<T> u = s2_sums<T, N>(a, x);   // (elements 0 .. 30: the fixup does not touch them)
    s2_pin(u);
    if (LAG2 && fix) {   // the deferred column j1 + 31 of rows i1 .. i1 + 31
        s2_fixup1<T>(a[N - 1], x[N - 1], fi, corner, lane);
        if (lane < 32) pa[N - 1] = a[N - 1];
        pub.publish(lane);
    }
    const T sigp = s2_apply<T, N>(a, x, u, fo);
    if (LAG2 && defer) {
        fo.sig = s2_readlane(sigp, 63);
        if ((lane & 31) == 31) fo.xl = x[N - 1];   // (the fixup above may have changed it)
    }
    if (rok && !(LAG2 && defer && lane == 63)) {
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (FULL || j < nc) pa[j] = a[j];
    }
}

// Left window rows [i1, i1 + nr) x cols [j1, j1 + nc) (interior 32 x 64 at
// j1 = i1); the reflector comes from column j1.  Lane q holds column j1 + q.
// Rows that do not wrap the ring sit P - 1 elements apart: one base address
// and immediate offsets.
template <typename T, bool FULL, bool LAG2>
__device__ __forceinline__ void s2_left_w1(const S2Ring<T> &rg, int i1, int j1, int nr, int nc, int lane,
                                           bool fix, const S2Fix<T> &fi, bool defer, S2Fix<T> &fo,
                                           const S2Pub &pub) {
    constexpr int N = 32;
    const bool cok = FULL || lane < nc;
    const int q = cok ? lane : 0;
    const int s0 = rg.slot(i1);
    T a[N], x[N];
    if (LAG2) fo.xl = rg.row(i1 + (lane & 31))[j1];
    auto finish = [&](T *e31, T corner, auto store) {
        S2Sums<T> u = s2_sums<T, N>(a, x);
        s2_pin(u);
        if (LAG2 && fix) {   // the deferred row i1 + 31 of columns j1 .. j1 + 31
            s2_fixup1<T>(a[N - 1], x[N - 1], fi, corner, lane);
            if (lane < 32) *e31 = a[N - 1];
            pub.publish(lane);
        }
        const T sigp = s2_apply<T, N>(a, x, u, fo);
        if (LAG2 && defer) {
            fo.sig = s2_readlane(sigp, 63);
            if ((lane & 31) == 31) fo.xl = x[N - 1];
        }
        if (cok && !(LAG2 && defer && lane == 63)) store();
    };
    if (s0 + N <= rg.R) {
        T *bx = rg.d + s0 * rg.P + 31 + (j1 - i1);   // element (i1 + j, j1) at bx[j (P - 1)]
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const bool rk = FULL || j < nr;
            x[j] = rk ? bx[j * (rg.P - 1)] : (T)0;
            a[j] = (rk && cok) ? bx[j * (rg.P - 1) + q] : (T)0;
        }
        T *b31 = bx + (N - 1) * (rg.P - 1);
        finish(b31 + q, LAG2 ? b31[31] : (T)0, [&]() {
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (FULL || j < nr) bx[j * (rg.P - 1) + q] = a[j];
        });
    } else {
        T *rows[N];
        int s = s0;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            rows[j] = rg.d + s * rg.P + 31 + (j1 - i1) - j;
            s = s + 1 == rg.R ? 0 : s + 1;
            const bool rk = FULL || j < nr;
            x[j] = rk ? rows[j][0] : (T)0;
            a[j] = (rk && cok) ? rows[j][q] : (T)0;
        }
        finish(rows[N - 1] + q, LAG2 ? rows[N - 1][31] : (T)0, [&]() {
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (FULL || j < nr) rows[j][q] = a[j];
        });
    }
}


}  // namespace brd
