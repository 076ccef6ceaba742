// Stage-2 window micro-benchmark (developer tool): one wave runs the interior
// windows of a few sweeps on a band held in an LDS ring, timing each full
// window with s_memtime.  Variant 0 = the production window code
// (win_right_full / win_left_full), variant 1 = the candidate in this file.
// Prints cycles per right / left window and the max difference of the bands.
#include "../svdsolver_amd/csrc/brd_stage2.hip"

#include <cmath>
#include <cstdio>
#include <vector>

namespace brd {

// ---------------- candidate window code ------------------------------------
// every load of the window is issued before any arithmetic (sched_barrier), the
// norm and sigma = sum_{c>=1} a_c x_c accumulate together; alpha = 1/u1 and
// 1/||x|| by rcp / rsq + Newton steps.
template <int B>
__device__ __forceinline__ void refl_apply_v1(double (&a)[B], const double (&x)[B]) {
    double q[4] = {0, 0, 0, 0}, sg[4] = {0, 0, 0, 0};
    q[0] = x[0] * x[0];
#pragma unroll
    for (int c = 1; c < B; ++c) {
        q[c & 3] = fma(x[c], x[c], q[c & 3]);
        sg[c & 3] = fma(a[c], x[c], sg[c & 3]);
    }
    const double qq = (q[0] + q[1]) + (q[2] + q[3]);
    const double sigma = (sg[0] + sg[1]) + (sg[2] + sg[3]);
    const double rn = rsq_nr(qq);
    const double nrm = qq * rn;
    const double s = x[0] >= 0.0 ? -1.0 : 1.0;
    const double u1 = fma(-s, nrm, x[0]);
    const double alpha = rcp_nr(u1);
    const double tau = -s * u1 * rn;
    const double dot = fma(alpha, sigma, a[0]);
    const double td = tau * dot;
    a[0] -= td;
    const double tda = td * alpha;
#pragma unroll
    for (int c = 1; c < B; ++c) a[c] = fma(-tda, x[c], a[c]);
}
// norm first (x only), sigma while the reflector scalars are formed
template <int B>
__device__ __forceinline__ void refl_apply_v2(double (&a)[B], const double (&x)[B]) {
    double q[4] = {0, 0, 0, 0}, sg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < B; ++c) q[c & 3] = fma(x[c], x[c], q[c & 3]);
    const double qq = (q[0] + q[1]) + (q[2] + q[3]);
    const double rn = rsq_nr(qq);
#pragma unroll
    for (int c = 1; c < B; ++c) sg[c & 3] = fma(a[c], x[c], sg[c & 3]);
    const double sigma = (sg[0] + sg[1]) + (sg[2] + sg[3]);
    const double nrm = qq * rn;
    const double s = x[0] >= 0.0 ? -1.0 : 1.0;
    const double u1 = fma(-s, nrm, x[0]);
    const double alpha = rcp_nr(u1);
    const double tau = -s * u1 * rn;
    const double dot = fma(alpha, sigma, a[0]);
    const double td = tau * dot;
    a[0] -= td;
    const double tda = td * alpha;
#pragma unroll
    for (int c = 1; c < B; ++c) a[c] = fma(-tda, x[c], a[c]);
}

__device__ unsigned long long g_ph[8];
template <int B, int RV>
__device__ __forceinline__ void right_v1(const RingAcc<double> &A, int i1, int j1, int lane) {
    const double *px = A.row(i1) + j1;
    double *pa = A.row(i1 + lane) + j1;   // 2B = 64 rows: every lane
    double a[B], x[B];
#pragma unroll
    for (int c = 0; c < B; ++c) x[c] = px[c];
#pragma unroll
    for (int c = 0; c < B; ++c) a[c] = pa[c];
    __builtin_amdgcn_sched_barrier(0);
    if (RV == 1) refl_apply_v1<B>(a, x); else refl_apply_v2<B>(a, x);
#pragma unroll
    for (int c = 0; c < B; ++c) pa[c] = a[c];
}
// left window: rows [i1, i1+B) x cols [j1, j1+2B), lane = column; rows that do
// not wrap the ring sit (P-1) elements apart: one base address + immediate offsets
template <int B, int P, int RV>
__device__ __forceinline__ void left_v1(const RingAcc<double> &A, int i1, int j1, int lane) {
    const int s0 = A.slot(i1);
    double a[B], x[B];
    if (s0 + B <= A.R) {
        const double *bx = A.d + s0 * P + A.off - i1 + j1;
        double *ba = const_cast<double *>(bx) + lane;
#pragma unroll
        for (int r = 0; r < B; ++r) x[r] = bx[r * (P - 1)];
#pragma unroll
        for (int r = 0; r < B; ++r) a[r] = ba[r * (P - 1)];
        __builtin_amdgcn_sched_barrier(0);
        if (RV == 1) refl_apply_v1<B>(a, x); else refl_apply_v2<B>(a, x);
#pragma unroll
        for (int r = 0; r < B; ++r) ba[r * (P - 1)] = a[r];
    } else {
        win_left_full<double, B>(A, i1, j1, lane);
    }
}

template <typename T, int V, int B>
__device__ __forceinline__ void win_right_v(const RingAcc<T> &A, int i1, int j1, int lane) {
    if constexpr (V == 0) {
        win_right_full<T, B>(A, i1, j1, lane);
    } else if constexpr (V == 2) {
        const int r = i1 + (lane < 2 * B ? lane : 0);
        const T *px = A.row(i1) + j1;
        T *pa = A.row(r) + j1;
        T a[B], x[B];
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < B; ++c) { x[c] = px[c]; a[c] = pa[c]; }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        refl_apply_v1<B>(a, x);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (lane < 2 * B) {
#pragma unroll
            for (int c = 0; c < B; ++c) pa[c] = a[c];
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (lane == 0) { g_ph[0] += t1 - t0; g_ph[1] += t2 - t1; g_ph[2] += t3 - t2; g_ph[3] += 1; }
    } else if constexpr (V == 4) {
        double *pa = A.row(i1 + lane) + j1;
        double a[B], x[B];
#pragma unroll
        for (int c = 0; c < B; ++c) a[c] = pa[c];
#pragma unroll
        for (int c = 0; c < B; ++c)
            x[c] = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(a[c])),
                                    __builtin_amdgcn_readfirstlane(__double2loint(a[c])));
        refl_apply_v1<B>(a, x);
#pragma unroll
        for (int c = 0; c < B; ++c) pa[c] = a[c];
    } else if constexpr (V == 1) {
        right_v1<B, 1>(A, i1, j1, lane);
    } else {
        right_v1<B, 2>(A, i1, j1, lane);
    }
}
template <typename T, int V, int B>
__device__ __forceinline__ void win_left_v(const RingAcc<T> &A, int i1, int j1, int lane) {
    if constexpr (V == 0) {
        win_left_full<T, B>(A, i1, j1, lane);
    } else if constexpr (V == 2) {
        const int col = lane < 2 * B ? lane : 0;
        int slot = A.slot(i1);
        T a[B], x[B];
        T *rows[B];
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < B; ++r) {
            rows[r] = A.d + slot * A.P + A.off - (i1 + r) + j1;
            x[r] = rows[r][0];
            a[r] = rows[r][col];
            slot = slot + 1 == A.R ? 0 : slot + 1;
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        refl_apply_v1<B>(a, x);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t2 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (lane < 2 * B) {
#pragma unroll
            for (int r = 0; r < B; ++r) rows[r][col] = a[r];
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        if (lane == 0) { g_ph[4] += t1 - t0; g_ph[5] += t2 - t1; g_ph[6] += t3 - t2; g_ph[7] += 1; }
    } else if constexpr (V == 4) {
        const int s0 = A.slot(i1);
        constexpr int P = 96;
        double a[B], x[B];
        if (s0 + B <= A.R) {
            double *ba = A.d + s0 * P + A.off - i1 + j1 + lane;
#pragma unroll
            for (int r = 0; r < B; ++r) a[r] = ba[r * (P - 1)];
#pragma unroll
            for (int r = 0; r < B; ++r)
                x[r] = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(a[r])),
                                        __builtin_amdgcn_readfirstlane(__double2loint(a[r])));
            refl_apply_v1<B>(a, x);
#pragma unroll
            for (int r = 0; r < B; ++r) ba[r * (P - 1)] = a[r];
        } else {
            win_left_full<double, B>(A, i1, j1, lane);
        }
    } else if constexpr (V == 1) {
        left_v1<B, 96, 1>(A, i1, j1, lane);
    } else {
        left_v1<B, 96, 2>(A, i1, j1, lane);
    }
}

template <typename T, int V>
__global__ void __launch_bounds__(64) k_winbench(T *band, int n, int nsweeps, unsigned long long *out) {
    extern __shared__ __align__(16) unsigned char smem[];
    constexpr int B = 32;
    const int P = ring_pitch<T>(B);
    T *ring = (T *)smem;
    const int lane = threadIdx.x;
    const RingAcc<T> acc{ring, P, n, B - 1, (unsigned)((0x100000000ull + n - 1) / n)};
    for (int e = lane; e < n * P; e += 64) ring[e] = band[e];
    __syncthreads();
    unsigned long long cr = 0, cl = 0;
    int nr = 0, nl = 0;
    for (int i = 0; i < nsweeps; ++i) {
        SweepIter it;
        it.init(n, n, B, i, 0);
        for (int t = 0; t < it.ntask; ++t) {
            bool right;
            const Win w = it.task(t, right);
            if (!(w.j2 > w.j1 && w.i2 > w.i1)) continue;
            const int wr = w.i2 - w.i1, wc = w.j2 - w.j1;
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
            if (right && wr == 2 * B && wc == B) {
                win_right_v<T, V, B>(acc, w.i1, w.j1, lane);
            } else if (!right && wr == B && wc == 2 * B) {
                win_left_v<T, V, B>(acc, w.i1, w.j1, lane);
            } else {
                WaveLds<T, false> *S = nullptr;
                __shared__ WaveLds<T, false> wl;
                S = &wl;
                if (right) win_right<T, false>(acc, w.i1, w.i2, w.j1, w.j2, *S, lane);
                else       win_left<T, false>(acc, w.i1, w.i2, w.j1, w.j2, *S, lane);
                continue;
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
            if (right) { cr += t1 - t0; ++nr; } else { cl += t1 - t0; ++nl; }
        }
    }
    __syncthreads();
    for (int e = lane; e < n * P; e += 64) band[e] = ring[e];
    if (lane == 0) { out[0] = cr; out[1] = nr; out[2] = cl; out[3] = nl; }
}

}  // namespace brd

template <int V>
static void run(const std::vector<double> &h0, int n, int nsw, std::vector<double> &res) {
    const int P = brd::ring_pitch<double>(32);
    double *d; unsigned long long *o;
    (void)hipMalloc(&d, sizeof(double) * h0.size());
    (void)hipMalloc(&o, 64);
    (void)hipMemcpy(d, h0.data(), sizeof(double) * h0.size(), hipMemcpyHostToDevice);
    const size_t lds = sizeof(double) * (size_t)n * P;
    (void)hipFuncSetAttribute((const void *)brd::k_winbench<double, V>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((brd::k_winbench<double, V>), dim3(1), dim3(64), lds, 0, d, n, nsw, o);
    unsigned long long ho[4];
    (void)hipMemcpy(ho, o, 32, hipMemcpyDeviceToHost);
    res.resize(h0.size());
    (void)hipMemcpy(res.data(), d, sizeof(double) * h0.size(), hipMemcpyDeviceToHost);
    const hipError_t e = hipGetLastError();
    printf("variant %d: %s  right %.0f cyc (%llu)  left %.0f cyc (%llu)\n", V, hipGetErrorString(e),
           (double)ho[0] / ho[1], ho[1], (double)ho[2] / ho[3], ho[3]);
    (void)hipFree(d); (void)hipFree(o);
}

int main() {
    const int n = 192, b = 32, P = brd::ring_pitch<double>(b), nsw = 8;
    // ring image of a random band: row r at r*P, element (r, c) at offset c - r + b - 1
    std::vector<double> h((size_t)n * P, 0.0);
    unsigned long long s = 12345;
    for (int r = 0; r < n; ++r)
        for (int c = r; c <= std::min(n - 1, r + b); ++c) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            h[(size_t)r * P + c - r + b - 1] = 1.0 + (double)(s >> 11) / 9007199254740992.0 * 4.0;
        }
    std::vector<double> r0, r1, r2, r3;
    run<0>(h, n, nsw, r0);
    run<1>(h, n, nsw, r1);
    run<2>(h, n, nsw, r2);
    run<3>(h, n, nsw, r3);
    std::vector<double> r4;
    run<4>(h, n, nsw, r4);
    unsigned long long ph[8];
    (void)hipMemcpyFromSymbol(ph, HIP_SYMBOL(brd::g_ph), sizeof(ph));
    printf("phases right: load %.0f compute %.0f store %.0f | left: load %.0f compute %.0f store %.0f\n",
           (double)ph[0] / ph[3], (double)ph[1] / ph[3], (double)ph[2] / ph[3], (double)ph[4] / ph[7], (double)ph[5] / ph[7], (double)ph[6] / ph[7]);
    double md = 0, mx = 0;
    double md3 = 0;
    for (size_t i = 0; i < r0.size(); ++i) {
        md = std::max(md, std::fabs(r0[i] - r1[i]));
        md3 = std::max(md3, std::fabs(r0[i] - r3[i]));
        mx = std::max(mx, std::fabs(r0[i]));
    }
    printf("max |v0 - v3| = %.3e\n", md3);
    md3 = 0;
    for (size_t i = 0; i < r0.size(); ++i) md3 = std::max(md3, std::fabs(r0[i] - r4[i]));
    printf("max |v0 - v4| = %.3e\n", md3);
    printf("max |v0 - v1| = %.3e (max |v0| = %.3e)\n", md, mx);
    return 0;
}
