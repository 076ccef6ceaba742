// Blocked stage 1: the block's delayed rank-256 update k_blkupd (gfx950).
#include "brd_blk.h"

namespace brd {
namespace blk {

// ==========================================================================
// k_blkupd: C[r][c] -= sum_{k < 256} Lw[r][k] RwT[k][c] for r >= r0, c >= c0:
// the block's delayed rank-256 update on the matrix cores.  Workgroup tile
// 128 x 128 (4 waves of 64 x 64: 16 accumulator tiles of 16 x 16), K in
// chunks of 16 through double-buffered LDS (Lw: pair-swizzled [kp][r][2];
// RwT: [k][c] with a 144-element pitch), the C tile in the accumulators.
// ==========================================================================
template <typename T>
struct GemmLds {
    T a[2][kGKC * kGM];     // Lw tile, pair-swizzled
    T b[2][kGKC * kGBP];    // RwT tile
};

template <typename T>
__global__ void __launch_bounds__(kGT, 2) k_blkupd(GemmArgs a) {
    typedef typename G2<T>::v2 v2;
    typedef typename Mf<T>::v4 v4;
    __shared__ GemmLds<T> L;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int q = lane >> 4, l15 = lane & 15;
    const int tr = blockIdx.x / a.tiles_c, tc = blockIdx.x % a.tiles_c;
    const int r0 = tr * kGM, c0 = tc * kGM;
    const int wr = (w >> 1) * 64, wc = (w & 1) * 64;
    T *C = (T *)a.C;
    const T *Lw = (const T *)a.Lw;
    const T *RwT = (const T *)a.RwT;

    // C tile into the accumulators
    v4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int r = r0 + wr + 16 * i + Mf<T>::crow(q, g), cc = c0 + wc + 16 * j + l15;
                acc[i][j][g] = (r < a.rows && cc < a.cols) ? C[(size_t)r * a.ldc + cc] : (T)0;
            }

    // per chunk: Lw 128 x 16 (1024 granules), RwT 16 x 128 (1024 granules): 4 + 4 per thread
    auto load = [&](int k0, v2 (&ga)[4], v2 (&gb)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + kGT * i;
            const int r = e >> 3, kp = e & 7;
            const int rg = r0 + r;
            ga[i] = rg < a.rows ? *(const v2 *)(Lw + (size_t)rg * 256 + k0 + 2 * kp) : v2{(T)0, (T)0};
            const int k = e >> 6, cp = e & 63;
            const int cg = c0 + 2 * cp;
            v2 v = {(T)0, (T)0};
            if (cg < a.cols) {
                const T *p = RwT + (size_t)(k0 + k) * a.ldr + cg;
                if (cg + 1 < a.cols) v = *(const v2 *)p; else v.x = p[0];
            }
            gb[i] = v;
        }
    };
    auto stage = [&](int buf, const v2 (&ga)[4], const v2 (&gb)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + kGT * i;
            const int r = e >> 3, kp = e & 7;
            // negated: the MFMA adds A B to the C tile
            *(v2 *)&L.a[buf][2 * (kp * kGM + (r ^ kp))] = v2{-ga[i].x, -ga[i].y};
            const int k = e >> 6, cp = e & 63;
            *(v2 *)&L.b[buf][k * kGBP + 2 * cp] = gb[i];
        }
    };
    const int nc = a.K / kGKC;
    v2 ga[4], gb[4];
    load(0, ga, gb);
    for (int c = 0; c < nc; ++c) {
        stage(c & 1, ga, gb);
        lds_barrier();
        if (c + 1 < nc) load((c + 1) * kGKC, ga, gb);
#pragma unroll
        for (int s = 0; s < kGKC / 4; ++s) {
            const int k = 4 * s + q, kp = k >> 1, hf = k & 1;
            T av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wr + 16 * i + l15;
                av[i] = L.a[c & 1][2 * (kp * kGM + (r ^ kp)) + hf];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = L.b[c & 1][k * kGBP + wc + 16 * j + l15];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = Mf<T>::mma(av[i], bv[j], acc[i][j]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int r = r0 + wr + 16 * i + Mf<T>::crow(q, g), cc = c0 + wc + 16 * j + l15;
                if (r < a.rows && cc < a.cols) C[(size_t)r * a.ldc + cc] = acc[i][j][g];
            }
}


template <typename T>
void launch_k_blkupd(dim3 grid, const GemmArgs &g, hipStream_t s, double fl, double by) {
    blk_launch("s1_blkupd", fl, by, k_blkupd<T>, grid, dim3(kGT), s, g);
}
template void launch_k_blkupd<double>(dim3, const GemmArgs &, hipStream_t, double, double);
template void launch_k_blkupd<float>(dim3, const GemmArgs &, hipStream_t, double, double);

}  // namespace blk
}  // namespace brd
