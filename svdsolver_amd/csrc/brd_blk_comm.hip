// Blocked stage 1 sharded over P GPUs (brd_stage1_blk.hip, blk_ge2band_dist):
// the data-movement kernels around its collectives.  All are
// HBM-bound copies of m x 32 or n_loc x 32 panels (one read + one write per
// element, 16-byte accesses along the 32 columns of a row).
#include "brd_blk.h"

namespace brd {
namespace blk {

// the broadcast column basis V' (rows [0, M) of a [M][32] buffer) into Lw's
// column block (Lw + c 256 + 32 j, leading dimension 256)
template <typename T>
__global__ void __launch_bounds__(256) k_dist_unpack_v(const T *__restrict__ src, T *__restrict__ dst, int M) {
    typedef typename G2<T>::v2 v2;
    const long e = (long)blockIdx.x * 256 + threadIdx.x;   // one 2-element pair
    const long row = e >> 4, p = e & 15;
    if (row < M) *(v2 *)(dst + row * 256 + 2 * p) = *(const v2 *)(src + row * 32 + 2 * p);
}

// The X pass's split-K partials (part [ks][mp][32], rows [0, rows)) summed in
// fixed order into buf [rows][32] -- the all-reduce's send / receive buffer
template <typename T>
__global__ void __launch_bounds__(256) k_dist_psum(const T *__restrict__ part, int ks, long mp, int rows,
                                                   T *__restrict__ buf) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long)rows * 32) return;
    T s = part[e];
    for (int k = 1; k < ks; ++k) s += part[(long)k * mp * 32 + e];
    buf[e] = s;
}

template <typename T>
void launch_dist_unpack_v(const T *src, T *dst, int M, hipStream_t s) {
    if (M <= 0) return;
    const long pairs = (long)M * 16;
    blk_launch("s1_comm", 0.0, 32.0 * M * 2 * sizeof(T), k_dist_unpack_v<T>, dim3((unsigned)((pairs + 255) / 256)),
               dim3(256), s, src, dst, M);
}
template <typename T>
void launch_dist_psum(const T *part, int ks, long mp, int rows, T *buf, hipStream_t s) {
    if (rows <= 0) return;
    const long el = (long)rows * 32;
    blk_launch("s1_comm", 0.0, (ks + 1.0) * el * sizeof(T), k_dist_psum<T>, dim3((unsigned)((el + 255) / 256)),
               dim3(256), s, part, ks, mp, rows, buf);
}

#define BRD_INST(T)                                                                                         \
    template void launch_dist_unpack_v<T>(const T *, T *, int, hipStream_t);                                \
    template void launch_dist_psum<T>(const T *, int, long, int, T *, hipStream_t);
BRD_INST(double)
BRD_INST(float)
#undef BRD_INST

}  // namespace blk
}  // namespace brd
