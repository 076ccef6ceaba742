// Integration check: INTEGRATION.md's C++ shim compiled against the
// REFERENCE's own boundary type.  `make -C oracle ref` builds this file with
// -I/root/reference, so `Matrix` below is csc586::gpu::Matrix<float> from the
// reference's matrix_gpu.h where it lies (never copied), and links it to
// libbrd_hip.so through include/brd.h; the binary goes to oracle/_ref/ (built
// in the dev container, run on the GPU box by tests/test_cli.py).
//
// It replaces the body of csc586::gpu::cuda_brd_p1 (svd_cuda_2.cu:1117) with
// the INTEGRATION.md shim, calls it through the benchmark's function-pointer
// shape Matrix<T>(*)(Matrix<T>&, const size_t) (svd_cuda_2.cu:1387,
// timing.h:55), and reports the reference's own check metrics
// (Matrix::mse, matrix_gpu.h:438) against the fixtures like `check`
// (svd_cuda_2.cu:1296-1347), with the band -> bidiagonal sweep of
// INTEGRATION.md as stage 2.
//
// usage: ref_shim_check <data dir> <N>   (float fixtures test/band/bidiagonal_float_N_N.bin)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "matrix_gpu.h"   // the reference's boundary type (matrix_gpu.h:79)
#include "brd.h"

namespace csc586 {
namespace gpu {

// --- INTEGRATION.md, "C++ shim in the reference tree" ---------------------
Matrix<float> cuda_brd_p1(Matrix<float> &A, size_t const b_size) {
    const int m = (int)A.nrows, n = (int)A.ncols;             // public members, matrix_gpu.h:84
    auto flat = A.flatten();                                   // 1 x (m n), row-major, matrix_gpu.h:223
    const int rc = brd_ge2band_f32(flat[0].data(), m, n, n, (int)b_size, 1, 0);
    if (rc != BRD_OK) {
        std::fprintf(stderr, "brd_ge2band_f32: %s\n", brd_last_error());
        std::abort();                                          // the reference only asserts
    }
    A = flat.reshape(m, n);                                    // matrix_gpu.h:245
    return A;                                                  // CUDA-1 semantics: A mutated and returned
}

}  // namespace gpu
}  // namespace csc586

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <data dir> <N>\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    const size_t n = (size_t)std::atoi(argv[2]);
    const std::string sz = std::to_string(n) + "_" + std::to_string(n) + ".bin";
    const size_t band_size = 4;   // the reference's check band (svd_cuda_2.cu:1300)

    csc586::gpu::Matrix<float> A(n, n);
    A.read(dir + "/test_float_" + sz);
    csc586::gpu::Matrix<float> (*brd_p1)(csc586::gpu::Matrix<float> &, const size_t) = csc586::gpu::cuda_brd_p1;
    csc586::gpu::Matrix<float> B = brd_p1(A, band_size);

    csc586::gpu::Matrix<float> band_ref(n, n);
    band_ref.read(dir + "/band_float_" + sz);
    std::printf("MSE of Band Reduction: %.9g\n", (double)B.mse(band_ref, band_size));

    // --- stage 2 where check runs it (svd_cuda_2.cu:1332) ---
    auto flat = B.flatten();
    std::vector<float> d(n), e(n - 1);
    if (brd_band2bd_f32(flat[0].data(), (int)n, (int)n, (int)band_size, d.data(), e.data(), 0) != BRD_OK) {
        std::fprintf(stderr, "brd_band2bd_f32: %s\n", brd_last_error());
        std::abort();
    }
    B = flat.reshape(n, n);
    csc586::gpu::Matrix<float> bd_ref(n, n);
    bd_ref.read(dir + "/bidiagonal_float_" + sz);
    std::printf("MSE of Bidiagonal Reduction: %.9g\n", (double)B.mse(bd_ref, 2));
    return 0;
}
