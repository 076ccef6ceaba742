// svd_gpu -- command-line front end with the reference's grammar
// (svd_cuda_2.cu:1251-1258, :1296-1434; README.md:77-83), on the MI355X library.
//
//   svd_gpu check <64|512|1024> [--dtype f32|f64] [--data-dir DIR]
//       Reads test_<T>_<N>_<N>.bin, runs stage 1 with band 4 (the reference's
//       check band, svd_cuda_2.cu:1300) and stage 2, and prints the reference's
//       band metric (Matrix::mse, matrix_gpu.h:438) against band_<T>_<N>_<N>.bin
//       and bidiagonal_<T>_<N>_<N>.bin when those fixtures are present.
//       Unlike the reference, stage 2 is the band->bidiagonal sweep whose output
//       the bidiagonal fixtures hold (the reference's check runs a one-stage GK
//       reduction there and never matches them).
//   svd_gpu benchmark <step> <nsteps> <ninst> <b> [--dtype f32|f64] [--csv PATH]
//       N = k*step for k = 1..nsteps, ninst matrices uniform in [0,5) each;
//       prints "N = <n> | <sec> sec" per size (the reference times the band
//       reduction, svd_cuda_2.cu:1397) and writes the reference's 2-line CSV
//       (svd_cuda_2.cu:1407-1426: the N values, then the stage-1 seconds, ", "
//       separated, no trailing newline) for its plotting notebook.  Stage 2 is
//       timed too: printed on the same line and written in the same 2-line
//       format to <csv stem>_stage2.csv.
//   svd_gpu svd <N> [--dtype f32|f64] [--band B] [--host-values]
//       Singular values of an N x N matrix uniform in [0,5): stage 1, stage 2 with
//       the sigma-preserving geometry (BRD_SIGMA) and the bidiagonal's values
//       on the GPU (brd_bdsvd_dev_*; --host-values: the host QR brd_bdsvd_*, the
//       reference's serial::qrd step); prints the largest and smallest values
//       and the time of each step (not in the reference CLI).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "brd.h"
#include "brd_matrix.hpp"

namespace {

template <typename T> int ge2band(T *A, int n, int b);
template <> int ge2band<double>(double *A, int n, int b) { return brd_ge2band_f64(A, n, n, n, b, 1, 0); }
template <> int ge2band<float>(float *A, int n, int b) { return brd_ge2band_f32(A, n, n, n, b, 1, 0); }
template <typename T> int band2bd(T *A, int n, int b, T *d, T *e);
template <> int band2bd<double>(double *A, int n, int b, double *d, double *e) { return brd_band2bd_f64(A, n, n, b, d, e, 0); }
template <> int band2bd<float>(float *A, int n, int b, float *d, float *e) { return brd_band2bd_f32(A, n, n, b, d, e, 0); }
template <typename T> int band2bd_sigma(T *A, int n, int b, T *d, T *e);
template <> int band2bd_sigma<double>(double *A, int n, int b, double *d, double *e) {
    return brd_band2bd_f64(A, n, n, b, d, e, BRD_SIGMA);
}
template <> int band2bd_sigma<float>(float *A, int n, int b, float *d, float *e) {
    return brd_band2bd_f32(A, n, n, b, d, e, BRD_SIGMA);
}
template <typename T> int bdsvd(const T *d, const T *e, int n, T *sv);
template <> int bdsvd<double>(const double *d, const double *e, int n, double *sv) { return brd_bdsvd_f64(d, e, n, sv); }
template <> int bdsvd<float>(const float *d, const float *e, int n, float *sv) { return brd_bdsvd_f32(d, e, n, sv); }
template <typename T> int bdsvd_dev(const T *d, const T *e, int n, T *sv);
template <> int bdsvd_dev<double>(const double *d, const double *e, int n, double *sv) {
    return brd_bdsvd_dev_f64(d, e, n, sv, 0);
}
template <> int bdsvd_dev<float>(const float *d, const float *e, int n, float *sv) {
    return brd_bdsvd_dev_f32(d, e, n, sv, 0);
}
// The bidiagonal's values on the GPU from host d, e: copies in, brd_bdsvd_dev_*, copy out.
template <typename T>
int bdsvd_gpu(const T *d, const T *e, int n, T *sv) {
    T *g = nullptr;
    if (hipMalloc(&g, sizeof(T) * (3 * (size_t)n)) != hipSuccess) return BRD_ENOMEM;
    T *gd = g, *ge = g + n, *gs = g + 2 * (size_t)n;
    int rc = BRD_OK;
    if (hipMemcpy(gd, d, sizeof(T) * n, hipMemcpyHostToDevice) != hipSuccess ||
        (n > 1 && hipMemcpy(ge, e, sizeof(T) * (n - 1), hipMemcpyHostToDevice) != hipSuccess))
        rc = BRD_EHIP;
    if (!rc) rc = bdsvd_dev<T>(gd, ge, n, gs);
    if (!rc && hipMemcpy(sv, gs, sizeof(T) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = BRD_EHIP;
    (void)hipFree(g);
    return rc;
}

void die(const char *what, int rc) {
    std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, brd_last_error());
    std::exit(1);
}

template <typename T>
int check(int n, const std::string &dir, const char *tname) {
    const int band = 4;
    const std::string sz = std::to_string(n) + "_" + std::to_string(n) + ".bin";
    brd::Matrix<T> A(n, n);
    const std::string in = dir + "/test_" + tname + "_" + sz;
    std::printf("Reading file: %s\n", in.c_str());
    if (!A.read(in)) { std::fprintf(stderr, "cannot read %s\n", in.c_str()); return 1; }
    A.print();
    int rc = ge2band<T>(A.data(), n, band);
    if (rc) die("brd_ge2band", rc);
    std::printf("\n\nMI355X Test (Band):\n");
    A.print(16);
    brd::Matrix<T> ref(n, n);
    if (ref.read(dir + "/band_" + tname + "_" + sz))
        std::printf("\n\nMSE of Band Reduction: %.9g\n", A.mse(ref, band));
    else
        std::printf("\n\nband fixture not found; MSE of Band Reduction not computed\n");
    std::vector<T> d(n), e(n > 1 ? n - 1 : 1);
    rc = band2bd<T>(A.data(), n, band, d.data(), e.data());
    if (rc) die("brd_band2bd", rc);
    std::printf("\n\nMI355X Test (Bidiagonal):\n");
    A.print(10);
    if (ref.read(dir + "/bidiagonal_" + tname + "_" + sz))
        std::printf("\n\nMSE of Bidiagonal Reduction: %.9g\n", A.mse(ref, 2));
    else
        std::printf("\n\nbidiagonal fixture not found; MSE of Bidiagonal Reduction not computed\n");
    return 0;
}

// The reference's result file (svd_cuda_2.cu:1407-1426): line 1 the sizes,
// line 2 the seconds, ", " between values, no newline after the last line.
bool write_csv(const std::string &path, const std::vector<int> &xs, const std::vector<double> &ys) {
    const std::filesystem::path parent = std::filesystem::path(path).parent_path();
    std::error_code ec;
    if (!parent.empty()) std::filesystem::create_directories(parent, ec);
    std::ofstream f(path);
    if (!f) {
        std::fprintf(stderr, "cannot write %s\n", path.c_str());
        return false;
    }
    for (size_t i = 0; i < xs.size(); ++i) f << xs[i] << (i + 1 < xs.size() ? ", " : "\n");
    for (size_t i = 0; i < ys.size(); ++i) f << (float)ys[i] << (i + 1 < ys.size() ? ", " : "");
    return (bool)f;
}

template <typename T>
int benchmark(int step, int nsteps, int ninst, int b, const std::string &csv) {
    std::printf("Benchmark: MI355X two-stage bidiagonal reduction (%s)\n", sizeof(T) == 8 ? "fp64" : "fp32");
    std::printf("\tBand size: %d\n\tStep size: %d\n\tNumber of steps: %d\n\tNumber of test instances: %d\n", b, step,
                nsteps, ninst);
    std::vector<int> xs;
    std::vector<double> y1, y2;
    for (int k = 1; k <= nsteps; ++k) {
        const int n = k * step;
        double t1 = 0, t2 = 0;
        for (int r = 0; r < ninst; ++r) {
            brd::Matrix<T> A(n, n);
            A.fill(T(0), T(5), 1000003ull * n + r);
            std::vector<T> d(n), e(n);
            auto a = std::chrono::steady_clock::now();
            int rc = ge2band<T>(A.data(), n, b);
            if (rc) die("brd_ge2band", rc);
            auto m = std::chrono::steady_clock::now();
            rc = band2bd<T>(A.data(), n, b, d.data(), e.data());
            if (rc) die("brd_band2bd", rc);
            auto z = std::chrono::steady_clock::now();
            t1 += std::chrono::duration<double>(m - a).count();
            t2 += std::chrono::duration<double>(z - m).count();
        }
        t1 /= ninst;
        t2 /= ninst;
        const double gf = 8.0 / 3.0 * (double)n * n * n / (t1 + t2) / 1e9;
        std::printf("N = %d | %g sec | band -> bidiagonal %g sec | %.2f GFLOP/s two-stage (host buffers, "
                    "PCIe included)\n", n, t1, t2, gf);
        xs.push_back(n);
        y1.push_back(t1);
        y2.push_back(t2);
    }
    std::printf("Writing results to file ... %s\n", csv.c_str());
    if (!write_csv(csv, xs, y1)) return 1;
    const size_t dot = csv.rfind('.');
    const std::string csv2 = (dot == std::string::npos || dot < csv.rfind('/') + 1 ? csv : csv.substr(0, dot)) +
                             "_stage2.csv";
    if (!write_csv(csv2, xs, y2)) return 1;
    std::printf("Done.\n");
    return 0;
}

template <typename T>
int svd(int n, int b, bool host_values) {
    brd::Matrix<T> A(n, n);
    A.fill(T(0), T(5), 1000003ull * n);
    std::vector<T> d(n), e(n), sv(n);
    auto t0 = std::chrono::steady_clock::now();
    int rc = ge2band<T>(A.data(), n, b);
    if (rc) die("brd_ge2band", rc);
    auto t1 = std::chrono::steady_clock::now();
    rc = band2bd_sigma<T>(A.data(), n, b, d.data(), e.data());
    if (rc) die("brd_band2bd (BRD_SIGMA)", rc);
    auto t2 = std::chrono::steady_clock::now();
    rc = host_values ? bdsvd<T>(d.data(), e.data(), n, sv.data()) : bdsvd_gpu<T>(d.data(), e.data(), n, sv.data());
    if (rc) die(host_values ? "brd_bdsvd" : "brd_bdsvd_dev", rc);
    auto t3 = std::chrono::steady_clock::now();
    auto sec = [](auto a, auto z) { return std::chrono::duration<double>(z - a).count(); };
    std::printf("N = %d (%s, band %d): dense -> band %g sec | band -> bidiagonal %g sec | bidiagonal -> "
                "values %g sec (%s)\n", n, sizeof(T) == 8 ? "fp64" : "fp32", b, sec(t0, t1), sec(t1, t2), sec(t2, t3),
                host_values ? "host" : "GPU");
    const int k = std::min(n, 5);
    std::printf("largest :");
    for (int i = 0; i < k; ++i) std::printf(" %.12g", (double)sv[i]);
    std::printf("\nsmallest:");
    for (int i = n - k; i < n; ++i) std::printf(" %.12g", (double)sv[i]);
    std::printf("\n");
    return 0;
}

void help() {
    std::printf("Options for MI355X two-stage bidiagonal reduction\n"
                "\n(1) Run benchmark tests.\n"
                "\t>> benchmark [<int> Step size] [<int> Number of steps] [<int> Number of test instances] "
                "[<int> Band size] [--dtype f32|f64] [--csv PATH]\n"
                "\tExample: ./svd_gpu benchmark 1024 4 1 32\n"
                "\n(2) Correctness test against the reference fixtures (band size 4).\n"
                "\t>> check [64|512|1024] [--dtype f32|f64] [--data-dir DIR]\n"
                "\tExample: ./svd_gpu check 64\n"
                "\n(3) Singular values (stage 1, sigma-preserving stage 2, the bidiagonal's values on the GPU;\n"
                "\t    --host-values: the host bidiagonal QR).\n"
                "\t>> svd [<int> N] [--dtype f32|f64] [--band B] [--host-values]\n"
                "\tExample: ./svd_gpu svd 2048 --dtype f64\n");
}

}  // namespace

int main(int argc, char **argv) {
    std::string dtype = "f32", dir = getenv("BRD_DATA_DIR") ? getenv("BRD_DATA_DIR") : "data",
                csv = "data/cuda_2_benchmark.csv";
    int band = 32;
    bool host_values = false;
    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--dtype" && i + 1 < argc) dtype = argv[++i];
        else if (a == "--data-dir" && i + 1 < argc) dir = argv[++i];
        else if (a == "--csv" && i + 1 < argc) csv = argv[++i];
        else if (a == "--band" && i + 1 < argc) band = std::atoi(argv[++i]);
        else if (a == "--host-values") host_values = true;
        else pos.push_back(a);
    }
    if (pos.size() >= 2 && pos[0] == "check") {
        const int n = std::atoi(pos[1].c_str());
        return dtype == "f64" ? check<double>(n, dir, "double") : check<float>(n, dir, "float");
    }
    if (pos.size() >= 5 && pos[0] == "benchmark") {
        const int step = std::atoi(pos[1].c_str()), ns = std::atoi(pos[2].c_str()), ni = std::atoi(pos[3].c_str()),
                  b = std::atoi(pos[4].c_str());
        return dtype == "f64" ? benchmark<double>(step, ns, ni, b, csv) : benchmark<float>(step, ns, ni, b, csv);
    }
    if (pos.size() >= 2 && pos[0] == "svd") {
        const int n = std::atoi(pos[1].c_str());
        return dtype == "f64" ? svd<double>(n, band, host_values) : svd<float>(n, band, host_values);
    }
    help();
    return 0;
}
