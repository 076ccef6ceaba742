// brd_matrix.hpp -- host matrix type for the C++ side of the drop-in.
//
// Provides the subset of the reference's csc586::gpu::Matrix<T> interface
// (matrix_gpu.h:79-535) that the stage-1/stage-2 path and its CLI use, on
// contiguous row-major storage (so flatten() is free and the buffer can be
// handed to the C ABI in include/brd.h directly):
//   Matrix(m, n), Matrix(const T*, m, n), nrows, ncols, operator[](i) -> row,
//   flatten()/data(), fill(min, max), read(path), write(path), mse(B, bs),
//   print(trunc), diag(offset).
// Deliberate differences from the reference:
//   read() reads sizeof(T) per element (the reference reads sizeof(float),
//   matrix_gpu.h:489), write() truncates instead of appending, fill() takes a
//   seed instead of a fresh std::random_device per element.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

namespace brd {

template <typename T>
class Matrix {
    std::vector<T> e_;

public:
    size_t nrows = 0, ncols = 0;

    Matrix() = default;
    Matrix(size_t m, size_t n) : e_(m * n, T(0)), nrows(m), ncols(n) {}
    Matrix(const T *a, size_t m, size_t n) : e_(a, a + m * n), nrows(m), ncols(n) {}

    T *operator[](size_t i) { return e_.data() + i * ncols; }
    const T *operator[](size_t i) const { return e_.data() + i * ncols; }
    T *data() { return e_.data(); }
    const T *data() const { return e_.data(); }
    size_t size() const { return e_.size(); }

    // contiguous row-major copy, the layout of the reference's flatten() (matrix_gpu.h:223)
    std::vector<T> flatten() const { return e_; }

    void fill(T min_val, T max_val, unsigned long long seed) {
        std::mt19937_64 g(seed);
        std::uniform_real_distribution<double> d(min_val, max_val);
        for (auto &x : e_) x = (T)d(g);
    }

    std::vector<T> diag(size_t offset = 0) const {
        std::vector<T> d;
        for (size_t i = 0; i + offset < ncols && i < nrows; ++i) d.push_back((*this)[i][i + offset]);
        return d;
    }

    // raw little-endian row-major binary, no header (the reference fixture format)
    bool read(const std::string &path) {
        std::ifstream f(path, std::ios::binary);
        if (!f) return false;
        f.read(reinterpret_cast<char *>(e_.data()), (std::streamsize)(sizeof(T) * e_.size()));
        return (size_t)f.gcount() == sizeof(T) * e_.size();
    }
    bool write(const std::string &path) const {
        std::ofstream f(path, std::ios::binary | std::ios::trunc);
        if (!f) return false;
        f.write(reinterpret_cast<const char *>(e_.data()), (std::streamsize)(sizeof(T) * e_.size()));
        return (bool)f;
    }

    // The reference's band metric (matrix_gpu.h:438-453): sum over i and
    // j in [i, i+bs) of ||a_ij| - |b_ij|| / (bs * nrows); sign-insensitive.
    double mse(const Matrix &B, size_t bs) const {
        if (B.nrows != nrows || B.ncols != ncols) throw std::invalid_argument("mse: shape mismatch");
        double err = 0;
        for (size_t i = 0; i < nrows; ++i)
            for (size_t j = i; j < std::min(i + bs, ncols); ++j)
                err += std::fabs(std::fabs((double)(*this)[i][j]) - std::fabs((double)B[i][j]));
        return err / (double)(bs * nrows);
    }

    void print(size_t trunc = 16) const {
        for (size_t i = 0; i < nrows && i <= trunc; ++i) {
            if (i == trunc) { std::printf(" ...\n"); i = nrows - 1; }
            for (size_t j = 0; j < ncols && j <= trunc; ++j) {
                if (j == trunc) { std::printf(" ... "); j = ncols - 1; }
                std::printf(" %.6f ", (double)(*this)[i][j]);
            }
            std::printf("\n");
        }
    }
};

}  // namespace brd
