// brd_matrix.hpp -- host matrix type for the C++ side of the drop-in.
//
// The public interface of the reference's csc586::gpu::Matrix<T>
// (matrix_gpu.h:79-535) together with its Slice (:40), norm (:58) and
// Reflection (:538), on ONE contiguous row-major buffer: the storage the C ABI
// (include/brd.h) reduces in place, so data() goes to brd_ge2band_* /
// brd_band2bd_* without the flatten()/reshape() copies the reference makes
// around every transfer (matrix_gpu.h:223, :245).
//
//   reference (matrix_gpu.h)                 here
//   Matrix(m, n), Matrix(const T*, m, n)     same
//   nrows, ncols (public)                    same
//   operator[](i) -> std::vector<T>&  :112   operator[](i) -> Row<T> (a view of row i:
//                                            r[j], r.data(), r.size(), begin/end,
//                                            assignment from a std::vector<T>,
//                                            conversion to std::vector<T>)
//   operator+= / -= / *=            :115-159 same
//   size, transpose, mm             :170-213 same (mm: i-k-j loop order, same sums in
//                                            the same order per element)
//   flatten(transpose), reshape     :223-257 same (1 x mn matrix / m x n matrix)
//   copy(src, s, t), copy(src, t), copy(src), row_concat, col_concat, resize
//                                   :263-331 same
//   fill(value, Slice)              :320     rows t.i1..t.i2, cols t.j1..t.j2 (the
//                                            reference fills EVERY row from column
//                                            t.i1)
//   fill(min, max)                  :336     same distribution; fill(min, max, seed)
//                                            adds a reproducible stream
//   diag, slice(4 ints), slice(Slice), get_tile, set_tile (2), col_slice
//                                   :352-434 same
//   mse(B, band_size)               :438     same metric, double accumulator
//   write, read, print              :463-533 read() takes sizeof(T) per element (the
//                                            reference reads sizeof(float), :489),
//                                            write() truncates; both report success
//   Reflection<T>{w, w_T, tau}      :538     same
// Everything else (std::vector row storage, per-element std::random_device) is
// deliberately not reproduced.
#pragma once

#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <fstream>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace brd {

// matrix_gpu.h:40
struct Slice {
    size_t i1;   // row start
    size_t i2;   // row end (exclusive)
    size_t j1;   // column start
    size_t j2;   // column end (exclusive)
    bool contains(const Slice s) const { return (s.i2 - s.i1 <= i2 - i1) && (s.j2 - s.j1 <= j2 - j1); }
};

// matrix_gpu.h:58: Euclidean norm of a vector
template <typename T>
T norm(const std::vector<T> &v) {
    return std::sqrt(std::inner_product(v.begin(), v.end(), v.begin(), T(0)));
}

// A row of a Matrix: a view into the contiguous buffer.
template <typename T>
class Row {
    using V = typename std::remove_const<T>::type;
    T *p_;
    size_t n_;

public:
    Row(T *p, size_t n) : p_(p), n_(n) {}
    T &operator[](size_t j) const { return p_[j]; }
    T &at(size_t j) const {
        if (j >= n_) throw std::out_of_range("Row::at");
        return p_[j];
    }
    T *data() const { return p_; }
    size_t size() const { return n_; }
    T *begin() const { return p_; }
    T *end() const { return p_ + n_; }
    operator std::vector<V>() const { return std::vector<V>(p_, p_ + n_); }
    Row &operator=(const std::vector<V> &v) {
        if (v.size() != n_) throw std::invalid_argument("Row: size mismatch");
        std::copy(v.begin(), v.end(), p_);
        return *this;
    }
};

template <typename T>
class Matrix {
    std::vector<T> e_;

public:
    size_t nrows = 0, ncols = 0;

    Matrix() = default;
    Matrix(size_t m, size_t n) : e_(m * n, T(0)), nrows(m), ncols(n) {}
    Matrix(const T *a, size_t m, size_t n) : e_(a, a + m * n), nrows(m), ncols(n) {}

    Row<T> operator[](size_t i) { return Row<T>(e_.data() + i * ncols, ncols); }
    Row<const T> operator[](size_t i) const { return Row<const T>(e_.data() + i * ncols, ncols); }
    T *data() { return e_.data(); }
    const T *data() const { return e_.data(); }
    size_t size() const { return nrows * ncols; }

    // ---- element-wise operators (matrix_gpu.h:115-159) ----------------------
    Matrix &operator+=(const Matrix &m) {
        same_shape(m, "operator+=");
        for (size_t k = 0; k < size(); ++k) e_[k] += m.e_[k];
        return *this;
    }
    Matrix &operator-=(const Matrix &m) {
        same_shape(m, "operator-=");
        for (size_t k = 0; k < size(); ++k) e_[k] -= m.e_[k];
        return *this;
    }
    Matrix &operator*=(const T alpha) {
        for (auto &x : e_) x *= alpha;
        return *this;
    }

    // ---- products and shape (matrix_gpu.h:176-257) --------------------------
    Matrix transpose() const {
        Matrix t(ncols, nrows);
        for (size_t i = 0; i < nrows; ++i)
            for (size_t j = 0; j < ncols; ++j) t.e_[j * nrows + i] = e_[i * ncols + j];
        return t;
    }
    // this (m x n) * M (n x p); each element summed over k in increasing order
    Matrix mm(const Matrix &M) const {
        if (ncols != M.nrows) throw std::invalid_argument("mm: inner dimensions differ");
        Matrix r(nrows, M.ncols);
        for (size_t i = 0; i < nrows; ++i)
            for (size_t k = 0; k < ncols; ++k) {
                const T a = e_[i * ncols + k];
                for (size_t j = 0; j < M.ncols; ++j) r.e_[i * M.ncols + j] += a * M.e_[k * M.ncols + j];
            }
        return r;
    }
    // 1 x (m n) copy: row-major, or column-major with transpose = true
    Matrix flatten(const bool transpose = false) const {
        Matrix f(1, size());
        if (!transpose) {
            f.e_ = e_;
        } else {
            for (size_t i = 0; i < nrows; ++i)
                for (size_t j = 0; j < ncols; ++j) f.e_[j * nrows + i] = e_[i * ncols + j];
        }
        return f;
    }
    Matrix reshape(const size_t m, const size_t n) const {
        if (m * n != size()) throw std::invalid_argument("reshape: element count differs");
        Matrix r(m, n);
        r.e_ = e_;
        return r;
    }

    // ---- copies, concatenation, fill (matrix_gpu.h:263-349) -----------------
    // rows s.i1..s.i2, cols s.j1..s.j2 of src -> this, starting at (t.i1, t.j1)
    void copy(const Matrix &src, const Slice s, const Slice t) {
        if (!t.contains(s)) throw std::invalid_argument("copy: source slice larger than target slice");
        for (size_t i = s.i1, it = t.i1; i < s.i2; ++i, ++it)
            std::copy(src.e_.begin() + (i * src.ncols + s.j1), src.e_.begin() + (i * src.ncols + s.j2),
                      e_.begin() + (it * ncols + t.j1));
    }
    void copy(const Matrix &src, const Slice t) {
        if (t.i1 + src.nrows > nrows || t.j1 + src.ncols > ncols)
            throw std::invalid_argument("copy: source does not fit at the target position");
        copy(src, Slice{0, src.nrows, 0, src.ncols}, Slice{t.i1, t.i1 + src.nrows, t.j1, t.j1 + src.ncols});
    }
    void copy(const Matrix &src) { copy(src, Slice{0, 0, 0, 0}); }
    void row_concat(const Matrix &B) {
        if (B.ncols != ncols) throw std::invalid_argument("row_concat: column counts differ");
        e_.insert(e_.end(), B.e_.begin(), B.e_.end());
        nrows += B.nrows;
    }
    void col_concat(const Matrix &B) {
        if (B.nrows != nrows) throw std::invalid_argument("col_concat: row counts differ");
        Matrix r(nrows, ncols + B.ncols);
        for (size_t i = 0; i < nrows; ++i) {
            std::copy(e_.begin() + i * ncols, e_.begin() + (i + 1) * ncols, r.e_.begin() + i * r.ncols);
            std::copy(B.e_.begin() + i * B.ncols, B.e_.begin() + (i + 1) * B.ncols, r.e_.begin() + i * r.ncols + ncols);
        }
        *this = std::move(r);
    }
    void fill(const T value, const Slice t) {
        for (size_t i = t.i1; i < std::min(t.i2, nrows); ++i)
            std::fill(e_.begin() + (i * ncols + t.j1), e_.begin() + (i * ncols + std::min(t.j2, ncols)), value);
    }
    // the reference's resize only relabels the dimensions (matrix_gpu.h:328);
    // here the buffer follows (contents of the leading rows kept)
    void resize(const size_t m, const size_t n) {
        Matrix r(m, n);
        for (size_t i = 0; i < std::min(m, nrows); ++i)
            std::copy(e_.begin() + i * ncols, e_.begin() + i * ncols + std::min(n, ncols), r.e_.begin() + i * n);
        *this = std::move(r);
    }
    void fill(const T min_val, const T max_val) { fill(min_val, max_val, std::random_device{}()); }
    void fill(T min_val, T max_val, unsigned long long seed) {
        std::mt19937_64 g(seed);
        std::uniform_real_distribution<double> d(min_val, max_val);
        for (auto &x : e_) x = (T)d(g);
    }

    // ---- views (matrix_gpu.h:352-434) -----------------------------------------
    std::vector<T> diag(size_t offset = 0) const {
        std::vector<T> d;
        for (size_t i = 0; i + offset < ncols && i < nrows; ++i) d.push_back(e_[i * ncols + i + offset]);
        return d;
    }
    Matrix slice(const size_t row_start, const size_t row_end, const size_t col_start, const size_t col_end) const {
        return slice(Slice{row_start, row_end, col_start, col_end});
    }
    Matrix slice(const Slice &s) const {
        if (s.i2 > nrows || s.j2 > ncols || s.i1 > s.i2 || s.j1 > s.j2) throw std::out_of_range("slice");
        Matrix r(s.i2 - s.i1, s.j2 - s.j1);
        for (size_t i = s.i1; i < s.i2; ++i)
            std::copy(e_.begin() + (i * ncols + s.j1), e_.begin() + (i * ncols + s.j2),
                      r.e_.begin() + (i - s.i1) * r.ncols);
        return r;
    }
    Matrix get_tile(const size_t i, const size_t j, const size_t nbt) const { return slice(tile(i, j, nbt)); }
    void set_tile(const Matrix &t, const size_t i, const size_t j, const size_t nbt) { copy(t, tile(i, j, nbt)); }
    void set_tile(const T value, const size_t i, const size_t j, const size_t nbt) { fill(value, tile(i, j, nbt)); }
    std::vector<T> col_slice(size_t j, size_t row_start, size_t row_end) const {
        if (row_end <= row_start) throw std::invalid_argument("col_slice: empty range");
        std::vector<T> c;
        for (size_t i = row_start; i < row_end; ++i) c.push_back(e_[i * ncols + j]);
        return c;
    }

    // The reference's band metric (matrix_gpu.h:438-453): sum over i and
    // j in [i, i+bs) of ||a_ij| - |b_ij|| / (bs * nrows); sign-insensitive.
    double mse(const Matrix &B, size_t bs) const {
        same_shape(B, "mse");
        double err = 0;
        for (size_t i = 0; i < nrows; ++i)
            for (size_t j = i; j < std::min(i + bs, ncols); ++j)
                err += std::fabs(std::fabs((double)e_[i * ncols + j]) - std::fabs((double)B.e_[i * ncols + j]));
        return err / (double)(bs * nrows);
    }

    // ---- I/O: raw little-endian row-major binary, no header (fixture format) ----
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

    void print(size_t trunc = 16) const {
        for (size_t i = 0; i < nrows && i <= trunc; ++i) {
            if (i == trunc) { std::printf(" ...\n"); i = nrows - 1; }
            for (size_t j = 0; j < ncols && j <= trunc; ++j) {
                if (j == trunc) { std::printf(" ... "); j = ncols - 1; }
                std::printf(" %.6f ", (double)e_[i * ncols + j]);
            }
            std::printf("\n");
        }
    }

private:
    void same_shape(const Matrix &m, const char *what) const {
        if (m.nrows != nrows || m.ncols != ncols) throw std::invalid_argument(std::string(what) + ": shape mismatch");
    }
    Slice tile(size_t i, size_t j, size_t nbt) const {
        const size_t t = nrows / nbt;
        const Slice s{i * t, i * t + t, j * t, j * t + t};
        if (s.i2 > nrows || s.j2 > ncols) throw std::out_of_range("tile out of range");
        return s;
    }
};

// matrix_gpu.h:538: Householder reflector H = I - tau w w^T
template <typename T>
struct Reflection {
    Matrix<T> w;     // Householder vector
    Matrix<T> w_T;   // its transpose
    T tau;           // scalar normaliser
};

}  // namespace brd
