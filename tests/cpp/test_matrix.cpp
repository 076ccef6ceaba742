// CPU unit test of include/brd_matrix.hpp, the C++ boundary type that stands in
// for the reference's csc586::gpu::Matrix<T> (matrix_gpu.h:79-535).  The cases
// follow the granularity the reference's own (non-compiling) Catch2 file meant
// to test -- set element, slice, matmul, transpose, add (cuda_unit_tests.cu:69-182)
// -- plus the rest of the interface.  Built and run by tests/test_matrix_type.py.
#include "brd_matrix.hpp"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

static int g_fail = 0;
#define CHECK(cond)                                                        \
    do {                                                                   \
        if (!(cond)) {                                                     \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
            ++g_fail;                                                      \
        }                                                                  \
    } while (0)

template <typename T>
static brd::Matrix<T> iota(size_t m, size_t n) {
    brd::Matrix<T> A(m, n);
    for (size_t i = 0; i < m; ++i)
        for (size_t j = 0; j < n; ++j) A[i][j] = T(10 * i + j);
    return A;
}

template <typename T>
static void run(const std::string &tmp) {
    using M = brd::Matrix<T>;
    // set element / row view
    M A = iota<T>(3, 4);
    CHECK(A.nrows == 3 && A.ncols == 4 && A.size() == 12);
    A[1][2] = T(-7);
    CHECK(A[1][2] == T(-7) && A.data()[1 * 4 + 2] == T(-7));
    std::vector<T> r1 = A[1];
    CHECK(r1.size() == 4 && r1[2] == T(-7) && r1[3] == T(13));
    A[2] = std::vector<T>{1, 2, 3, 4};
    CHECK(A[2][0] == T(1) && A[2][3] == T(4));
    CHECK(A[0].data() == A.data() && A[0].size() == 4);
    // array constructor
    const T raw[6] = {1, 2, 3, 4, 5, 6};
    M R(raw, 2, 3);
    CHECK(R[1][0] == T(4) && R[0][2] == T(3));
    // +=, -=, *=
    M B = iota<T>(3, 4), C = iota<T>(3, 4);
    B += C;
    CHECK(B[2][3] == T(46));
    B -= C;
    CHECK(B[2][3] == T(23));
    B *= T(2);
    CHECK(B[1][1] == T(22));
    // transpose
    M At = iota<T>(3, 4).transpose();
    CHECK(At.nrows == 4 && At.ncols == 3 && At[3][2] == T(23));
    // mm: [[1,2,3],[4,5,6]] x [[1,0],[0,1],[1,1]] = [[4,5],[10,11]]
    const T rb[6] = {1, 0, 0, 1, 1, 1};
    M P = R.mm(M(rb, 3, 2));
    CHECK(P.nrows == 2 && P.ncols == 2);
    CHECK(P[0][0] == T(4) && P[0][1] == T(5) && P[1][0] == T(10) && P[1][1] == T(11));
    // flatten / reshape (row-major; transpose = column-major)
    M F = R.flatten();
    CHECK(F.nrows == 1 && F.ncols == 6 && F[0][3] == T(4));
    M Ft = R.flatten(true);
    CHECK(Ft[0][1] == T(4) && Ft[0][2] == T(2));
    M Rs = F.reshape(3, 2);
    CHECK(Rs.nrows == 3 && Rs[1][0] == T(3) && Rs[2][1] == T(6));
    bool threw = false;
    try { F.reshape(4, 2); } catch (const std::invalid_argument &) { threw = true; }
    CHECK(threw);
    // slice, copy
    M S = iota<T>(5, 5).slice(1, 3, 2, 5);
    CHECK(S.nrows == 2 && S.ncols == 3 && S[0][0] == T(12) && S[1][2] == T(24));
    M S2 = iota<T>(5, 5).slice(brd::Slice{1, 3, 2, 5});
    CHECK(S2[1][1] == S[1][1]);
    M D(4, 4);
    D.copy(S, brd::Slice{0, 2, 1, 3}, brd::Slice{1, 3, 0, 2});   // S[0:2, 1:3] -> D[1:3, 0:2]
    CHECK(D[1][0] == T(13) && D[2][1] == T(24) && D[0][0] == T(0));
    M E(4, 4);
    E.copy(S, brd::Slice{2, 4, 1, 4});
    CHECK(E[2][1] == T(12) && E[3][3] == T(24));
    M G(3, 3);
    G.copy(M(raw, 2, 3));
    CHECK(G[1][2] == T(6) && G[2][2] == T(0));
    // concat
    M H = iota<T>(2, 2);
    H.row_concat(iota<T>(1, 2));
    CHECK(H.nrows == 3 && H[2][1] == T(1));
    M K = iota<T>(2, 2);
    K.col_concat(iota<T>(2, 1));
    CHECK(K.ncols == 3 && K[1][2] == T(10) && K[1][1] == T(11));
    // fill(value, Slice): rows i1..i2, cols j1..j2 only
    M Z(4, 4);
    Z.fill(T(9), brd::Slice{1, 3, 2, 4});
    CHECK(Z[1][2] == T(9) && Z[2][3] == T(9) && Z[0][2] == T(0) && Z[1][1] == T(0) && Z[3][3] == T(0));
    // fill(min, max[, seed]): in range, reproducible with a seed
    M U1(8, 8), U2(8, 8);
    U1.fill(T(0), T(5), 42);
    U2.fill(T(0), T(5), 42);
    bool same = true, inrange = true;
    for (size_t i = 0; i < 8; ++i)
        for (size_t j = 0; j < 8; ++j) {
            same &= U1[i][j] == U2[i][j];
            inrange &= U1[i][j] >= T(0) && U1[i][j] <= T(5);
        }
    CHECK(same && inrange);
    // diag, col_slice, tiles
    M Q = iota<T>(4, 4);
    std::vector<T> d0 = Q.diag(), d1 = Q.diag(1);
    CHECK(d0.size() == 4 && d0[3] == T(33) && d1.size() == 3 && d1[2] == T(23));
    std::vector<T> c = Q.col_slice(2, 1, 4);
    CHECK(c.size() == 3 && c[0] == T(12) && c[2] == T(32));
    M Tl = Q.get_tile(1, 0, 2);
    CHECK(Tl.nrows == 2 && Tl[0][0] == T(20) && Tl[1][1] == T(31));
    Q.set_tile(T(-1), 0, 1, 2);
    CHECK(Q[0][2] == T(-1) && Q[1][3] == T(-1) && Q[0][1] == T(1));
    Q.set_tile(Tl, 0, 0, 2);
    CHECK(Q[0][0] == T(20) && Q[1][1] == T(31));
    // resize keeps the leading block
    M Y = iota<T>(3, 3);
    Y.resize(2, 4);
    CHECK(Y.nrows == 2 && Y.ncols == 4 && Y[1][2] == T(12) && Y[1][3] == T(0));
    // mse (matrix_gpu.h:438): sign-insensitive over j in [i, i+bs)
    M X1 = iota<T>(3, 3), X2 = iota<T>(3, 3);
    X2 *= T(-1);
    CHECK(X1.mse(X2, 2) == 0.0);
    X2[0][1] = T(-3);   // |3| vs |1|: 2
    X2[2][0] = T(100);  // below the band: ignored
    CHECK(X1.mse(X2, 2) == 2.0 / 6.0);
    // write / read round trip (sizeof(T) per element)
    const std::string path = tmp + "/m_" + std::to_string(sizeof(T)) + ".bin";
    M W = iota<T>(5, 3);
    W[4][2] = T(0.1);
    CHECK(W.write(path));
    M Wr(5, 3);
    CHECK(Wr.read(path));
    CHECK(Wr[4][2] == T(0.1) && Wr[3][1] == T(31));
    M Big(6, 3);
    CHECK(!Big.read(path));   // short file: reported, not silently accepted
    // norm, Reflection
    CHECK(brd::norm(std::vector<T>{3, 4}) == T(5));
    brd::Reflection<T> h{M(2, 1), M(1, 2), T(2)};
    CHECK(h.w.nrows == 2 && h.w_T.ncols == 2 && h.tau == T(2));
    // const access
    const M &cq = Q;
    CHECK(cq[1][1] == T(31) && std::vector<T>(cq[1]).size() == 4);
}

int main(int argc, char **argv) {
    const std::string tmp = argc > 1 ? argv[1] : ".";
    run<float>(tmp);
    run<double>(tmp);
    if (g_fail) {
        std::printf("%d FAILED\n", g_fail);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
