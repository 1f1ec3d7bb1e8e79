// Replays the reference's gtests (evanwporter/SparseCholesky tests/test_chol.cpp)
// through the drop-in header include/sparsecholesky/chol.hpp, plus the README
// example and the reference data file.  Built and run by tests/test_cpp_api.py.
#include <sparsecholesky/chol.hpp>

#include <cmath>
#include <cstdlib>
#include <string>

#include "mini_test.hpp"

static std::string data_dir() {
    const char* d = std::getenv("SC_GOLDEN_DIR");
    return d ? d : "tests/golden";
}

// tests/test_chol.cpp:6-25
TEST(CholeskyTest, EliminationTree) {
    std::vector<std::vector<int>> pattern = {{0}, {1}, {0, 2}, {3}, {0, 2, 4}, {0, 1, 3, 5}, {0, 2, 5, 6}};
    csc_matrix<double, sym::upper> A = build_csc_matrix_from_pattern<double>(pattern);
    auto parent = etree(A);
    const std::vector<int> expected = {2, 5, 4, 5, 5, 6, -1};
    ASSERT_EQ(parent.size(), A.size());
    EXPECT_EQ(parent, expected);
}

// tests/test_chol.cpp:27-57
TEST(CholeskyTest, ColumnReach) {
    std::vector<std::vector<int>> pattern = {{0}, {1}, {0, 2}, {3}, {0, 2, 4}, {0, 1, 3, 5}, {0, 2, 5, 6}};
    const std::vector<int> expected = {3, 1, 0, 2, 4, 5, 6};
    csc_matrix<double, sym::upper> A = build_csc_matrix_from_pattern<double>(pattern);
    const auto n = A.size();
    std::vector<int> w(n, -1);
    std::vector<int> s(n);
    std::vector<double> x(n);
    auto parent = etree(A);
    auto _ = ereach(A, 5, parent, s, w, x, n);
    EXPECT_EQ(s, expected);
    _ = ereach(A, 5, parent, s, w, n);
    EXPECT_EQ(s, expected);
    (void)_;
}

// LAPACK dpotrf('L') of [[4,1,1],[1,3,0],[1,0,2]] -- what tests/test_chol.cpp:73
// computes with dpotrf_; recorded in tests/golden/known_answers.json (gtest3).
static const double kDpotrf3[9] = {2.0, 0.5, 0.5, 0.0, 1.6583123951777, -0.15075567228888181,
                                   0.0, 0.0, 1.3142574813455419};

// tests/test_chol.cpp:59-97
GPU_TEST(CholeskyTest, SimplicialCholesky) {
    int n = 3;
    std::vector<int> ti = {0, 0, 0, 1, 1, 2};
    std::vector<int> tj = {0, 1, 2, 1, 2, 2};
    std::vector<double> tx = {4.0, 1.0, 1.0, 3.0, 0.0, 2.0};
    auto A = triplet_to_csc_matrix(ti, tj, tx, n);
    auto L = chol(A);
    ASSERT_TRUE(L.has_value());
    auto result = csc_to_dense(*L);
    for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) EXPECT_NEAR(result[i + j * n], kDpotrf3[i + j * n], 1e-9);
}

// tests/test_chol.cpp:99-136 (fails in the reference; passes here)
GPU_TEST(CholeskyTest, SupernodalCholesky) {
    int n = 3;
    std::vector<int> ti = {0, 0, 0, 1, 1, 2};
    std::vector<int> tj = {0, 1, 2, 1, 2, 2};
    std::vector<double> tx = {4.0, 1.0, 1.0, 3.0, 0.0, 2.0};
    auto A = triplet_to_csc_matrix(ti, tj, tx, n);
    auto L = chol_sn(A);
    ASSERT_TRUE(L.has_value());
    auto result = csc_to_dense(*L);
    for (int j = 0; j < n; ++j)
        for (int i = j; i < n; ++i) EXPECT_NEAR(result[i + j * n], kDpotrf3[i + j * n], 1e-9);
}

// README.md:6-37 (L printed to two decimals)
GPU_TEST(Readme, FiveByFive) {
    std::vector<int> ti = {0, 1, 2, 1, 3, 2, 3, 3, 4, 4};
    std::vector<int> tj = {0, 0, 0, 1, 1, 2, 2, 3, 3, 4};
    std::vector<double> tx = {5, 1, 1, 4, 1, 4, 1, 5, 1, 3};
    const int n = 5;
    auto A = triplet_to_csc_matrix(ti, tj, tx, n);
    auto S = schol(A);
    auto L = chol(A, S).value();
    const double want[11] = {2.24, 0.45, 0.45, 1.95, -0.10, 0.51, 1.95, 0.54, 2.11, 0.47, 1.67};
    ASSERT_EQ(L.x().size(), 11u);
    for (int q = 0; q < 11; ++q) EXPECT_NEAR(L.x()[q], want[q], 0.0051);
    EXPECT_EQ(L.p(), S.p());
    EXPECT_EQ(L.i(), S.i());
#if defined(__cpp_multidimensional_subscript)
    EXPECT_NEAR((L[3, 1]), 0.51, 0.0051);
#endif
    EXPECT_NEAR(L(3, 1), 0.51, 0.0051);
}

TEST(Readme, SymbolicPattern) {
    std::vector<int> ti = {0, 1, 2, 1, 3, 2, 3, 3, 4, 4};
    std::vector<int> tj = {0, 0, 0, 1, 1, 2, 2, 3, 3, 4};
    std::vector<double> tx = {5, 1, 1, 4, 1, 4, 1, 5, 1, 3};
    auto A = triplet_to_csc_matrix(ti, tj, tx, 5);
    auto S = schol(A);
    const std::vector<int64_t> p = {0, 3, 6, 8, 10, 11};
    const std::vector<int> i = {0, 1, 2, 1, 2, 3, 2, 3, 3, 4, 4};
    EXPECT_EQ(S.p(), p);
    EXPECT_EQ(S.i(), i);
    EXPECT_TRUE(S(3, 1));
    EXPECT_TRUE(!S(4, 0));
}

// reference data file, src/main.cpp:344 + SURVEY.md 8c checksums
GPU_TEST(Data, Bcsstk01) {
    auto A = load_matrix_market_to_csc<double>(data_dir() + "/bcsstk01.mtx");
    ASSERT_EQ(A.size(), 48u);
    auto L = chol(A);
    ASSERT_TRUE(L.has_value());
    double fro = 0;
    for (double v : L->x()) fro += v * v;
    fro = std::sqrt(fro);
    EXPECT_NEAR(fro / 1.800918549429466e5, 1.0, 1e-12);
    EXPECT_EQ(L->x().size(), 877u);
}

TEST(Data, SupernodesAndAtree) {  // src/chol.cpp:42-136, SURVEY.md Appendix C
    auto A = load_matrix_market_to_csc<double>(data_dir() + "/bcsstk01.mtx");
    auto S = schol(A);
    std::vector<std::size_t> sup;
    auto sn_id = compute_supernodes(S, sup);
    EXPECT_EQ(sup.size() - 1, 15u);
    auto at = atree(S, sn_id, sup);
    EXPECT_EQ(compute_levels(at).size(), 13u);
}

GPU_TEST(Errors, NotPositiveDefinite) {  // chol.hpp:849-850
    std::vector<int> ti = {0, 0, 1};
    std::vector<int> tj = {0, 1, 1};
    std::vector<double> tx = {1.0, 2.0, 1.0};
    auto A = triplet_to_csc_matrix(ti, tj, tx, 2);
    auto L = chol(A);
    EXPECT_TRUE(!L.has_value());
    if (!L.has_value()) EXPECT_EQ(L.error(), std::string("A is not positive definite."));
}

TEST(Errors, OutOfRange) {  // chol.hpp:224
    std::vector<int> ti = {0, 1};
    std::vector<int> tj = {0, 1};
    std::vector<double> tx = {1.0, 1.0};
    auto A = triplet_to_csc_matrix(ti, tj, tx, 2);
    bool threw = false;
    try {
        A(0, 1) = 3.0;
    } catch (const std::out_of_range&) {
        threw = true;
    }
    EXPECT_TRUE(threw);
    const auto& C = A;
    EXPECT_EQ(C(0, 1), 0.0);
}

int main(int argc, char** argv) { return mini::run_all(argc, argv); }
