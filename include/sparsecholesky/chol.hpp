// sparsecholesky/chol.hpp -- C++ drop-in for evanwporter/SparseCholesky's
// include/chol.hpp, implemented over the C ABI of libsparsecholesky_amd
// (include/sparsecholesky.h).  Same names, argument meaning and error
// behaviour as the reference; the numeric factorization runs on an MI355X.
//
// Differences a user of the reference will notice:
//   * column pointers are int64_t (the reference's int overflows past 2^31-1
//     nonzeros, chol.hpp:52,765); p() returns std::vector<int64_t>&;
//   * chol()/chol_sn() require T = double (the device path is fp64);
//   * chol_sn() is correct (the reference's is not) and
//     is the same GPU path as chol();
//   * the README's chol(A, S) form exists;
//   * operator[](i, j) needs C++23 multidimensional subscript; operator()(i, j)
//     is always available.
#pragma once

#include <algorithm>
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <variant>
#include <vector>

#if __has_include(<expected>)
#include <expected>
#endif

#include "../sparsecholesky.h"

// ---------------------------------------------------------------------------
// std::expected (C++23), or a minimal stand-in where the library lacks it
// ---------------------------------------------------------------------------
namespace sc_compat {
#if defined(__cpp_lib_expected)
using std::expected;
using std::unexpected;
#else
template <class E>
class unexpected {
public:
    explicit unexpected(E e) : e_(std::move(e)) { }
    const E& error() const { return e_; }

private:
    E e_;
};
unexpected(const char*) -> unexpected<std::string>;

template <class T, class E>
class expected {
public:
    expected(T v) : v_(std::in_place_index<0>, std::move(v)) { }
    template <class G>
    expected(unexpected<G> u) : v_(std::in_place_index<1>, E(u.error())) { }
    bool has_value() const { return v_.index() == 0; }
    explicit operator bool() const { return has_value(); }
    T& value() {
        if (!has_value()) throw std::runtime_error(error());
        return std::get<0>(v_);
    }
    const T& value() const {
        if (!has_value()) throw std::runtime_error(error());
        return std::get<0>(v_);
    }
    T& operator*() { return std::get<0>(v_); }
    const T& operator*() const { return std::get<0>(v_); }
    T* operator->() { return &std::get<0>(v_); }
    const T* operator->() const { return &std::get<0>(v_); }
    const E& error() const { return std::get<1>(v_); }

private:
    std::variant<T, E> v_;
};
#endif
}  // namespace sc_compat

// chol.hpp:26-30
enum class sym { none, upper, lower };

// chol.hpp:36
using elimination_tree = std::vector<int>;

namespace internal {
// chol.hpp:39-96
class csc_storage {
protected:
    std::size_t m_ = 0, n_ = 0, nnz_ = 0;
    std::vector<int64_t> p_;  // column pointers (n+1)
    std::vector<int> i_;      // row indices

    csc_storage() = default;
    csc_storage(std::size_t m, std::size_t n, std::size_t nnz) : m_(m), n_(n), nnz_(nnz), p_(n + 1, 0), i_(nnz) { }

public:
    std::size_t rows() const { return m_; }
    std::size_t cols() const { return n_; }
    std::size_t size() const { return n_; }
    std::size_t capacity() const { return nnz_; }
    std::vector<int64_t>& p() { return p_; }
    std::vector<int>& i() { return i_; }
    const std::vector<int64_t>& p() const { return p_; }
    const std::vector<int>& i() const { return i_; }

    // binary search of row i in column j; -1 if absent (chol.hpp:76-88)
    int64_t find_index(std::size_t i, std::size_t j) const {
        auto b = i_.begin() + p_[j], e = i_.begin() + p_[j + 1];
        auto it = std::lower_bound(b, e, static_cast<int>(i));
        return (it != e && *it == static_cast<int>(i)) ? static_cast<int64_t>(it - i_.begin()) : -1;
    }
};
}  // namespace internal

// chol.hpp:99-132
struct SChol : public internal::csc_storage {
    SChol(std::size_t n, std::size_t nnz) : internal::csc_storage(n, n, nnz) { }
    SChol() = default;
    std::vector<int> parent;  // elimination tree

    bool contains(int i, int j) const {
        if (i < j) std::swap(i, j);
        return find_index(i, j) != -1;
    }
#if defined(__cpp_multidimensional_subscript)
    bool operator[](int i, int j) const { return contains(i, j); }
#endif
    bool operator()(int i, int j) const { return contains(i, j); }
    void set_capacity(std::size_t nnz) {
        nnz_ = nnz;
        i_.resize(nnz);
    }
    std::size_t size() const { return p_.empty() ? 0 : p_.size() - 1; }
    std::size_t capacity() const { return i_.size(); }
};

// chol.hpp:134-299
template <typename T, sym S = sym::upper>
class csc_matrix : public internal::csc_storage {
    std::vector<T> x_;

    T* find_entry(std::size_t i, std::size_t j) {
        if constexpr (S == sym::upper) {
            if (j < i) std::swap(i, j);
        } else if constexpr (S == sym::lower) {
            if (i < j) std::swap(i, j);
        }
        int64_t idx = find_index(i, j);
        return idx == -1 ? nullptr : &x_[idx];
    }

public:
    csc_matrix() = default;
    csc_matrix(std::size_t m, std::size_t n, std::size_t nnz) : internal::csc_storage(m, n, nnz), x_(nnz, T {}) { }
    csc_matrix(std::size_t n, std::size_t nnz)
        requires(S != sym::none)
        : internal::csc_storage(n, n, nnz), x_(nnz, T {}) { }
    explicit csc_matrix(const SChol& s) : internal::csc_storage(s.size(), s.size(), s.capacity()), x_(s.capacity(), T {}) {
        p_ = s.p();
        i_ = s.i();
    }

    T& at(std::size_t i, std::size_t j) {
        T* p = find_entry(i, j);
        if (!p) throw std::out_of_range("Element not present in CSC structure");  // chol.hpp:224
        return *p;
    }
    T at(std::size_t i, std::size_t j) const {
        T* p = const_cast<csc_matrix*>(this)->find_entry(i, j);
        return p ? *p : T(0);  // chol.hpp:230-237
    }
#if defined(__cpp_multidimensional_subscript)
    T& operator[](std::size_t i, std::size_t j) { return at(i, j); }
    const T operator[](std::size_t i, std::size_t j) const { return at(i, j); }
#endif
    T& operator()(std::size_t i, std::size_t j) { return at(i, j); }
    T operator()(std::size_t i, std::size_t j) const { return at(i, j); }

    std::vector<T>& x() { return x_; }
    const std::vector<T>& x() const { return x_; }

    // chol.hpp:244-298
    auto transpose() const {
        constexpr sym ST = S == sym::upper ? sym::lower : (S == sym::lower ? sym::upper : sym::none);
        csc_matrix<T, ST> AT(n_, m_, nnz_);
        auto& tp = AT.p();
        auto& ti = AT.i();
        auto& tx = AT.x();
        for (std::size_t j = 0; j < n_; ++j)
            for (int64_t q = p_[j]; q < p_[j + 1]; ++q) tp[i_[q] + 1]++;
        for (std::size_t r = 0; r < m_; ++r) tp[r + 1] += tp[r];
        std::vector<int64_t> nxt(tp.begin(), tp.end() - 1);
        for (std::size_t j = 0; j < n_; ++j)
            for (int64_t q = p_[j]; q < p_[j + 1]; ++q) {
                int64_t d = nxt[i_[q]]++;
                ti[d] = static_cast<int>(j);
                tx[d] = x_[q];
            }
        return AT;
    }
};

namespace sparsecholesky_detail {
inline std::string status_message(int64_t st) {
    std::string s = sc_status_string(st);
    const char* e = sc_last_error();
    if (st < 0 && e && *e) s += std::string(" (") + e + ")";
    return s;
}

// RAII over sc_symbolic / sc_numeric
struct analysis {
    sc_symbolic* handle = nullptr;
    int64_t status = 0;
    template <typename T, sym S>
    explicit analysis(const csc_matrix<T, S>& A, const sc_options* opt = nullptr) {
        status = sc_analyze(static_cast<int64_t>(A.size()), A.p().data(), A.i().data(), opt, &handle);
    }
    ~analysis() { sc_free_symbolic(handle); }
    analysis(const analysis&) = delete;
    analysis& operator=(const analysis&) = delete;
};
}  // namespace sparsecholesky_detail

// ---------------------------------------------------------------------------
// input construction
// ---------------------------------------------------------------------------
// chol.hpp:308-369
template <typename T>
csc_matrix<T, sym::upper> triplet_to_csc_matrix(const std::vector<int>& ti, const std::vector<int>& tj,
                                                const std::vector<T>& tx, int n) {
    assert(ti.size() == tj.size() && tj.size() == tx.size());
    std::vector<double> txd(tx.begin(), tx.end());
    std::vector<int64_t> Ap(static_cast<std::size_t>(n) + 1);
    int64_t nnz = sc_triplet_to_csc(n, static_cast<int64_t>(ti.size()), ti.data(), tj.data(), txd.data(),
                                    Ap.data(), nullptr, nullptr);
    if (nnz < 0) throw std::invalid_argument("triplet_to_csc_matrix: bad triplets");
    csc_matrix<T, sym::upper> A(n, n, static_cast<std::size_t>(nnz));
    std::vector<double> Ax(static_cast<std::size_t>(nnz));
    sc_triplet_to_csc(n, static_cast<int64_t>(ti.size()), ti.data(), tj.data(), txd.data(), A.p().data(),
                      A.i().data(), Ax.data());
    std::copy(Ax.begin(), Ax.end(), A.x().begin());
    return A;
}

// chol.hpp:412-435
template <typename T>
csc_matrix<T, sym::upper> build_csc_matrix_from_pattern(const std::vector<std::vector<int>>& pattern) {
    std::vector<int> ti, tj;
    std::vector<T> tx;
    for (int i = 0; i < static_cast<int>(pattern.size()); ++i)
        for (int c : pattern[i]) {
            int r = i, cc = c;
            if (cc < r) std::swap(r, cc);
            ti.push_back(r);
            tj.push_back(cc);
            tx.push_back(T(1));
        }
    return triplet_to_csc_matrix(ti, tj, tx, static_cast<int>(pattern.size()));
}

// include/mtx_reader.hpp:16-62 (banner honoured)
template <typename T>
csc_matrix<T, sym::upper> load_matrix_market_to_csc(const std::string& filename) {
    int64_t n = 0;
    int64_t nnz = sc_read_mtx(filename.c_str(), &n, nullptr, nullptr, nullptr);
    if (nnz == SC_ERR_NOTSYM) throw std::runtime_error("Matrix in " + filename + " is not symmetric");
    if (nnz == SC_ERR_NOTIMPL) throw std::runtime_error("Unsupported MatrixMarket format in " + filename);
    if (nnz == SC_ERR_IO) throw std::runtime_error("Could not open file " + filename);
    if (nnz < 0) throw std::runtime_error("Malformed MatrixMarket file " + filename);
    csc_matrix<T, sym::upper> A(static_cast<std::size_t>(n), static_cast<std::size_t>(n),
                                static_cast<std::size_t>(nnz));
    std::vector<double> Ax(static_cast<std::size_t>(nnz));
    sc_read_mtx(filename.c_str(), &n, A.p().data(), A.i().data(), Ax.data());
    std::copy(Ax.begin(), Ax.end(), A.x().begin());
    return A;
}

// ---------------------------------------------------------------------------
// symbolic helpers
// ---------------------------------------------------------------------------
// chol.hpp:377-410
template <typename T>
elimination_tree etree(const csc_matrix<T, sym::upper>& A) {
    elimination_tree parent(A.size());
    sc_etree(static_cast<int64_t>(A.size()), A.p().data(), A.i().data(), parent.data());
    return parent;
}

// chol.hpp:466-499
inline std::vector<int> post_order(const elimination_tree& parent) {
    std::vector<int> post(parent.size());
    sc_post_order(static_cast<int64_t>(parent.size()), parent.data(), post.data());
    return post;
}

// chol.hpp:567-622 (counts as int64_t)
template <typename T, sym S>
std::vector<int64_t> col_count(const csc_matrix<T, S>& A, const std::vector<int>& parent,
                               const std::vector<int>& post) {
    std::vector<int64_t> cc(A.size());
    sc_col_count(static_cast<int64_t>(A.size()), A.p().data(), A.i().data(), parent.data(), post.data(), cc.data());
    return cc;
}

// chol.hpp:725-731: pattern of row k of L into s[top..n), scattering A(:,k) into x
template <typename T, sym S>
std::size_t ereach(const csc_matrix<T, S>& A, std::size_t k, const std::vector<int>& parent, std::vector<int>& s,
                   std::vector<int>& w, std::vector<T>& x, std::size_t top) {
    (void)top;
    std::vector<double> xd(x.begin(), x.end());
    std::vector<double> Axd(A.x().begin(), A.x().end());
    int64_t r = sc_ereach(static_cast<int64_t>(A.size()), A.p().data(), A.i().data(), Axd.data(),
                          static_cast<int64_t>(k), parent.data(), s.data(), w.data(), xd.data());
    std::copy(xd.begin(), xd.end(), x.begin());
    return static_cast<std::size_t>(r);
}

// chol.hpp:737-739: purely symbolic
template <typename T, sym S>
std::size_t ereach(const csc_matrix<T, S>& A, std::size_t k, const std::vector<int>& parent, std::vector<int>& s,
                   std::vector<int>& w, std::size_t top) {
    (void)top;
    return static_cast<std::size_t>(sc_ereach(static_cast<int64_t>(A.size()), A.p().data(), A.i().data(), nullptr,
                                              static_cast<int64_t>(k), parent.data(), s.data(), w.data(), nullptr));
}

// src/chol.cpp:7-40: levels by depth, deepest first
inline std::vector<std::vector<int>> compute_levels(const std::vector<int>& parent) {
    std::vector<int> lev(parent.size());
    int64_t nl = sc_compute_levels(static_cast<int64_t>(parent.size()), parent.data(), lev.data());
    std::vector<std::vector<int>> levels(static_cast<std::size_t>(std::max<int64_t>(nl, 0)));
    for (std::size_t j = 0; j < parent.size(); ++j) levels[lev[j]].push_back(static_cast<int>(j));
    return levels;
}

// chol.hpp:873-946
template <typename T>
SChol schol(const csc_matrix<T, sym::upper>& A) {
    sparsecholesky_detail::analysis an(A);
    if (an.status != SC_OK) throw std::invalid_argument(sparsecholesky_detail::status_message(an.status));
    const std::size_t n = A.size();
    const int64_t nnz = sc_nnz_L(an.handle);
    SChol S(n, static_cast<std::size_t>(nnz));
    sc_symbolic_pattern(an.handle, S.p().data(), S.i().data());
    S.parent.resize(n);
    sc_symbolic_etree(an.handle, S.parent.data(), nullptr);
    return S;
}

// src/chol.cpp:42-100
inline std::vector<int> compute_supernodes(const SChol& S, std::vector<std::size_t>& supernodes) {
    const std::size_t n = S.parent.size();
    std::vector<int> sn_id(n);
    std::vector<int64_t> sup(n + 1);
    int64_t ns = sc_compute_supernodes(static_cast<int64_t>(n), S.parent.data(), S.p().data(), sn_id.data(),
                                       sup.data());
    supernodes.assign(sup.begin(), sup.begin() + (ns + 1));
    return sn_id;
}

// src/chol.cpp:102-136
inline std::vector<int> atree(const SChol& S, const std::vector<int>& sn_id, const std::vector<std::size_t>& supernodes) {
    const int64_t ns = static_cast<int64_t>(supernodes.size()) - 1;
    std::vector<int64_t> sup(supernodes.begin(), supernodes.end());
    std::vector<int> sp(static_cast<std::size_t>(std::max<int64_t>(ns, 0)));
    sc_atree(static_cast<int64_t>(S.size()), S.p().data(), S.i().data(), sn_id.data(), sup.data(), ns, sp.data());
    return sp;
}

// ---------------------------------------------------------------------------
// numeric factorization (GPU)
// ---------------------------------------------------------------------------
namespace sparsecholesky_detail {
template <typename T>
sc_compat::expected<csc_matrix<T, sym::none>, std::string> factor(const csc_matrix<T, sym::upper>& A) {
    static_assert(std::is_same_v<T, double>, "the MI355X numeric path is fp64");
    analysis an(A);
    if (an.status != SC_OK) return sc_compat::unexpected<std::string>(status_message(an.status));
    sc_numeric* num = nullptr;
    int64_t st = sc_numeric_create(an.handle, -1, &num);
    if (st != SC_OK) return sc_compat::unexpected<std::string>(status_message(st));
    st = sc_factor(num, A.x().data());
    if (st > 0) {
        sc_free_numeric(num);
        return sc_compat::unexpected<std::string>("A is not positive definite.");  // chol.hpp:850
    }
    if (st < 0) {
        std::string msg = status_message(st);
        sc_free_numeric(num);
        return sc_compat::unexpected<std::string>(msg);
    }
    const std::size_t n = A.size();
    const int64_t nnz = sc_nnz_L(an.handle);
    csc_matrix<T, sym::none> L(n, n, static_cast<std::size_t>(nnz));
    st = sc_export_L(num, L.p().data(), L.i().data(), L.x().data());
    sc_free_numeric(num);
    if (st != SC_OK) return sc_compat::unexpected<std::string>(status_message(st));
    return L;
}
}  // namespace sparsecholesky_detail

// chol.hpp:749-863
template <typename T>
sc_compat::expected<csc_matrix<T, sym::none>, std::string> chol(const csc_matrix<T, sym::upper>& A) {
    return sparsecholesky_detail::factor(A);
}

// README.md:26-27: chol(A, S) with a precomputed symbolic factor (the pattern
// must be schol(A)'s; the device plan is rebuilt from A).
template <typename T>
sc_compat::expected<csc_matrix<T, sym::none>, std::string> chol(const csc_matrix<T, sym::upper>& A, const SChol& S) {
    if (S.size() != A.size()) return sc_compat::unexpected<std::string>("SChol does not match A.");
    return sparsecholesky_detail::factor(A);
}

// chol.hpp:1406-1446 (same device path; the reference's supernodal result is wrong)
template <typename T>
sc_compat::expected<csc_matrix<T, sym::none>, std::string> chol_sn(csc_matrix<T, sym::upper>& A) {
    return sparsecholesky_detail::factor(A);
}

// chol.hpp:1448-1479: column-major dense copy (mirrors symmetric storage)
template <typename T, sym S>
std::vector<T> csc_to_dense(const csc_matrix<T, S>& A) {
    const std::size_t m = A.rows(), n = A.cols();
    std::vector<T> d(m * n, T(0));
    for (std::size_t j = 0; j < n; ++j)
        for (int64_t q = A.p()[j]; q < A.p()[j + 1]; ++q) {
            const std::size_t i = static_cast<std::size_t>(A.i()[q]);
            d[i + j * m] = A.x()[q];
            if constexpr (S != sym::none)
                if (i != j) d[j + i * m] = A.x()[q];
        }
    return d;
}
