"""Product host symbolic analysis (C++) vs the oracle and the reference's known answers."""
import numpy as np
import pytest

import oracle
import sparsecholesky_amd as sc


def inputs(mtx):
    yield "readme5", sc.triplet_to_csc_matrix([0, 1, 2, 1, 3, 2, 3, 3, 4, 4], [0, 0, 0, 1, 1, 2, 2, 3, 3, 4],
                                              [5, 1, 1, 4, 1, 4, 1, 5, 1, 3], 5)
    yield "bcsstk01", mtx("bcsstk01")
    yield "1138_bus", mtx("1138_bus")
    yield "lap8", sc.laplacian3d(8)
    yield "lap16", sc.laplacian3d(16)
    yield "lap12nat", sc.laplacian3d(12, nd=False)


def test_reference_helpers_match_oracle(mtx):
    for name, A in inputs(mtx):
        sy = oracle.symbolic(A)
        parent = sc.etree(A)
        assert np.array_equal(parent, sy["parent"]), name
        post = sc.post_order(parent)
        assert np.array_equal(post, sy["post"]), name
        cc = sc.col_count(A, parent, post)
        assert np.array_equal(cc, sy["colcount"]), name


def test_schol_pattern_matches_oracle(mtx):
    for name, A in inputs(mtx):
        S = sc.schol(A)
        Lp, Li, parent = oracle.schol(A)
        assert np.array_equal(S.p, Lp) and np.array_equal(S.i, Li), name
        assert np.array_equal(S.parent, parent), name


def test_symbolic_stats(mtx, known):
    for name in ("bcsstk01", "1138_bus"):
        s = sc.Symbolic(mtx(name)).stats()
        g = known[name]
        assert s["nnz_L"] == g["nnz_L"] and s["flops"] == g["flops"] and s["etree_depth"] == g["etree_depth"]
        assert s["flops_executed"] >= s["flops"]


def test_reference_supernodes_and_atree(mtx, known):  # src/chol.cpp:42-136, SURVEY App. C
    for name in ("bcsstk01", "1138_bus"):
        S = sc.schol(mtx(name))
        sn_id, sup = sc.compute_supernodes(S)
        g = known[name]
        assert len(sup) - 1 == g["ref_supernodes"]
        at = sc.atree(S, sn_id, sup)
        assert len(sc.compute_levels(at)) == g["ref_atree_levels"]
    S = sc.schol(mtx("bcsstk01"))
    _, sup = sc.compute_supernodes(S)
    w, c = np.unique(np.diff(sup), return_counts=True)
    assert {str(a): int(b) for a, b in zip(w, c)} == known["bcsstk01"]["ref_sn_widths"]
    S = sc.schol(mtx("1138_bus"))
    _, sup = sc.compute_supernodes(S)
    assert np.diff(sup).max() == known["1138_bus"]["ref_max_width"]


def test_gtest_etree_and_reach(known):  # tests/test_chol.cpp:6-57 through the product library
    A = sc.build_csc_matrix_from_pattern(known["etree_pattern"])
    parent = sc.etree(A)
    assert parent.tolist() == known["etree_expected"]
    n = A.size()
    for use_x in (True, False):
        s = np.zeros(n, dtype=np.int32)
        w = np.full(n, -1, dtype=np.int32)
        x = np.zeros(n) if use_x else None
        top = sc.ereach(A, known["reach_k"], parent, s, w, x)
        assert top == 0 and s.tolist() == known["reach_expected"]


def test_compute_levels_deepest_first():
    parent = np.array([2, 5, 4, 5, 5, 6, -1], dtype=np.int32)
    lv = sc.compute_levels(parent)
    assert lv[-1] == [6] and sorted(sum(lv, [])) == list(range(7))
    assert lv[0] == [0]  # 0 -> 2 -> 4 -> 5 -> 6 is the deepest chain


@pytest.mark.parametrize("k", [48, 64])
def test_laplacian_table_large(k, known):  # product symbolic on the bigger Appendix B rows
    row = [r for r in known["laplacian_nd"] if r[0] == k][0]
    A = sc.laplacian3d(k)
    s = sc.Symbolic(A).stats()
    assert (s["n"], s["nnz_A"], s["nnz_L"], s["flops"], s["etree_depth"]) == tuple(row[1:])


def test_options_relaxation_changes_partition():
    A = sc.laplacian3d(16)
    a = sc.Symbolic(A, relax=0).stats()
    b = sc.Symbolic(A).stats()
    assert a["n_supernodes"] == a["n_fundamental"]
    assert b["n_supernodes"] < a["n_supernodes"]
    assert a["flops_executed"] == pytest.approx(a["flops"], rel=1e-12)  # no padding without relaxation


def test_triplet_to_csc_contract():  # chol.hpp:308-369: swap to upper, sort, sum duplicates
    A = sc.triplet_to_csc_matrix([1, 0, 0, 2, 2], [0, 1, 0, 2, 0], [1.0, 2.0, 4.0, 5.0, 7.0], 3)
    assert A.p.tolist() == [0, 1, 2, 4]
    assert A.i.tolist() == [0, 0, 0, 2]
    assert A.x.tolist() == [4.0, 3.0, 7.0, 5.0]


def test_lower_entries_ignored():
    # entries with row > col are ignored (chol.hpp:392,696)
    A = sc.triplet_to_csc_matrix([0, 0, 1], [0, 1, 1], [4.0, 1.0, 3.0], 2)
    B = sc.csc_matrix(2, 2, np.array([0, 2, 4], dtype=np.int64), np.array([0, 1, 0, 1], dtype=np.int32),
                      np.array([4.0, 99.0, 1.0, 3.0]))
    assert np.array_equal(sc.etree(A), sc.etree(B))
    assert sc.Symbolic(B).nnz_L == sc.Symbolic(A).nnz_L == 3


def test_mtx_loader(mtx, known):
    A = mtx("bcsstk01")
    assert A.size() == 48 and A.capacity() == known["bcsstk01"]["nnz_A_upper"]
    assert np.all(A.i <= np.repeat(np.arange(48), np.diff(A.p)))


def test_laplacian_generator_is_permuted_stencil():
    k = 6
    A, perm = sc.laplacian3d(k, with_perm=True)
    n = k ** 3
    assert sorted(perm.tolist()) == list(range(n))
    D = sc.csc_to_dense(A)
    # undo the permutation and compare with the natural-order stencil
    N = sc.csc_to_dense(sc.laplacian3d(k, nd=False))
    assert np.array_equal(D, N[np.ix_(perm, perm)])
    assert np.allclose(np.diag(D), 6.0)


def test_invalid_input_rejected():
    A = sc.csc_matrix(2, 2, np.array([0, 1, 3], dtype=np.int64), np.array([0, 5, 1], dtype=np.int32),
                      np.array([1.0, 1.0, 1.0]))
    with pytest.raises(sc.LibraryError):
        sc.Symbolic(A)


def test_empty_and_single():
    A0 = sc.csc_matrix(0, 0, np.zeros(1, dtype=np.int64), np.zeros(0, dtype=np.int32), np.zeros(0))
    s = sc.Symbolic(A0).stats()
    assert s["n"] == 0 and s["nnz_L"] == 0 and s["n_supernodes"] == 0
    A1 = sc.triplet_to_csc_matrix([0], [0], [9.0], 1)
    s = sc.Symbolic(A1).stats()
    assert s["nnz_L"] == 1 and s["n_supernodes"] == 1


def _ordering_case(mtx, name):
    if name == "1138_bus":
        A = mtx(name)
    elif name == "lap20nat":
        A = sc.laplacian3d(20, nd=False)
    else:
        rng = np.random.default_rng(3)
        n = 400
        i = rng.integers(0, n, 2000)
        j = rng.integers(0, n, 2000)
        A = sc.triplet_to_csc_matrix(np.concatenate([np.minimum(i, j), np.arange(n)]).astype(np.int32),
                                     np.concatenate([np.maximum(i, j), np.arange(n)]).astype(np.int32),
                                     np.concatenate([-np.ones(2000), np.full(n, 50.0)]), n)
    return A


@pytest.mark.parametrize("ordering", [1, 2], ids=["nd", "amd"])
@pytest.mark.parametrize("name", ["1138_bus", "lap20nat", "random"])
def test_nd_ordering_pattern_and_fill(mtx, name, ordering):
    # the factor of P A P^T (nested dissection, or approximate minimum degree)
    # has the oracle's pattern of P A P^T and less fill than the given order
    A = _ordering_case(mtx, name)
    s = sc.Symbolic(A, ordering=ordering)
    p = s.perm()
    assert np.array_equal(np.sort(p), np.arange(A.size()))
    B = sc.permute_symmetric(A, p)
    Lp, Li = s.pattern()
    Op, Oi, _ = oracle.schol(B)
    assert np.array_equal(Lp, Op) and np.array_equal(Li, Oi)
    s0 = sc.Symbolic(A)
    assert s.nnz_L < s0.nnz_L and s.flops < s0.flops
    assert np.array_equal(s0.perm(), np.arange(A.size()))  # default: the given order


def _arrow_plus_grid(n_grid=12, n_dense=3):
    """2D 5-point grid plus n_dense rows coupled to every vertex (AMD's dense-row path)."""
    k = n_grid
    n = k * k + n_dense
    ti, tj = list(range(n)), list(range(n))
    tx = [float(n)] * n
    for x in range(k):
        for y in range(k):
            v = x * k + y
            for u in ((x + 1) * k + y if x + 1 < k else -1, v + 1 if y + 1 < k else -1):
                if u >= 0:
                    ti.append(v), tj.append(u), tx.append(-1.0)
    for d in range(n_dense):
        for v in range(k * k):
            ti.append(v), tj.append(k * k + d), tx.append(-0.01)
    return sc.triplet_to_csc_matrix(np.array(ti, np.int32), np.array(tj, np.int32), np.array(tx), n)


@pytest.mark.parametrize("case", ["1138_bus", "lap16nat", "arrow", "disconnected", "duplicates", "diag"])
def test_amd_ordering_properties(mtx, case):
    # the approximate-minimum-degree ordering (ordering = SC_ORDER_AMD): a permutation,
    # oracle pattern of P A P^T, fill no worse than the given order; dense rows ordered
    # last; isolated vertices and duplicate entries handled
    if case == "1138_bus":
        A = mtx(case)
    elif case == "lap16nat":
        A = sc.laplacian3d(16, nd=False)
    elif case == "arrow":
        A = _arrow_plus_grid()
    elif case == "disconnected":  # two grids and isolated vertices
        B = sc.laplacian3d(6, nd=False)
        n1 = B.size()
        col = np.repeat(np.arange(n1), np.diff(B.p))
        ti = np.concatenate([B.i, B.i + n1, np.arange(2 * n1, 2 * n1 + 5)]).astype(np.int32)
        tj = np.concatenate([col, col + n1, np.arange(2 * n1, 2 * n1 + 5)]).astype(np.int32)
        tx = np.concatenate([B.x, B.x, np.ones(5)])
        A = sc.triplet_to_csc_matrix(ti, tj, tx, 2 * n1 + 5)
    elif case == "duplicates":
        g = _arrow_plus_grid(8, 0)
        col = np.repeat(np.arange(g.size()), np.diff(g.p))
        A = sc.csc_matrix(g.size(), g.size(), *_dup_cols(g.p, g.i, g.x))
    else:
        A = sc.triplet_to_csc_matrix(np.arange(7, dtype=np.int32), np.arange(7, dtype=np.int32), np.ones(7), 7)
    s = sc.Symbolic(A, ordering=2)
    p = s.perm()
    n = A.size()
    assert np.array_equal(np.sort(p), np.arange(n))
    B = sc.permute_symmetric(A, p)
    Lp, Li = s.pattern()
    Op, Oi, _ = oracle.schol(B)
    assert np.array_equal(Lp, Op) and np.array_equal(Li, Oi)
    s0 = sc.Symbolic(A)
    assert s.nnz_L <= s0.nnz_L
    if case == "arrow":  # the dense rows come last
        assert set(p[-3:].tolist()) == {n - 3, n - 2, n - 1}
    if case == "1138_bus":  # a power network: minimum degree leaves almost no fill
        assert s.nnz_L < 4000 < sc.Symbolic(A, ordering=1).nnz_L


def _dup_cols(Ap, Ai, Ax):
    """Every stored entry twice (the second copy is the one the reference keeps)."""
    p = [0]
    i, x = [], []
    for j in range(len(Ap) - 1):
        for q in range(Ap[j], Ap[j + 1]):
            i += [Ai[q], Ai[q]]
            x += [Ax[q] * 0.5, Ax[q]]
        p.append(len(i))
    return np.array(p, np.int64), np.array(i, np.int32), np.array(x)


def test_ordering_value_checked():
    A = sc.laplacian3d(4)
    with pytest.raises(Exception):
        sc.Symbolic(A, ordering=7)
