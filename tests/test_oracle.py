"""Pins the CPU oracle (oracle/refchol.c) against the reference's known answers.

The oracle restates the reference's chol() (include/chol.hpp:749-863); these
tests replay the reference's gtests (tests/test_chol.cpp) and compare with the
reference outputs recorded in SURVEY.md (tests/golden/known_answers.json).
"""
import numpy as np
import pytest
from scipy.linalg import cho_factor

import oracle
import sparsecholesky_amd as sc


def dense_lower(Lp, Li, Lx, n):
    D = np.zeros((n, n))
    cols = np.repeat(np.arange(n), np.diff(Lp))
    D[Li, cols] = Lx
    return D


def test_elimination_tree(known):  # tests/test_chol.cpp:6-25
    A = sc.build_csc_matrix_from_pattern(known["etree_pattern"])
    assert oracle.etree(A).tolist() == known["etree_expected"]


def test_column_reach(known):  # tests/test_chol.cpp:27-57 (w not pre-marked: climbs to the root)
    A = sc.build_csc_matrix_from_pattern(known["etree_pattern"])
    n = A.size()
    parent = oracle.etree(A)
    for with_x in (True, False):
        s = np.zeros(n, dtype=np.int32)
        w = np.full(n, -1, dtype=np.int32)
        top, _ = oracle.ereach(A, known["reach_k"], parent, s, w, with_x=with_x)
        assert top == 0
        assert s.tolist() == known["reach_expected"]


def test_simplicial_cholesky_vs_dpotrf(known):  # tests/test_chol.cpp:59-97
    g = known["gtest3"]
    A = sc.triplet_to_csc_matrix(g["ti"], g["tj"], g["tx"], 3)
    st, Lp, Li, Lx = oracle.chol(A)
    assert st == 0
    expected = np.array(g["L_dpotrf_colmajor"]).reshape(3, 3).T
    got = dense_lower(Lp, Li, Lx, 3)
    assert np.allclose(np.tril(got), np.tril(expected), atol=g["tol"], rtol=0)


def test_readme_example(known):  # README.md:6-37
    g = known["readme5"]
    A = sc.triplet_to_csc_matrix(g["ti"], g["tj"], g["tx"], 5)
    st, Lp, Li, Lx = oracle.chol(A)
    assert st == 0
    assert Lp.tolist() == g["Lp"] and Li.tolist() == g["Li"]
    assert np.max(np.abs(Lx - np.array(g["Lx_2dec"]))) < g["tol"]


@pytest.mark.parametrize("name", ["bcsstk01", "1138_bus"])
def test_reference_outputs(name, known, mtx):  # SURVEY.md 8c checksums of the reference chol()
    g = known[name]
    A = mtx(name)
    assert A.size() == g["n"] and A.capacity() == g["nnz_A_upper"]
    st, Lp, Li, Lx = oracle.chol(A)
    assert st == 0
    assert len(Lx) == g["nnz_L"]
    assert abs(np.linalg.norm(Lx) / g["fro"] - 1) < 1e-14
    assert abs(Lx.sum() / g["sum"] - 1) < 1e-13
    assert abs(Lx[-1] / g["last_diag"] - 1) < 1e-14
    sy = oracle.symbolic(A)
    assert sy["flops"] == g["flops"] and sy["depth"] == g["etree_depth"]
    # dense LAPACK cross-check (the gtest's own oracle is dpotrf_)
    n = A.size()
    D = sc.csc_to_dense(A)
    Ld = np.tril(cho_factor(D, lower=True)[0])
    Lo = dense_lower(Lp, Li, Lx, n)
    assert np.linalg.norm(Lo - Ld) / np.linalg.norm(Ld) < 1e-13


@pytest.mark.parametrize("k", [8, 16, 24, 32])
def test_laplacian_symbolic_table(k, known):
    row = [r for r in known["laplacian_nd"] if r[0] == k][0]
    A = sc.laplacian3d(k)
    assert A.size() == row[1] and A.capacity() == row[2]
    sy = oracle.symbolic(A)
    assert sy["nnz_L"] == row[3] and sy["flops"] == row[4] and sy["depth"] == row[5]


def test_laplacian_natural_order(known):
    A = sc.laplacian3d(16, nd=False)
    sy = oracle.symbolic(A)
    assert sy["nnz_L"] == known["laplacian_natural_k16"]["nnz_L"]
    assert sy["flops"] == known["laplacian_natural_k16"]["flops"]


@pytest.mark.parametrize("k", [8, 16])
def test_laplacian_factor_norm(k, known):
    A = sc.laplacian3d(k)
    st, Lp, Li, Lx = oracle.chol(A)
    assert st == 0
    assert abs(np.linalg.norm(Lx) / known["laplacian_fro"][str(k)] - 1) < 1e-11


def test_schol_matches_chol_pattern(mtx):
    A = mtx("1138_bus")
    Lp, Li, _ = oracle.schol(A)
    st, Lp2, Li2, _ = oracle.chol(A)
    assert np.array_equal(Lp, Lp2) and np.array_equal(Li, Li2)


def test_not_positive_definite():
    # chol.hpp:849-850: d <= 0 -> "A is not positive definite."
    A = sc.triplet_to_csc_matrix([0, 0, 1], [0, 1, 1], [1.0, 2.0, 1.0], 2)
    st, *_ = oracle.chol(A)
    assert st == 2


def test_faithful_workspace_same_result(mtx):
    A = mtx("1138_bus")
    a = oracle.chol(A, faithful_workspace=True)
    b = oracle.chol(A, faithful_workspace=False)
    assert np.array_equal(a[3], b[3])
