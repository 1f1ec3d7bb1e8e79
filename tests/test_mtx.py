"""MatrixMarket banner handling (reference loader
include/mtx_reader.hpp:16-62).  The fixtures under tests/golden/mtx/ are written
for this test (the README 5x5 matrix of the reference, README.md:33-37, in each
banner form, plus malformed and non-symmetric files)."""
import os

import numpy as np
import pytest

import oracle
import sparsecholesky_amd as sc

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mtx")


def load(name):
    return sc.load_matrix_market_to_csc(os.path.join(HERE, name))


@pytest.fixture(scope="module")
def readme5(known):
    r = known["readme5"]
    return sc.triplet_to_csc_matrix(r["ti"], r["tj"], r["tx"], 5)


def same(A, B):
    return (A.n_cols == B.n_cols and np.array_equal(A.p, B.p) and np.array_equal(A.i, B.i)
            and np.array_equal(A.x, B.x))


@pytest.mark.parametrize("name", ["readme5_general.mtx", "readme5_integer_hermitian.mtx"])
def test_symmetric_forms_equal_reference_input(name, readme5):
    # general: both triangles, duplicates summed, only the upper side kept (the
    # reference's swap would double every off-diagonal entry)
    assert same(load(name), readme5)


@pytest.mark.parametrize("name", ["readme5_pattern.mtx", "readme5_pattern_general.mtx"])
def test_pattern_forms(name, readme5):
    A = load(name)
    assert np.array_equal(A.p, readme5.p) and np.array_equal(A.i, readme5.i)
    assert np.all(A.x == 1.0)


def test_general_input_factors_like_symmetric(readme5):
    A = load("readme5_general.mtx")
    st, Lp, Li, Lx = oracle.chol(A)
    rs, Rp, Ri, Rx = oracle.chol(readme5)
    assert st == rs == 0
    assert np.array_equal(Lp, Rp) and np.array_equal(Li, Ri) and np.array_equal(Lx, Rx)


@pytest.mark.parametrize("name,code", [
    ("nonsym_missing_mirror.mtx", "not symmetric"),
    ("nonsym_values.mtx", "not symmetric"),
    ("skew.mtx", "not symmetric"),
    ("array.mtx", "not implemented"),
    ("out_of_range.mtx", "invalid argument"),
])
def test_rejected_inputs(name, code):
    with pytest.raises(sc.LibraryError, match=code):
        load(name)


def test_missing_file():
    with pytest.raises(sc.LibraryError, match="could not be opened"):
        load("does_not_exist.mtx")


def test_banner_without_symmetry_token(readme5, tmp_path):
    # "%%MatrixMarket matrix coordinate real" with no symmetry token: the reference
    # reads every header the same way (mtx_reader.hpp:26-27) and swaps each entry to
    # the upper triangle, so this is the symmetric form
    src = open(os.path.join(HERE, "readme5_integer_hermitian.mtx")).read().splitlines()
    body = [l for l in src[1:]]
    p = tmp_path / "nosym.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real\n" + "\n".join(body) + "\n")
    assert same(sc.load_matrix_market_to_csc(str(p)), readme5)
