"""Generates tests/golden/known_answers.json (committed).

Every value is either
  (a) a known answer held by the reference's own tests / README, transcribed
      with its file:line, or
  (b) LAPACK dpotrf output, which is what the reference's gtest compares chol()
      against (tests/test_chol.cpp:73 calls dpotrf_; here scipy's LAPACK), or
  (c) a reference output recorded by the survey run of the unmodified
      reference in the survey container.
The reference itself cannot be built in this image without stand-in headers
(cblas.h, <expected>, Eigen, pcg), so (c) is the pin for the bigger inputs.

bcsstk01.mtx and 1138_bus.mtx are the reference's data files
(data/bcsstk01/bcsstk01.mtx, data/1138_bus/1138_bus.mtx; public HB matrices).

Run: python tests/golden/make_golden.py
"""
import json
import os

import numpy as np
from scipy.linalg import lapack

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    out = {}
    # tests/test_chol.cpp:8-21 -- EliminationTree
    out["etree_pattern"] = [[0], [1], [0, 2], [3], [0, 2, 4], [0, 1, 3, 5], [0, 2, 5, 6]]
    out["etree_expected"] = [2, 5, 4, 5, 5, 6, -1]
    # tests/test_chol.cpp:38 -- ColumnReach of row 5 with w not pre-marked
    out["reach_k"] = 5
    out["reach_expected"] = [3, 1, 0, 2, 4, 5, 6]
    # tests/test_chol.cpp:59-97 -- SimplicialCholesky vs dpotrf_('L')
    A3 = np.array([[4.0, 1.0, 1.0], [1.0, 3.0, 0.0], [1.0, 0.0, 2.0]])
    c, info = lapack.dpotrf(A3, lower=1)
    assert info == 0
    out["gtest3"] = {
        "ti": [0, 0, 0, 1, 1, 2], "tj": [0, 1, 2, 1, 2, 2], "tx": [4.0, 1.0, 1.0, 3.0, 0.0, 2.0],
        "L_dpotrf_colmajor": np.tril(c).T.ravel().tolist(),  # column-major like the gtest buffer
        "tol": 1e-9,
    }
    # README.md:6-8 (input) and README.md:33-37 (L printed to 2 decimals, lower part, CSC order)
    out["readme5"] = {
        "ti": [0, 1, 2, 1, 3, 2, 3, 3, 4, 4], "tj": [0, 0, 0, 1, 1, 2, 2, 3, 3, 4],
        "tx": [5, 1, 1, 4, 1, 4, 1, 5, 1, 3],
        "Lp": [0, 3, 6, 8, 10, 11],
        "Li": [0, 1, 2, 1, 2, 3, 2, 3, 3, 4, 4],
        "Lx_2dec": [2.24, 0.45, 0.45, 1.95, -0.10, 0.51, 1.95, 0.54, 2.11, 0.47, 1.67],
        "tol": 0.0051,
    }
    # SURVEY.md 8c (reference chol() outputs) + 8a/Appendix C (symbolic, reference code)
    out["bcsstk01"] = {
        "n": 48, "nnz_A_upper": 224, "nnz_L": 877, "flops": 20151,
        "fro": 1.800918549429466e5, "sum": 9.509143040157269e5, "last_diag": 1.564520071583823e4,
        "etree_depth": 46, "ref_supernodes": 15, "ref_atree_levels": 13,
        "ref_sn_widths": {"1": 12, "2": 2, "32": 1},
    }
    out["1138_bus"] = {
        "n": 1138, "nnz_A_upper": 2596, "nnz_L": 38312, "flops": 2741254,
        "fro": 9.868639266501233e2, "sum": 5.415340469981376e1, "last_diag": 1.594360725216931,
        "etree_depth": 544, "ref_supernodes": 804, "ref_max_width": 15, "ref_atree_levels": 302,
    }
    # (k, n, nnz(A_upper), nnz(L), F, etree depth)
    out["laplacian_nd"] = [
        [8, 512, 1856, 16894, 823684, 148],
        [16, 4096, 15616, 388432, 72222454, 596],
        [24, 13824, 53568, 2327735, 942687659, 1338],
        [32, 32768, 128000, 8148387, 5716335203, 2388],
        [48, 110592, 435456, 46374041, 70667957375, 5370],
        [64, 262144, 1036288, 156926630, 414773835364, 9556],
        [128, 2097152, 8339456, 2833223743, 28447486012263, 38228],
    ]
    out["laplacian_natural_k16"] = {"nnz_L": 990991, "flops": 249087421}
    out["laplacian_fro"] = {"8": 55.42562584220, "16": 156.7673435381}
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
