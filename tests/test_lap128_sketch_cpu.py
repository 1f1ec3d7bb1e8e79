"""The 128^3 parity sketch (tests/lap128_sketch.py) checked on the host: the reduction does
not depend on how the columns are blocked, and a perturbation of one column of L is seen by
the sketches at about its relative size (TEST INFRASTRUCTURE, no GPU)."""
import numpy as np

import lap128_sketch as ls


def _diag_blocks(acc, bounds, vals):
    # L = diag(vals) in the given column blocks (CSC, one entry per column)
    for c0, c1 in zip(bounds[:-1], bounds[1:]):
        cp = np.arange(c0, c1 + 1, dtype=np.int64)
        ri = np.arange(c0, c1, dtype=np.int32)
        acc.add(c0, c1, cp, ri, vals[c0:c1])


def test_sketch_blocking_invariant_and_sensitive():
    rng = np.random.default_rng(7)
    vals = 1.0 + rng.random(ls.N)
    a = ls.Accumulator()
    _diag_blocks(a, [0, ls.CHUNK // 3, ls.N - 5000, ls.N], vals)
    b = ls.Accumulator()
    _diag_blocks(b, list(range(0, ls.N, ls.CHUNK)) + [ls.N], vals)
    ra, rb = a.result(), b.result()
    c = ls.compare(ra, rb)
    assert c["chunk_norm_rel"] < 1e-15 and c["group_norm_rel"] < 1e-15
    assert c["sketch_J_rel_fro"] < 1e-15 and c["sketch_chunk_rel_fro_max"] < 1e-13
    # one root column scaled by (1 + 1e-6): a relative change of ~1e-6 / sqrt(1024) in its group
    v2 = vals.copy()
    j = ls.N - 10
    v2[j] *= 1.0 + 1e-6
    d = ls.Accumulator()
    _diag_blocks(d, [0, ls.N], v2)
    e = ls.compare(d.result(), ra)
    assert 1e-9 < e["group_norm_rel"] < 1e-6
    assert e["sketch_J_rel_fro"] > 1e-10
