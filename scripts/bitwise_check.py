"""Bitwise comparison of factors across schedule options (GPU box):
python scripts/bitwise_check.py K '{"opt": v}' '{"opt": v}' ...  (the first set is the base)."""
import json, sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc

k = int(sys.argv[1])
sets = [json.loads(a) for a in sys.argv[2:]] or [{}]
A = sc.laplacian3d(k)
base = None
for o in sets:
    num = sc.Numeric(sc.Symbolic(A, **o))
    assert num.factor(A.x) == 0
    _, L = num.export()
    x = L.x.copy()
    if base is None:
        base = (o, x, L.p.copy())
        print(f"k={k} base {o}: nnz {x.size}", flush=True)
        continue
    d = np.nonzero(x != base[1])[0]
    msg = "bitwise equal" if d.size == 0 else f"{d.size} entries differ, max rel {np.max(np.abs(x[d] - base[1][d]) / np.maximum(np.abs(base[1][d]), 1e-300)):.3e}"
    if d.size:
        cols = np.searchsorted(base[2], d, side="right") - 1
        msg += f", first columns {np.unique(cols)[:5].tolist()} of {np.unique(cols).size}"
    print(f"k={k} {o} vs {base[0]}: {msg}", flush=True)
