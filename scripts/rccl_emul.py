"""Multi-rank plan through real RCCL on one GPU: every rank of an N-rank plan in this
process with its own memory, every comm step one ncclGroupStart/End of ncclSend /
ncclRecv to self on a 1-rank communicator (sc_numeric_create_dist_emulated).  Checks
the factor against the oracle and prints one JSON line per rank count.  Run under
rocprofv3 --kernel-trace to see the RCCL send/recv kernels."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
import sparsecholesky_amd as sc  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
A = sc.laplacian3d(k)
s = sc.Symbolic(A, panel_nb_outer=128, dist_cbb=64, small_front_max=32)
_, Lp, Li, Lx = oracle.chol(A)
for nranks in (2, 4, 8):
    v = sc.Numeric(s, nranks=nranks, virtual=True, rccl_self=True)
    assert v.factor(A.x) == 0
    _, L = v.export()
    err = float(np.linalg.norm(L.x - Lx) / np.linalg.norm(Lx))
    info = s.dist_plan_info(nranks)
    print(json.dumps({"k": k, "nranks": nranks, "rel_fro": err, "pattern_equal": bool(np.array_equal(L.p, Lp)),
                      "messages": int(info["n_msgs"]), "comm_steps": int(info["n_steps"])}), flush=True)
    assert err < 1e-12
