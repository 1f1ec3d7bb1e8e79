import sys, os, numpy as np
sys.path.insert(0, "/root/repo")
import sparsecholesky_amd as sc, oracle
def run(name, A, **kw):
    st,Lp,Li,Lx = oracle.chol(A)
    r = sc.chol(A, **kw)
    if not r.has_value():
        print(name, "GPU error", r.error()); return
    L = r.value()
    same = np.array_equal(L.p, Lp) and np.array_equal(L.i, Li)
    err = np.linalg.norm(L.x - Lx)/np.linalg.norm(Lx)
    bad = [j for j in range(A.size()) if np.abs(L.x[Lp[j]:Lp[j+1]] - Lx[Lp[j]:Lp[j+1]]).max() > 1e-8*np.abs(Lx).max()] if same else []
    print(name, kw, "pattern", same, "err %.3e" % err, "bad cols", bad[:20], len(bad))
    s = sc.Symbolic(A, **kw).supernodes()
    print("  sn start", s['start'][:20], "w", s['w'][:20], "m", s['m'][:20], "lev", s['level'][:20])
G = "/root/repo/tests/golden/"
A = sc.load_matrix_market_to_csc(G + "bcsstk01.mtx")
run("bcsstk01", A)
run("bcsstk01", A, relax=0)
B = sc.load_matrix_market_to_csc(G + "1138_bus.mtx")
run("1138", B)
run("lap8", sc.laplacian3d(8))
run("lap12", sc.laplacian3d(12))
