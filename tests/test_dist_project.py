"""CPU test of the N-GPU critical-path replay (scripts/dist_project.py) on synthetic
per-rank timelines over a real plan: the backtracked chain must add up to the finish
time and name real comm steps."""
import importlib.util
import os

import numpy as np

import sparsecholesky_amd as sc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("dist_project", os.path.join(ROOT, "scripts", "dist_project.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_critical_path_chain_adds_up():
    dp = _load()
    symb = sc.Symbolic(sc.laplacian3d(20), panel_nb_outer=128, dist_cbb=128)
    n = 4
    steps = symb.dist_steps(n)
    nst = len(steps["kind"])
    assert nst > 4
    rng = np.random.default_rng(0)
    tls = []
    for r in range(n):
        # a monotone dry timeline: step st posted at st + jitter, needed 0.3 ms later
        post = {st: st * 1.0 + float(rng.uniform(0, 0.5)) for st in range(nst)}
        need = {st: post[st] + 0.3 for st in range(nst)}
        total = nst * 1.0 + 2.0
        main = [(0.0, total / 2, 4), (total / 2, total, 5)]
        tls.append((total, post, need, main))
    fin, why = dp.critical_path(symb, n, tls, 50.0, 10.0, explain=True)
    plain = dp.critical_path(symb, n, tls, 50.0, 10.0)
    assert fin == plain
    tot = why["totals"]["compute_ms"] + why["totals"]["wait_ms"]
    assert abs(tot - max(fin)) < 1e-2, (tot, max(fin))
    for c in why["chain"]:
        if "step" in c:
            assert 0 <= c["step"] < nst and c["step_kind"] in ("INIT", "SLAB", "DELIVER")
    # slow links move the critical path onto the transfers
    fin2, why2 = dp.critical_path(symb, n, tls, 0.05, 10.0, explain=True)
    assert max(fin2) > max(fin)
    assert why2["totals"]["wait_ms"] > why["totals"]["wait_ms"]
