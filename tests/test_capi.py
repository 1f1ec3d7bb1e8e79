"""C-ABI boundary: the library loads and exports every symbol include/*.h declares."""
import ctypes
import os
import re

import numpy as np

import sparsecholesky_amd as sc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if fn.endswith(".h"):
            txt = open(os.path.join(inc, fn)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            names |= set(re.findall(r"\b(sc_[A-Za-z0-9_]+)\s*\(", txt))
    return names


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(sc.LIB_PATH)
    decl = declared_symbols()
    assert len(decl) >= 30
    missing = [s for s in sorted(decl) if not hasattr(L, s)]
    assert not missing, missing
    # the Python mirror binds exactly the declared C ABI
    assert set(sc.exported_symbols()) == decl


def test_version_and_status_strings():
    L = sc.lib()
    assert L.sc_version() == 121
    assert L.sc_status_string(3) == b"A is not positive definite."
    assert L.sc_status_string(0) == b"ok"
    assert L.sc_status_string(-1) == b"invalid argument"


def test_default_options():
    o = sc.default_options()
    assert o.relax == 1 and list(o.nrelax) == [4, 16, 48] and o.small_front_max == 128
    assert o.panel_nb == 64 and o.panel_nb_outer == 1024 and o.syrk_tile == 0
    assert o.dist_asm == 1 and o.dist_pieces == 4
    assert o.lookahead == 1 and o.inner_order == 1 and o.asm_tile_min_m == 0
    # round 5: the measured-slower schedule knobs are gone from the ABI
    names = {f[0] for f in type(o)._fields_}
    for gone in ("panel_tall", "trsm_fold", "la_grid", "cb_slab", "cb_gather_min_w", "la_split", "la_after",
                 "cb_lean_kmin", "cb_small_kmax"):
        assert gone not in names


def test_debug_hooks_live_in_their_own_header():
    inc = os.path.join(ROOT, "include")
    main = re.sub(r"/\*.*?\*/", "", open(os.path.join(inc, "sparsecholesky.h")).read(), flags=re.S)
    dbg = open(os.path.join(inc, "sparsecholesky_debug.h")).read()
    assert "sc_debug_" not in main
    assert "sc_debug_contention" in dbg and "sc_debug_syrk" in dbg


def test_bad_arguments_return_errors():
    L = sc.lib()
    assert L.sc_analyze(-1, None, None, None, ctypes.byref(ctypes.c_void_p())) == -1
    assert L.sc_etree(-1, None, None, None) == -1
    assert L.sc_export_L(None, None, None, None) == -1
    assert L.sc_factor(None, None) == -1
    assert L.sc_laplacian3d(0, 1, None, None, None, None) == -1


def test_symbolic_handle_lifecycle_no_gpu_needed():
    A = sc.laplacian3d(6)
    s = sc.Symbolic(A)
    Lp, Li = s.pattern()
    assert Lp[-1] == s.nnz_L == len(Li)
    del s
