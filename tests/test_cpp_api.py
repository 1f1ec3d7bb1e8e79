"""The C++ drop-in header (include/sparsecholesky/chol.hpp) replays the reference's
gtests (tests/test_chol.cpp of the reference) against libsparsecholesky_amd."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "sparsecholesky_amd")


def _compiler():
    for cxx, std in (("/opt/rocm/lib/llvm/bin/clang++", "c++23"), ("g++", "c++20")):
        if shutil.which(cxx) or os.path.exists(cxx):
            return cxx, std
    pytest.skip("no C++ compiler")


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    cxx, std = _compiler()
    out = str(tmp_path_factory.mktemp("cpp") / "test_chol")
    subprocess.run([cxx, f"-std={std}", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_chol.cpp"), "-o", out, "-L", LIBDIR,
                    "-lsparsecholesky_amd", f"-Wl,-rpath,{LIBDIR}"], check=True)
    return out


def _run(binary, *args):
    env = dict(os.environ, SC_GOLDEN_DIR=os.path.join(ROOT, "tests", "golden"))
    r = subprocess.run([binary, *args], capture_output=True, text=True, env=env, timeout=300)
    return r.returncode, r.stdout + r.stderr


def test_cpp_dropin_host_cases(binary):
    rc, out = _run(binary, "--cpu-only")
    assert rc == 0, out
    assert "0 failed" in out


def test_cpp_dropin_cxx20_compiles(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    out = str(tmp_path / "t20")
    subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_chol.cpp")], check=True)


@pytest.mark.gpu
def test_cpp_dropin_all_cases(gpu, binary):
    rc, out = _run(binary)
    assert rc == 0, out
    assert "0 failed" in out
    assert "SupernodalCholesky" in out
