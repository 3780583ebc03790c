"""The C++ host mirror (include/hdrf_scheme.hpp) compiles against the C-ABI (CPU) and, on the
GPU, reduces blocks identically to the oracle (tests/cpp/scheme_test.cpp)."""
import os
import subprocess

import pytest

from conftest import ROOT


def _build(tmp_path):
    import hdrf_amd.lib as lib
    if not os.path.exists(lib.LIB_PATH):
        lib.build()
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    exe = str(tmp_path / "scheme_test")
    libdir = os.path.dirname(lib.LIB_PATH)
    odir = os.path.join(ROOT, "oracle", "_build")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests", "cpp", "scheme_test.cpp"), "-o", exe,
                    "-L", libdir, "-lhdrf", "-L", odir, "-lhdrf_oracle",
                    "-Wl,-rpath," + libdir + ":" + odir], check=True)
    return exe


def test_cpp_scheme_compiles(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_cpp_scheme_matches_oracle_on_gpu(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "PASS" in r.stdout


def test_jni_shim_compiles():
    """integration/jni/hdrf_jni.c (the binding a maintainer adds to the DataNode) compiles against
    include/hdrf.h; the JDK is absent here, so a minimal jni.h with the spec's signatures stands in."""
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "tests", "cpp", "jni_mock"),
                    os.path.join(ROOT, "integration", "jni", "hdrf_jni.c")], check=True)
