"""The JNI binding a DataNode loads (integration/jni/hdrf_jni.c) executed through a working JNIEnv
(tests/cpp/jni_driver.c: direct buffers, arrays, strings, per-thread exceptions; the JDK is absent
here): the JNI's own context shape (open0: 256 arena slots, retain_containers, 16-block batches),
ticketed reductions on threads started in reverse, packet receive with submitBlocks, reduceAsync,
drain0 into a chunkDir after every batch — every file compared with the oracle's container
(DN/DataDeduplicator.java:748-818), recipe0 / length0 / reconstruct0 / stream0 / streamDecode0, and
the argument checks raising IOException."""
import os
import subprocess

import pytest

from conftest import ROOT


def build_driver(out):
    import hdrf_amd.lib as lib
    if not os.path.exists(lib.LIB_PATH):
        lib.build()
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    libdir = os.path.dirname(lib.LIB_PATH)
    odir = os.path.join(ROOT, "oracle", "_build")
    subprocess.run(["gcc", "-std=gnu11", "-O2", "-Wall", "-Wextra", "-Werror", "-pthread",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
                    "-I", os.path.join(ROOT, "tests", "cpp", "jni_mock"),
                    os.path.join(ROOT, "tests", "cpp", "jni_driver.c"),
                    os.path.join(ROOT, "integration", "jni", "hdrf_jni.c"), "-o", out,
                    "-L", libdir, "-lhdrf", "-L", odir, "-lhdrf_oracle", "-Wl,-rpath," + libdir + ":" + odir],
                   check=True)
    return out


def test_jni_driver_builds(tmp_path):
    """The shim and its driver compile and link against libhdrf (no GPU call here)."""
    assert os.path.exists(build_driver(str(tmp_path / "jni_driver")))


@pytest.mark.gpu
@pytest.mark.parametrize("compressor", [1, 2])
def test_jni_binding_end_to_end(tmp_path, compressor):
    exe = build_driver(str(tmp_path / "jni_driver"))
    chunk_dir = tmp_path / "chunkDir"
    chunk_dir.mkdir()
    r = subprocess.run([exe, str(compressor), str(chunk_dir) + "/", "16", "18"], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and r.stdout.rstrip().endswith("PASS"), r.stdout[-2000:]
    assert "closed)" in r.stdout and len(os.listdir(chunk_dir)) > 0
