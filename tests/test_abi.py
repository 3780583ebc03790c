"""C-ABI boundary: libhdrf.so loads on CPU and exports every symbol include/hdrf.h declares.
No compute calls (no GPU needed)."""
import ctypes
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "hdrf.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hdrf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    import hdrf_amd.lib as lib
    decl = _declared()
    assert decl == sorted(lib.EXPORTS), (set(decl) ^ set(lib.EXPORTS))


def test_library_exports_every_declared_symbol():
    import hdrf_amd.lib as lib
    if not os.path.exists(lib.LIB_PATH):
        lib.build()
    so = ctypes.CDLL(lib.LIB_PATH)
    missing = [s for s in _declared() if not hasattr(so, s)]
    assert not missing, missing


def test_default_config_and_bad_config_are_rejected_without_gpu():
    import hdrf_amd.lib as lib
    cfg = lib.default_config()
    assert (cfg.window, cfg.max_chunk, cfg.n_thread, cfg.min_mt_chunks, cfg.container_max) == \
        (700, 1000000, 3, 25, 1 << 25)
    bad = lib.default_config(window=5)
    h = ctypes.c_void_p()
    assert lib.load().hdrf_open(ctypes.byref(bad), ctypes.byref(h)) == -1
    unsupported = lib.default_config(compressor=3)          # stream codecs: not in this build
    assert lib.load().hdrf_open(ctypes.byref(unsupported), ctypes.byref(h)) == -6
    node_lz4 = lib.default_config(compressor=2, n_ranks=2, rank=0)   # node-global compressor 2: accepted
    assert lib.load().hdrf_open(ctypes.byref(node_lz4), ctypes.byref(h)) != -6
    bad_rank = lib.default_config(n_ranks=2, rank=2)
    assert lib.load().hdrf_open(ctypes.byref(bad_rank), ctypes.byref(h)) == -1


def test_product_package_does_not_import_oracle():
    """The oracle is test infrastructure: the product package never imports or links it."""
    pkg = os.path.join(ROOT, "hdrf_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", txt, re.M), f
                assert "hdrf_oracle" not in txt, f
