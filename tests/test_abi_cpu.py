"""CPU checks of the C-ABI library: it loads without a GPU and exports exactly
the entry points include/dlamd.h declares (no compute calls here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "dlamd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:int|int32_t|int64_t|const char\*)\s+(dl_\w+)\s*\(", src, flags=re.M))


@pytest.fixture(scope="module")
def lib():
    from deep_learning_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from deep_learning_amd import build
        build.build(verbose=False)
    return _lib


def test_header_symbols_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T dl_" in l}
    declared = _declared()
    assert declared, "no declarations parsed"
    assert declared <= exported, "declared but not exported: %s" % sorted(declared - exported)
    assert set(lib.SIGNATURES) == declared, "ctypes table out of sync: %s" % sorted(set(lib.SIGNATURES) ^ declared)


def test_library_loads_and_reports_errors(lib):
    L = lib.lib()
    assert L.dl_abi_version() == 1
    # argument validation runs on the host: a bad GEMM call fails with a message, no launch
    rc = L.dl_gemm_f32(0, 0, 4, 4, 4, None, 4, None, 4, None, 4, 0, None, 0, 1, 0, None)
    assert rc != 0
    assert b"NULL" in L.dl_last_error()


def test_layout_struct_size(lib):
    import ctypes
    assert ctypes.sizeof(lib.EmbLayout) == 4 * 8 + 21 * 4 + 4  # 4 int64 + 21 int32 + pad


def test_reader_header_symbols_exported():
    """libdlio.so (native TFRecord reader, load-style batch decoder) exports exactly what include/dlio.h
    declares."""
    from deep_learning_amd.utils import native_reader as nr
    if not os.path.exists(nr.LIB_PATH):
        from deep_learning_amd import build
        build.build_host(verbose=False)
    src = open(os.path.join(ROOT, "include", "dlio.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    declared = set(re.findall(r"^\s*(?:void\*|void|int32_t|int64_t|uint32_t|const char\*)\s+(dlio_\w+)\s*\(",
                              src, flags=re.M))
    out = subprocess.run(["nm", "-D", "--defined-only", nr.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T dlio_" in l}
    assert len(declared) == 9 and declared == exported == set(nr.SIGNATURES)
    nr.lib()
