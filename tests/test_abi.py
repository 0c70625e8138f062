"""CPU: the C-ABI library loads, exports every symbol include/gelly_cc.h declares, and fails loudly without
a GPU (no CPU fallback on the product path). No compute call is made here."""
import ctypes
import os
import re
import subprocess

import pytest

from gelly_stream import native
from gelly_stream.native import GenParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gelly_cc.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gcc_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for must in ("gcc_forest_create", "gcc_forest_union", "gcc_forest_fold_device", "gcc_forest_merge",
                 "gcc_forest_find", "gcc_forest_size", "gcc_forest_labels", "gcc_last_error"):
        assert must in fns


def test_every_declared_symbol_is_exported_and_bound():
    lib = native.lib()
    fns = declared_functions()
    assert fns == native.exported_symbols(), "native._SIGS must bind exactly the header's functions"
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r" T (gcc_\w+)$", out.stdout, flags=re.M))
    for fn in fns:
        assert fn in exported, fn
        assert hasattr(lib, fn)


def test_library_is_gfx950_code_object():
    # the fat binary embeds the offload target id of its only code object
    data = open(native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data


def test_version():
    assert native.lib().gcc_version() == 1


@pytest.mark.skipif(native.device_count() > 0, reason="checks the no-GPU failure path")
def test_create_fails_loudly_without_gpu():
    h = ctypes.c_void_p()
    rc = native.lib().gcc_forest_create(0, 16, ctypes.byref(h))
    assert rc == -3  # GCC_E_NODEV
    assert b"no HIP device" in native.lib().gcc_last_error()
    with pytest.raises(native.GellyCCError):
        from gelly_stream import DisjointSet

        DisjointSet(16)


def test_gen_info_validation():
    e, v = ctypes.c_uint64(), ctypes.c_uint64()
    bad = GenParams(99, 0, 0, 0, 0, 0, 0, 0, 0)
    assert native.lib().gcc_gen_info(ctypes.byref(bad), ctypes.byref(e), ctypes.byref(v)) == -1
    assert b"unknown generator" in native.lib().gcc_last_error()
    ok = GenParams(native.GCC_GEN_ADVERSARIAL, 23, 0, 0, 5, 1024, 8192, 0, 0)
    native.call("gcc_gen_info", ctypes.byref(ok), ctypes.byref(e), ctypes.byref(v))
    assert v.value == 1 << 24 and e.value == (1 << 23) - 1 + 1024 * 8191


def test_null_handle_is_an_error_not_a_crash():
    rc = native.lib().gcc_forest_size(None, None)
    assert rc == -1
    assert native.lib().gcc_forest_destroy(None) == 0


def test_every_error_code_is_named():
    """Each GCC_E_* code the header defines has its name in the Python binding's ERRORS table."""
    import re

    from gelly_stream import native

    text = open(os.path.join(ROOT, "include", "gelly_cc.h")).read()
    codes = {int(v): k for k, v in re.findall(r"#define (GCC_E_\w+) \((-\d+)\)", text)}
    assert codes, "no error codes found in the header"
    assert {c: native.ERRORS.get(c) for c in codes} == codes
