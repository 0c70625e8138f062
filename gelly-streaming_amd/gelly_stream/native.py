"""ctypes binding of the C ABI declared in include/gelly_cc.h (libgelly_cc.so, built for gfx950).

The product path has no CPU fallback: if the library is missing or no gfx950 device is visible, calls
raise GellyCCError. Build with ``python -c "import __graft_entry__ as g; g.build()"`` (or ``make -C
gelly-streaming_amd``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_char_p, c_float, c_int, c_uint32, c_uint64, c_void_p

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GELLY_CC_LIB: an alternative build of the same ABI (A/B measurements of kernel variants; the CPU tests' host build
# of the group merge, tests/cpp/build/libgelly_group_host.so, which exports only the merge's part of the ABI)
LIB_PATH = os.environ.get("GELLY_CC_LIB") or os.path.join(PKG_ROOT, "lib", "libgelly_cc.so")

UNSEEN = 0xFFFFFFFF

GCC_GEN_EXAMPLE = 1
GCC_GEN_RMAT = 2
GCC_GEN_GNM = 3
GCC_GEN_ADVERSARIAL = 4

ERRORS = {-1: "GCC_E_INVALID", -2: "GCC_E_HIP", -3: "GCC_E_NODEV", -4: "GCC_E_OOM", -5: "GCC_E_INTERNAL"}


class GellyCCError(RuntimeError):
    """A C-ABI call returned a negative status (the JNI glue maps the same codes to Java exceptions)."""

    def __init__(self, code: int, fn: str, msg: str):
        super().__init__(f"{fn}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


class GenParams(ctypes.Structure):
    """gcc_gen_params (include/gelly_cc.h)."""

    _fields_ = [
        ("kind", c_uint32),
        ("scale", c_uint32),
        ("n_vertices", c_uint64),
        ("n_edges", c_uint64),
        ("seed", c_uint64),
        ("n_stars", c_uint32),
        ("star_size", c_uint32),
        ("permute", c_uint32),
        ("reserved", c_uint32),
    ]


# exported symbol -> (restype, argtypes); the not-gpu tests check that every symbol in include/*.h is here
_SIGS = {
    "gcc_last_error": (c_char_p, []),
    "gcc_version": (c_int, []),
    "gcc_device_count": (c_int, [POINTER(c_int)]),
    "gcc_init": (c_int, [c_int]),
    "gcc_gen_info": (c_int, [POINTER(GenParams), POINTER(c_uint64), POINTER(c_uint64)]),
    "gcc_gen_host": (c_int, [POINTER(GenParams), c_uint64, c_uint64, c_void_p]),
    "gcc_gen_device": (c_int, [POINTER(GenParams), c_uint64, c_uint64, c_void_p, c_void_p]),
    "gcc_forest_create": (c_int, [c_int, c_uint32, POINTER(c_void_p)]),
    "gcc_forest_create_ext": (c_int, [c_int, c_uint32, c_void_p, c_void_p, POINTER(c_void_p)]),
    "gcc_forest_destroy": (c_int, [c_void_p]),
    "gcc_forest_set_stream": (c_int, [c_void_p, c_void_p, c_int]),
    "gcc_forest_get_stream": (c_int, [c_void_p, POINTER(c_void_p)]),
    "gcc_forest_capacity": (c_int, [c_void_p, POINTER(c_uint32)]),
    "gcc_forest_device": (c_int, [c_void_p, POINTER(c_int)]),
    # cross-GPU group merge over RCCL (gelly_group.cpp)
    "gcc_comm_unique_id": (c_int, [c_void_p]),
    "gcc_comm_init": (c_int, [c_int, c_int, c_int, c_void_p, POINTER(c_void_p)]),
    "gcc_comm_init_all": (c_int, [c_int, c_void_p, c_void_p]),
    "gcc_comm_destroy": (c_int, [c_void_p]),
    "gcc_comm_info": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_uint64)]),
    "gcc_comm_last_merge": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_uint64)]),
    "gcc_comm_last_merge_kind": (c_int, [c_void_p, POINTER(c_int), POINTER(c_uint64), POINTER(c_uint64)]),
    "gcc_forest_group_merge": (c_int, [c_void_p, c_void_p]),
    "gcc_group_merge": (c_int, [c_void_p, c_int, c_void_p]),
    "gcc_forest_device_ptr": (c_int, [c_void_p, POINTER(c_void_p)]),
    "gcc_forest_reset": (c_int, [c_void_p]),
    "gcc_forest_union": (c_int, [c_void_p, c_uint32, c_uint32]),
    "gcc_forest_make_set": (c_int, [c_void_p, c_uint32]),
    "gcc_forest_staging": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint64)]),
    "gcc_forest_submit": (c_int, [c_void_p, c_uint64]),
    "gcc_forest_fold_host": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_fold_device": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_fold_pinned": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_labels_device": (c_int, [c_void_p, POINTER(c_void_p)]),
    "gcc_forest_flush": (c_int, [c_void_p]),
    "gcc_forest_sync": (c_int, [c_void_p]),
    "gcc_forest_merge": (c_int, [c_void_p, c_void_p]),
    "gcc_forest_merge_labels_device": (c_int, [c_void_p, c_void_p, c_uint32]),
    "gcc_forest_compress": (c_int, [c_void_p]),
    "gcc_forest_labels": (c_int, [c_void_p, c_void_p, c_uint32]),
    "gcc_forest_find": (c_int, [c_void_p, c_uint32, POINTER(c_uint32)]),
    "gcc_forest_raw_parent": (c_int, [c_void_p, c_void_p, c_uint32]),
    "gcc_forest_size": (c_int, [c_void_p, POINTER(c_uint64)]),
    "gcc_forest_count_components": (c_int, [c_void_p, POINTER(c_uint64)]),
    "gcc_forest_import_pairs": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_serialized_size": (c_int, [c_void_p, POINTER(c_uint64)]),
    "gcc_forest_serialize": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "gcc_forest_deserialize": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_enable_timing": (c_int, [c_void_p, c_int]),
    "gcc_forest_last_fold_ms": (c_int, [c_void_p, POINTER(c_float)]),
    "gcc_forest_fold_profile": (c_int, [c_void_p, c_char_p, c_uint64]),
    "gcc_step_mark": (c_int, [c_void_p]),
    "gcc_forest_tune": (c_int, [c_void_p, c_char_p, ctypes.c_double]),
    "gcc_forest_label_digest": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)]),
    "gcc_forest_inc_check_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)]),
    "gcc_forest_post_check_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), c_void_p, c_uint32]),
    "gcc_msg_bytes": (c_uint64, [c_uint32, c_uint64]),
    "gcc_forest_encode": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_absorb": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_absorb_many": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_uint64]),
    "gcc_delta_msg_bytes": (c_uint64, [c_uint64]),
    "gcc_forest_delta_arm": (c_int, [c_void_p]),
    "gcc_forest_encode_delta": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_forest_absorb_delta_many": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_uint64]),
    # id dictionary for Java Long vertex ids (host-only)
    "gcc_idmap_create": (c_int, [c_uint32, POINTER(c_void_p)]),
    "gcc_idmap_destroy": (c_int, [c_void_p]),
    "gcc_idmap_size": (c_int, [c_void_p, POINTER(c_uint64)]),
    "gcc_idmap_map": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "gcc_idmap_lookup": (c_int, [c_void_p, ctypes.c_int64, POINTER(c_uint32)]),
    "gcc_idmap_ids": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_idmap_canonical": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, ctypes.c_int64]),
    # BipartitenessCheck's Candidates summary (signed forest)
    "gcc_signed_create": (c_int, [c_int, c_uint32, POINTER(c_void_p)]),
    "gcc_signed_destroy": (c_int, [c_void_p]),
    "gcc_signed_set_stream": (c_int, [c_void_p, c_void_p, c_int]),
    "gcc_signed_capacity": (c_int, [c_void_p, POINTER(c_uint32)]),
    "gcc_signed_reset": (c_int, [c_void_p]),
    "gcc_signed_fold_host": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_signed_fold_device": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_signed_merge": (c_int, [c_void_p, c_void_p]),
    "gcc_signed_compress": (c_int, [c_void_p]),
    "gcc_signed_merge_words": (c_int, [c_void_p, c_void_p, c_uint32, c_int]),
    "gcc_signed_device_words": (c_int, [c_void_p, POINTER(c_void_p)]),
    "gcc_signed_tune": (c_int, [c_void_p, c_char_p, ctypes.c_double]),
    "gcc_signed_words": (c_int, [c_void_p, c_void_p, c_uint32]),
    "gcc_signed_success": (c_int, [c_void_p, POINTER(c_int)]),
    "gcc_literal_create": (c_int, [c_int, c_uint32, c_uint32, POINTER(c_void_p)]),
    "gcc_literal_destroy": (c_int, [c_void_p]),
    "gcc_literal_reset": (c_int, [c_void_p]),
    "gcc_literal_fold_host": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gcc_literal_merge": (c_int, [c_void_p, c_void_p]),
    "gcc_literal_success": (c_int, [c_void_p, POINTER(c_int)]),
    "gcc_literal_entries": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
}

MSG_HEADER_BYTES = 16  # GCC_MSG_HEADER_BYTES


def msg_bytes(id_capacity: int, cap_others: int) -> int:
    """gcc_msg_bytes: size of a cross-GPU merge message (header + giant bitmap + cap_others (v, label) pairs)."""
    return MSG_HEADER_BYTES + (int(id_capacity) + 63) // 64 * 8 + int(cap_others) * 8

_lib = None


def _bind_torch_runtime_first() -> None:
    """One HIP runtime per process: torch ships its own libamdhip64 / libhsa-runtime64 (same soname as
    /opt/rocm's). If libgelly_cc were loaded first, torch would map a second HIP + HSA runtime and see no GPU
    (measured on the MI355X box: tools/probe_runtime.py). Importing torch first makes libgelly_cc bind to the
    already-loaded runtime by soname. Processes without torch (C/C++/JNI consumers) use /opt/rocm's."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> ctypes.CDLL:
    """Load libgelly_cc.so (once). Raises GellyCCError if it has not been built."""
    global _lib
    if _lib is None:
        _bind_torch_runtime_first()
        if not os.path.exists(LIB_PATH):
            raise GellyCCError(-3, "load", f"{LIB_PATH} not found: build it first (__graft_entry__.build())")
        l = ctypes.CDLL(LIB_PATH)
        partial = bool(os.environ.get("GELLY_CC_LIB"))
        for name, (res, args) in _SIGS.items():
            if partial and not hasattr(l, name):
                continue  # an alternative build may carry part of the ABI; calling a missing symbol raises
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def call(name: str, *args) -> None:
    """Call a status-returning C-ABI function; raise GellyCCError on a negative status."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().gcc_last_error()
        raise GellyCCError(rc, name, msg.decode() if msg else "")


def device_count() -> int:
    n = c_int(0)
    call("gcc_device_count", byref(n))
    return n.value


def exported_symbols() -> list[str]:
    return sorted(_SIGS)
