"""ctypes binding of libmirsha.so (the C ABI in include/mirsha.h).

The library is built in-tree (``mirbft_amd/libmirsha.so``, see
``mirbft_amd/csrc/Makefile`` and ``__graft_entry__.build()``). Loading fails
loudly when it is missing: there is no Python or CPU fallback for hashing.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB_PATH = os.path.join(_HERE, "libmirsha.so")
# MSHA_LIB_PATH loads a diagnostic or A/B variant built OUTSIDE the package
# (mirbft_amd/csrc/Makefile: BUILD=... OUT=...), so no experiment ever writes
# over the product library. Such a build is not the tree's: GPU test sessions
# and bench.py refuse it unless MSHA_ALLOW_FOREIGN_LIB=1.
LIB_PATH = os.environ.get("MSHA_LIB_PATH") or PRODUCT_LIB_PATH
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mirsha.h")

ABI_VERSION = 10
MSHA_OK = 0
MSHA_ERR_INVALID_ARG = 1
MSHA_ERR_NO_DEVICE = 2
MSHA_ERR_HIP = 3
MSHA_ERR_OUT_OF_MEMORY = 4
MSHA_ERR_ALIGNMENT = 5
MSHA_DEVICE_ARENA_SLACK = 64
MSHA_DEVICE_ALIGN = 16
MSHA_KERNEL_AUTO = 0
MSHA_KERNEL_LANE = 1
MSHA_KERNEL_COOP = 2

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_ctxp = ctypes.c_void_p


class MshaStats(ctypes.Structure):
    _fields_ = [
        ("calls", ctypes.c_uint64),
        ("messages", ctypes.c_uint64),
        ("message_bytes", ctypes.c_uint64),
        ("blocks", ctypes.c_uint64),
        ("plan_ms", ctypes.c_double),
        ("pack_ms", ctypes.c_double),
        ("device_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("direct_calls", ctypes.c_uint64),
        ("launches_lane", ctypes.c_uint64),
        ("launches_pipe", ctypes.c_uint64),
        ("launches_coop", ctypes.c_uint64),
        ("launches_split", ctypes.c_uint64),
        ("launches_dod", ctypes.c_uint64),
        ("split_retries", ctypes.c_uint64),
        ("h2d_bytes", ctypes.c_uint64),
        ("d2h_bytes", ctypes.c_uint64),
        ("small_calls", ctypes.c_uint64),
        ("staged_calls", ctypes.c_uint64),
        ("planned_device_calls", ctypes.c_uint64),
        ("launches_chain2", ctypes.c_uint64),
        ("launches_chain8", ctypes.c_uint64),
        ("small_zc_calls", ctypes.c_uint64),
        ("launches_lane_ws", ctypes.c_uint64),
    ]


class MshaShardStats(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("head_lanes", ctypes.c_uint32),
        ("messages", ctypes.c_uint64),
        ("lanes", ctypes.c_uint64),
        ("h2d_payload_bytes", ctypes.c_uint64),
        ("h2d_bytes", ctypes.c_uint64),
        ("d2h_bytes", ctypes.c_uint64),
        ("launches", ctypes.c_uint64),
        ("gather_begin_ms", ctypes.c_double),
        ("gather_end_ms", ctypes.c_double),
        ("gather_ms", ctypes.c_double),
        ("device_ms", ctypes.c_double),
        ("upload_ms", ctypes.c_double),
        ("kernel_ms", ctypes.c_double),
        ("first_launch_ms", ctypes.c_double),
        ("plan_kernel_ms", ctypes.c_double),
    ]


class MshaClockInfo(ctypes.Structure):
    _fields_ = [
        ("ghz_median", ctypes.c_double),
        ("ghz_min", ctypes.c_double),
        ("ghz_max", ctypes.c_double),
        ("kernel_ms", ctypes.c_double),
        ("gblocks_per_s", ctypes.c_double),
        ("workgroups", ctypes.c_uint32),
        ("blocks_per_lane", ctypes.c_uint32),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "msha_abi_version": (ctypes.c_uint32, []),
    "msha_build_id": (ctypes.c_char_p, []),
    "msha_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "msha_ctx_create": (ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(_ctxp)]),
    "msha_ctx_create_err": (ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(_ctxp), ctypes.c_char_p,
                                           ctypes.c_uint64]),
    "msha_ctx_destroy": (None, [_ctxp]),
    "msha_last_error": (ctypes.c_char_p, [_ctxp]),
    "msha_last_error_copy": (ctypes.c_uint64, [_ctxp, ctypes.c_char_p, ctypes.c_uint64]),
    "msha_get_stats": (ctypes.c_int, [_ctxp, ctypes.POINTER(MshaStats)]),
    "msha_shard_count": (ctypes.c_int, [_ctxp, ctypes.POINTER(ctypes.c_uint32)]),
    "msha_get_shard_stats": (ctypes.c_int, [_ctxp, ctypes.c_uint32, ctypes.POINTER(MshaShardStats)]),
    "msha_hash_actions": (ctypes.c_int, [_ctxp, _u8p, ctypes.c_uint64, _u64p, _u64p, ctypes.c_uint64,
                                         _u64p, ctypes.c_uint64, _u8p]),
    "msha_digest_batch": (ctypes.c_int, [_ctxp, _u8p, ctypes.c_uint64, _u64p, _u64p, ctypes.c_uint64,
                                         _u8p]),
    "msha_digest_of_digests": (ctypes.c_int, [_ctxp, _u8p, ctypes.c_uint64, _u32p, ctypes.c_uint64,
                                              _u64p, ctypes.c_uint64, _u8p]),
    "msha_digest_batch_device": (ctypes.c_int, [_ctxp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                ctypes.c_void_p]),
    "msha_digest_batch_device_planned": (ctypes.c_int, [_ctxp, ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                        ctypes.c_void_p, ctypes.c_void_p]),
    "msha_digest_uniform_device": (ctypes.c_int, [_ctxp, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "msha_digest_of_digests_device": (ctypes.c_int, [_ctxp, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                     ctypes.c_void_p]),
    "msha_device_status": (ctypes.c_int, [_ctxp]),
    "msha_clock_probe": (ctypes.c_int, [_ctxp, ctypes.c_uint32, ctypes.POINTER(MshaClockInfo)]),
    "msha_set_kernel_policy": (ctypes.c_int, [_ctxp, ctypes.c_int]),
    "msha_pinned_alloc": (ctypes.c_int, [_ctxp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]),
    "msha_pinned_free": (ctypes.c_int, [_ctxp, ctypes.c_void_p]),
    "msha_blocks_for_len": (ctypes.c_uint64, [ctypes.c_uint64]),
    "msha_order_by_blocks": (ctypes.c_int, [_u64p, ctypes.c_uint64, _u32p]),
    "msha_partition_by_blocks": (ctypes.c_int, [_u64p, ctypes.c_uint64, ctypes.c_uint32, _u64p]),
    "msha_alias_first": (ctypes.c_int, [_u64p, _u64p, ctypes.c_uint64, _u64p]),
}

_lib = None


def header_symbols() -> list[str]:
    """Every function the public header declares."""
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(msha_\w+)\s*\(", text, re.M)))


def lib() -> ctypes.CDLL:
    """Load libmirsha.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C mirbft_amd/csrc` (there is no CPU fallback)")
    # One HIP runtime per process: torch ships its own libamdhip64 (NEEDED as
    # "libamdhip64.so", SONAME libamdhip64.so.7). Loaded first, it satisfies our
    # NEEDED libamdhip64.so.7 by SONAME and both share it; loaded second, torch
    # would bring a second runtime and fail to initialise. So when torch is
    # installed it is imported before libmirsha.so is opened.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.msha_abi_version() != ABI_VERSION:
        raise ImportError("libmirsha ABI version mismatch")
    _lib = L
    return L


# The files msha_build_id()'s src hash covers, in the Makefile's order (SRCS).
_SRC_FILES = ("sha256_device.hpp", "kernels.hpp", "kernels.hip", "plan.hip", "mirsha.cpp",
              os.path.join("..", "..", "include", "mirsha.h"))


def source_id() -> str:
    """The src hash of the tree's sources, as the Makefile computes it for msha_build_id()."""
    import hashlib
    h = hashlib.sha256()
    for f in _SRC_FILES:
        with open(os.path.join(_HERE, "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id() -> dict:
    """The loaded library's build: its src hash and flags, and whether it is the tree's own
    build (src equal to source_id() and no experiment's -D overrides in the flags)."""
    raw = lib().msha_build_id().decode()
    fields = dict(kv.split("=", 1) for kv in raw.split(";"))
    src, flags = fields.get("src", ""), fields.get("flags", "")
    tree = source_id()
    return {"id": raw, "src": src, "flags": flags, "tree_src": tree, "path": LIB_PATH,
            "matches_tree": (src == tree and not any(t.startswith("-D") for t in flags.split())
                             and os.path.realpath(LIB_PATH) == os.path.realpath(PRODUCT_LIB_PATH))}


def foreign_allowed() -> bool:
    """MSHA_ALLOW_FOREIGN_LIB=1: run on a library that is not the tree's build (A/B, diagnostics)."""
    return os.environ.get("MSHA_ALLOW_FOREIGN_LIB") == "1"


def require_tree_build(who: str) -> dict:
    """The loaded library's build_id(); raises unless it is the tree's own build or
    MSHA_ALLOW_FOREIGN_LIB=1 (results of an experiment's build must not be reported
    as the product's)."""
    b = build_id()
    if not b["matches_tree"] and not foreign_allowed():
        raise RuntimeError("%s: %s is not this tree's build (%s; tree src %s): rebuild it "
                           "(make -C mirbft_amd/csrc) or set MSHA_ALLOW_FOREIGN_LIB=1"
                           % (who, b["path"], b["id"], b["tree_src"]))
    return b
