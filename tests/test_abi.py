"""The C-ABI library loads and exports every symbol include/mirsha.h declares;
host-only helpers work without a GPU. No compute calls here (CPU suite)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from mirbft_amd import _lib as L
from mirbft_amd.engine import blocks_for_len, partition_by_blocks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    syms = L.header_symbols()
    assert len(syms) >= 17
    lib = L.lib()
    for s in syms:
        assert hasattr(lib, s), s
    # and the ctypes signature table covers the whole header
    assert set(syms) == set(L.SIGNATURES), set(syms) ^ set(L.SIGNATURES)


def test_exports_via_nm():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in L.header_symbols():
        assert s in exported, s


def test_abi_version():
    assert L.lib().msha_abi_version() == L.ABI_VERSION == 10


def test_build_id_is_the_trees():
    """The built library says which sources it came from (msha_build_id), and they are
    this tree's: a library left behind by an experiment (an A/B build copied over the
    product .so, as round 4's wrong-digest log ran) is told apart from the product."""
    b = L.build_id()
    assert b["src"] and len(b["src"]) == 16 and "gfx950" in b["flags"], b
    assert b["matches_tree"], b


def test_library_is_gfx950_code_object():
    import re
    data = open(L.LIB_PATH, "rb").read()
    assert set(re.findall(rb"amdgcn-amd-amdhsa--gfx[0-9a-z]+", data)) == {b"amdgcn-amd-amdhsa--gfx950"}


@pytest.mark.parametrize("L_,blocks", [(0, 1), (1, 1), (55, 1), (56, 2), (63, 2), (64, 2), (119, 2),
                                       (120, 3), (512, 9), (640, 11), (65536, 1025)])
def test_blocks_for_len(L_, blocks):
    assert blocks_for_len(L_) == blocks


def test_partition_by_blocks_balanced():
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 100_000, 10_000).astype(np.uint64)
    for k in (1, 2, 3, 8):
        b = partition_by_blocks(lens, k)
        assert b[0] == 0 and b[-1] == lens.size and np.all(np.diff(b.astype(np.int64)) >= 0)
        blocks = np.array([blocks_for_len(int(x)) for x in lens])
        per = [blocks[b[i]:b[i + 1]].sum() for i in range(k)]
        assert max(per) - min(per) <= blocks.max() * 2, per


def test_partition_edge_cases():
    assert list(partition_by_blocks(np.zeros(0, dtype=np.uint64), 4)) == [0, 0, 0, 0, 0]
    b = partition_by_blocks(np.array([10**9], dtype=np.uint64), 3)
    assert b[0] == 0 and b[-1] == 1


def test_ctx_create_without_gpu_fails_loudly():
    n = ctypes.c_int(-1)
    L.lib().msha_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    from mirbft_amd import Engine, MshaError
    with pytest.raises(MshaError) as ei:
        Engine(1)
    assert ei.value.code == L.MSHA_ERR_NO_DEVICE


def test_null_args_rejected_without_gpu():
    lib = L.lib()
    assert lib.msha_get_stats(None, None) == L.MSHA_ERR_INVALID_ARG
    assert lib.msha_digest_batch(None, None, 0, None, None, 0, None) == L.MSHA_ERR_INVALID_ARG
    assert lib.msha_partition_by_blocks(None, 1, 1, None) == L.MSHA_ERR_INVALID_ARG


def test_order_by_blocks_is_descending_stable_permutation():
    from mirbft_amd.engine import order_by_blocks
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 5000, 20_000).astype(np.uint64)
    o = order_by_blocks(lens)
    assert sorted(o.tolist()) == list(range(lens.size))
    b = np.array([blocks_for_len(int(x)) for x in lens])[o]
    assert np.all(np.diff(b) <= 0)
    # stable: equal block counts keep index order
    for v in np.unique(b)[:5]:
        idx = o[b == v]
        assert np.all(np.diff(idx.astype(np.int64)) > 0)
    assert order_by_blocks(np.zeros(0, dtype=np.uint64)).size == 0


@pytest.mark.parametrize("n,maxlen", [(300_000, 5000), (300_000, 1 << 23), (70_000, 1 << 27)])
def test_order_by_blocks_threaded_matches_stable_argsort(n, maxlen):
    """Large batches take the threaded counting sort (per-thread histograms), or the
    single-thread/radix paths for huge block counts: all equal a stable argsort."""
    from mirbft_amd.engine import order_by_blocks
    rng = np.random.default_rng(n ^ maxlen)
    lens = rng.integers(0, maxlen, n).astype(np.uint64)
    lens[::7] = 512                     # many ties
    blocks = (lens >> 6) + np.where((lens & 63) < 56, 1, 2)
    exp = np.argsort(-blocks.astype(np.int64), kind="stable")
    assert np.array_equal(order_by_blocks(lens).astype(np.int64), exp)


def test_create_error_travels_with_the_call_and_across_threads():
    """msha_ctx_create_err writes the reason into the caller's buffer; the
    process-wide msha_last_error(NULL) is readable from ANOTHER thread (a Go
    caller's goroutine may resume on a different OS thread between two cgo calls)."""
    import threading
    n = ctypes.c_int(-1)
    L.lib().msha_device_count(ctypes.byref(n))
    lib = L.lib()
    ctx = ctypes.c_void_p()
    mask = 1 << 31 if n.value > 0 else 1      # device 31 does not exist; no device at all on CPU
    exp_code = L.MSHA_ERR_NO_DEVICE
    res = {}

    def create():
        buf = ctypes.create_string_buffer(256)
        res["rc"] = lib.msha_ctx_create_err(mask, ctypes.byref(ctx), buf, len(buf))
        res["buf"] = buf.value.decode()

    t = threading.Thread(target=create)
    t.start()
    t.join()
    assert res["rc"] == exp_code and ctx.value is None
    assert res["buf"], "error text returned with the call"
    seen = {}
    t2 = threading.Thread(target=lambda: seen.update(msg=lib.msha_last_error(None).decode()))
    t2.start()
    t2.join()
    assert seen["msg"] == res["buf"]
    # a tiny buffer is NUL-terminated, truncated, never overrun
    small = ctypes.create_string_buffer(b"\xff" * 8, 8)
    assert lib.msha_ctx_create_err(mask, ctypes.byref(ctx), small, 4) == exp_code
    assert small.raw[3] == 0 and small.raw[4:] == b"\xff" * 4
    assert lib.msha_ctx_create_err(mask, None, None, 0) == L.MSHA_ERR_INVALID_ARG


def test_last_error_copy_truncates_and_reports_length():
    """msha_last_error_copy copies the last error under a lock (ctx == NULL: the
    last failed creation), NUL-terminates inside the buffer, never overruns it and
    returns the full length; a NULL or empty buffer only reports the length."""
    lib = L.lib()
    ctx = ctypes.c_void_p()
    n = ctypes.c_int(-1)
    lib.msha_device_count(ctypes.byref(n))
    mask = 1 << 31 if n.value > 0 else 1
    full = ctypes.create_string_buffer(256)
    assert lib.msha_ctx_create_err(mask, ctypes.byref(ctx), full, len(full)) == L.MSHA_ERR_NO_DEVICE
    text = full.value
    buf = ctypes.create_string_buffer(512)
    assert lib.msha_last_error_copy(None, buf, len(buf)) == len(text) and buf.value == text
    small = ctypes.create_string_buffer(b"\xff" * 8, 8)
    assert lib.msha_last_error_copy(None, small, 4) == len(text)
    assert small.raw[:3] == text[:3] and small.raw[3] == 0 and small.raw[4:] == b"\xff" * 4
    assert lib.msha_last_error_copy(None, None, 0) == len(text)


def test_stats_and_shard_stats_null_args():
    lib = L.lib()
    n = ctypes.c_uint32(0)
    assert lib.msha_shard_count(None, ctypes.byref(n)) == L.MSHA_ERR_INVALID_ARG
    assert lib.msha_get_shard_stats(None, 0, None) == L.MSHA_ERR_INVALID_ARG
    assert ctypes.sizeof(L.MshaShardStats) == 8 * 15
    assert ctypes.sizeof(L.MshaStats) == 8 * 24


def _first_ref(off, ln):
    seen, out = {}, np.empty(off.size, dtype=np.uint64)
    for i, k in enumerate(zip(off.tolist(), ln.tolist())):
        out[i] = seen.setdefault(k, i)
    return out


@pytest.mark.parametrize("case", ["forward", "pool", "all_alias", "zero_len", "random", "large_pool"])
def test_alias_first_matches_dict(case):
    """msha_alias_first (the host pipeline's alias detection, candidates-first):
    forward-only batches, a shared pool pointed back into (c5 shape, both below
    and above the 2^20-key region split), zero-length messages at shared
    offsets, and dense random repeats (the whole-table path)."""
    from mirbft_amd.engine import alias_first
    rng = np.random.default_rng(len(case))
    if case == "forward":
        ln = rng.integers(0, 600, 50_000).astype(np.uint64)
        off = np.concatenate([[0], np.cumsum((ln + 15) // 16 * 16)[:-1]]).astype(np.uint64)
    elif case in ("pool", "large_pool"):
        n = 60_000 if case == "pool" else (1 << 20) + 777
        pool_off = np.arange(100, dtype=np.uint64) * np.uint64(4096)
        pool_len = rng.integers(1, 4000, 100).astype(np.uint64)
        kind = rng.random(n) < 0.05
        pick = rng.integers(0, 100, n)
        own_len = rng.integers(1, 640, n).astype(np.uint64)
        own_off = np.uint64(1 << 20) + np.concatenate([[0], np.cumsum(own_len)[:-1]]).astype(np.uint64)
        off = np.where(kind, pool_off[pick], own_off).astype(np.uint64)
        ln = np.where(kind, pool_len[pick], own_len).astype(np.uint64)
        if case == "pool":
            off[7], ln[7] = off[3], ln[3]          # an own payload repeated later
    elif case == "all_alias":
        off = np.full(20_000, 64, dtype=np.uint64)
        ln = np.full(20_000, 100, dtype=np.uint64)
    elif case == "zero_len":
        off = rng.integers(0, 50, 30_000).astype(np.uint64) * np.uint64(16)
        ln = np.where(rng.random(30_000) < 0.5, 0, 16).astype(np.uint64)
    else:
        off = rng.integers(0, 5_000, 40_000).astype(np.uint64)
        ln = rng.integers(0, 3, 40_000).astype(np.uint64)
    got = alias_first(off, ln)
    exp = _first_ref(off, ln)
    assert np.array_equal(got, exp)


def _dpp_checker():
    import importlib.util
    import os
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "check_dpp_hazards.py")
    spec = importlib.util.spec_from_file_location("check_dpp_hazards", p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_dpp_hazard_checker_flags_a_close_write():
    """The checker itself: a VALU write of the DPP source one instruction before
    is a hazard, two instructions or an s_nop 0 + one instruction before is not."""
    m = _dpp_checker()
    body = ["f:", "v_add3_u32 v90, v79, v59, v91", "v_bitop3_b32 v91, v78, v61, v60 bitop3:0xe8",
            "v_add_u32_e32 v79, v79, v91"]
    ok = body + ["v_add_u32_dpp v79, v59, v90 row_mirror row_mask:0xf bank_mask:0x3", "s_nop 0",
                 "v_add_u32_dpp v79, v90, v79 row_mirror row_mask:0xf bank_mask:0xc"]
    assert m.check(ok) == (2, [])
    bad = ["f:", "v_add3_u32 v90, v79, v59, v91", "v_add_u32_e32 v79, v79, v91",
           "v_add_u32_dpp v79, v90, v79 row_mirror row_mask:0xf bank_mask:0xc"]
    n, hz = m.check(bad)
    assert n == 1 and len(hz) == 1 and "1 wait state" in hz[0]
    assert len(m.check(["f:", "v_add_u32_dpp v1, v2, v3 row_mirror"])[1]) == 1   # block start: unknown


def test_no_dpp_read_hazard_in_device_code():
    """k_digest_chain2's DPP adds are inline asm (the compiler's hazard recognizer
    does not see them): every DPP of the built library has its 2 wait states."""
    import os
    m = _dpp_checker()
    if not os.path.exists(f"{m.LLVM}/llvm-objdump"):
        pytest.skip("no ROCm llvm-objdump")
    n, hz = m.check(m.disassemble(L.LIB_PATH))
    assert n >= 128 and hz == [], hz[:5]


def test_device_entry_points_validate_tensors_before_the_call():
    """engine.*_device take raw device pointers: wrong device, dtype width,
    contiguity or a short out must raise before anything reaches the C ABI."""
    import torch
    from mirbft_amd.engine import Engine
    eng = Engine.__new__(Engine)      # no context needed: validation runs first
    eng._dev_index = 0
    eng._ctx = None

    class NoCall:
        def __getattr__(self, name):
            raise AssertionError(f"{name} called")
    eng._lib = NoCall()
    arena = torch.zeros(128, dtype=torch.uint8)
    off = torch.zeros(2, dtype=torch.int64)
    out = torch.zeros((2, 32), dtype=torch.uint8)
    with pytest.raises(ValueError, match="cuda:0"):
        eng.digest_batch_device(arena, off, off, out)
    with pytest.raises(ValueError, match="cuda:0"):
        eng.digest_batch_device_planned(arena, off, off, out)
    with pytest.raises(ValueError, match="cuda:0"):
        eng.digest_of_digests_device(arena.view(-1, 32), off.int(), off, out)


def test_stats_structs_match_the_header(tmp_path):
    """The ctypes mirrors of msha_stats / msha_shard_stats / msha_clock_info have the
    C layout of include/mirsha.h (ABI 10 appended launches_chain2/chain8)."""
    import ctypes
    import subprocess
    src = tmp_path / "layout.c"
    names = {"msha_stats": (L.MshaStats, "launches_lane_ws"), "msha_shard_stats": (L.MshaShardStats, "plan_kernel_ms"),
             "msha_clock_info": (L.MshaClockInfo, "blocks_per_lane")}
    body = "".join('printf("%%s %%zu %%zu\\n", "%s", sizeof(%s), offsetof(%s, %s));\n' % (n, n, n, last)
                   for n, (_, last) in names.items())
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "mirsha.h"\nint main(void) {\n%s return 0;\n}\n'
                   % body)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    for line in filter(None, out):
        n, size, off = line.split()
        cls, last = names[n]
        assert ctypes.sizeof(cls) == int(size), n
        assert getattr(cls, last).offset == int(off), n
