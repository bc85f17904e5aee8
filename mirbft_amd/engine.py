"""Python handle on a libmirsha context (one or more GPUs).

``Engine`` is a thin, allocation-light wrapper over the C ABI
(include/mirsha.h). Host-memory calls take numpy arrays; device-resident calls
take torch tensors already on the GPU (``torch`` supplies device memory and
streams only -- all hashing happens in the HIP kernels of libmirsha.so).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib as L


class MshaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libmirsha error {code}: {msg}")
        self.code = code


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def blocks_for_len(length: int) -> int:
    """FIPS 180-4 padded block count of an L-byte message (host-only helper)."""
    return int(L.lib().msha_blocks_for_len(int(length)))


def partition_by_blocks(lengths: np.ndarray, n_shards: int) -> np.ndarray:
    """Contiguous shard bounds with near-equal cumulative block counts."""
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    bounds = np.zeros(n_shards + 1, dtype=np.uint64)
    arg = lengths if lengths.size else np.zeros(1, dtype=np.uint64)
    rc = L.lib().msha_partition_by_blocks(_p(arg, ctypes.c_uint64), lengths.size, n_shards,
                                          _p(bounds, ctypes.c_uint64))
    if rc != L.MSHA_OK:
        raise MshaError(rc, "partition_by_blocks")
    return bounds


def order_by_blocks(lengths: np.ndarray) -> np.ndarray:
    """Permutation ordering messages by descending block count (for d_order)."""
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    order = np.zeros(max(lengths.size, 1), dtype=np.uint32)
    arg = lengths if lengths.size else np.zeros(1, dtype=np.uint64)
    rc = L.lib().msha_order_by_blocks(_p(arg, ctypes.c_uint64), lengths.size, _p(order, ctypes.c_uint32))
    if rc != L.MSHA_OK:
        raise MshaError(rc, "order_by_blocks")
    return order[: lengths.size]


def alias_first(off: np.ndarray, length: np.ndarray) -> np.ndarray:
    """first[i] = smallest j <= i with the same (off, len) (host-only helper)."""
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint64)
    first = np.zeros(max(off.size, 1), dtype=np.uint64)
    a = off if off.size else np.zeros(1, dtype=np.uint64)
    b = length if length.size else np.zeros(1, dtype=np.uint64)
    rc = L.lib().msha_alias_first(_p(a, ctypes.c_uint64), _p(b, ctypes.c_uint64), off.size,
                                  _p(first, ctypes.c_uint64))
    if rc != L.MSHA_OK:
        raise MshaError(rc, "alias_first")
    return first[: off.size]


def device_count() -> int:
    n = ctypes.c_int(0)
    L.lib().msha_device_count(ctypes.byref(n))
    return n.value


class Engine:
    """A libmirsha context on the GPUs in ``device_mask`` (bit i = device i)."""

    def __init__(self, device_mask: int = 1):
        self._lib = L.lib()
        ctx = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = self._lib.msha_ctx_create_err(device_mask, ctypes.byref(ctx), err, len(err))
        if rc != L.MSHA_OK:
            raise MshaError(rc, err.value.decode())
        self._ctx = ctx

    # -- lifecycle -------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None):
            for p in getattr(self, "_pinned", []):
                self._lib.msha_pinned_free(self._ctx, p)
            self._pinned = []
            self._lib.msha_ctx_destroy(self._ctx)
            self._ctx = None

    def pinned_empty(self, nbytes: int) -> np.ndarray:
        """A uint8 numpy array in page-locked host memory (msha_pinned_alloc).
        Packing a batch into it (16-byte aligned message starts) lets
        digest_batch DMA it as is. Valid until close()."""
        p = ctypes.c_void_p()
        self._check(self._lib.msha_pinned_alloc(self._ctx, max(int(nbytes), 1), ctypes.byref(p)))
        if not hasattr(self, "_pinned"):
            self._pinned = []
        self._pinned.append(p.value)
        buf = (ctypes.c_uint8 * max(int(nbytes), 1)).from_address(p.value)
        return np.frombuffer(buf, dtype=np.uint8, count=int(nbytes))

    def pinned_free(self, a: np.ndarray) -> None:
        """Release a buffer from pinned_empty (by its base address)."""
        addr = a.__array_interface__["data"][0]
        if addr in getattr(self, "_pinned", []):
            self._pinned.remove(addr)
            self._check(self._lib.msha_pinned_free(self._ctx, addr))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        if rc != L.MSHA_OK:
            buf = ctypes.create_string_buffer(512)
            self._lib.msha_last_error_copy(self._ctx, buf, len(buf))   # under the context's lock
            raise MshaError(rc, buf.value.decode())

    def set_kernel_policy(self, policy: str) -> None:
        """"auto" (default), "lane" (one lane per message) or "coop" (cooperative chaining)."""
        code = {"auto": L.MSHA_KERNEL_AUTO, "lane": L.MSHA_KERNEL_LANE, "coop": L.MSHA_KERNEL_COOP}[policy]
        self._check(self._lib.msha_set_kernel_policy(self._ctx, code))

    def stats(self) -> dict:
        s = L.MshaStats()
        self._check(self._lib.msha_get_stats(self._ctx, ctypes.byref(s)))
        return {name: getattr(s, name) for name, _ in L.MshaStats._fields_}

    def shard_stats(self) -> list[dict]:
        """Per-GPU (per-shard) figures of the last host-memory call."""
        n = ctypes.c_uint32(0)
        self._check(self._lib.msha_shard_count(self._ctx, ctypes.byref(n)))
        out = []
        for i in range(n.value):
            s = L.MshaShardStats()
            self._check(self._lib.msha_get_shard_stats(self._ctx, i, ctypes.byref(s)))
            out.append({name: getattr(s, name) for name, _ in L.MshaShardStats._fields_})
        return out

    # -- host-memory entry points -----------------------------------------
    def digest_batch(self, arena: np.ndarray, off: np.ndarray, length: np.ndarray,
                     out: Optional[np.ndarray] = None) -> np.ndarray:
        """out[i] = SHA-256(arena[off[i] : off[i]+len[i]]) -> uint8 [n, 32]
        (``out``: an optional caller-owned C-contiguous uint8 [n, 32] result buffer)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8).reshape(-1)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        n = off.size
        if out is None:
            out = np.empty((n, 32), dtype=np.uint8)
        elif out.shape != (n, 32) or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous uint8 array of shape (n, 32)")
        if n == 0:
            return out
        ap = arena if arena.size else np.zeros(1, dtype=np.uint8)
        self._check(self._lib.msha_digest_batch(self._ctx, _p(ap, ctypes.c_uint8), arena.size,
                                                _p(off, ctypes.c_uint64), _p(length, ctypes.c_uint64),
                                                n, _p(out, ctypes.c_uint8)))
        return out

    def hash_actions_packed(self, arena: np.ndarray, part_off: np.ndarray, part_len: np.ndarray,
                            action_part_begin: np.ndarray) -> np.ndarray:
        """msha_hash_actions over a packed arena -> uint8 [n_actions, 32]."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8).reshape(-1)
        part_off = np.ascontiguousarray(part_off, dtype=np.uint64)
        part_len = np.ascontiguousarray(part_len, dtype=np.uint64)
        begin = np.ascontiguousarray(action_part_begin, dtype=np.uint64)
        n_actions = begin.size - 1
        out = np.empty((max(n_actions, 0), 32), dtype=np.uint8)
        if n_actions <= 0:
            return out
        ap = arena if arena.size else np.zeros(1, dtype=np.uint8)
        po = part_off if part_off.size else np.zeros(1, dtype=np.uint64)
        pl = part_len if part_len.size else np.zeros(1, dtype=np.uint64)
        self._check(self._lib.msha_hash_actions(self._ctx, _p(ap, ctypes.c_uint8), arena.size,
                                                _p(po, ctypes.c_uint64), _p(pl, ctypes.c_uint64),
                                                part_off.size, _p(begin, ctypes.c_uint64), n_actions,
                                                _p(out, ctypes.c_uint8)))
        return out

    def hash_actions(self, actions: Sequence[Sequence[bytes]]) -> list[bytes]:
        """One digest per action = SHA-256(concat(parts)), in input order."""
        arena, part_off, part_len, begin = pack_parts(actions)
        out = self.hash_actions_packed(arena, part_off, part_len, begin)
        return [bytes(r) for r in out]

    def digest_of_digests(self, table: np.ndarray, idx: np.ndarray, begin: np.ndarray) -> np.ndarray:
        table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1, 32)
        idx = np.ascontiguousarray(idx, dtype=np.uint32)
        begin = np.ascontiguousarray(begin, dtype=np.uint64)
        n = begin.size - 1
        out = np.empty((n, 32), dtype=np.uint8)
        if n <= 0:
            return out
        tp = table if table.size else np.zeros((1, 32), dtype=np.uint8)
        ip = idx if idx.size else np.zeros(1, dtype=np.uint32)
        self._check(self._lib.msha_digest_of_digests(self._ctx, _p(tp, ctypes.c_uint8), table.shape[0],
                                                     _p(ip, ctypes.c_uint32), idx.size,
                                                     _p(begin, ctypes.c_uint64), n,
                                                     _p(out, ctypes.c_uint8)))
        return out

    # -- device-resident entry points (torch tensors on the GPU) ----------
    @staticmethod
    def _stream_ptr(stream) -> Optional[int]:
        if stream is None:
            return None
        return int(getattr(stream, "cuda_stream", stream))

    def _device_index(self) -> int:
        n = ctypes.c_uint32(0)
        self._check(self._lib.msha_shard_count(self._ctx, ctypes.byref(n)))
        s = L.MshaShardStats()
        self._check(self._lib.msha_get_shard_stats(self._ctx, 0, ctypes.byref(s)))
        return int(s.device)

    def _check_device_args(self, n: int, out, **tensors) -> None:
        """The *_device entry points take raw device pointers: check here what
        the C ABI cannot -- every tensor contiguous on the context's first GPU,
        8-byte integers for off/len/begin, 4-byte for order/idx, out a uint8
        buffer of at least 32 n bytes -- so a mismatch raises instead of
        reading or writing out of bounds on the GPU."""
        import torch
        dev = getattr(self, "_dev_index", None)
        if dev is None:
            dev = self._dev_index = self._device_index()
        sizes = {"off": 8, "length": 8, "begin": 8, "order": 4, "idx": 4, "arena": 1, "table": 1}
        for name, t in list(tensors.items()) + [("out", out)]:
            if t is None:
                continue
            if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.device.index != dev:
                raise ValueError(f"{name} must be a torch tensor on cuda:{dev} (the context's first GPU)")
            if not t.is_contiguous():
                raise ValueError(f"{name} must be contiguous")
            want = 1 if name == "out" else sizes[name]
            if t.element_size() != want or t.is_floating_point():
                raise ValueError(f"{name} must hold {want}-byte integers (got {t.dtype})")
        for name in ("off", "length", "order"):
            t = tensors.get(name)
            if t is not None and t.numel() != n:
                raise ValueError(f"{name} has {t.numel()} entries, expected {n}")
        if out.numel() < 32 * n:
            raise ValueError(f"out holds {out.numel()} bytes, needs {32 * n}")

    def digest_batch_device(self, arena, off, length, out, stream=None, order=None) -> None:
        self._check_device_args(off.numel(), out, arena=arena, off=off, length=length, order=order)
        self._check(self._lib.msha_digest_batch_device(self._ctx, arena.data_ptr(), off.data_ptr(),
                                                       length.data_ptr(),
                                                       None if order is None else order.data_ptr(),
                                                       off.numel(), out.data_ptr(), self._stream_ptr(stream)))

    def digest_batch_device_planned(self, arena, off, length, out, stream=None, fold: bool = False) -> None:
        """msha_digest_batch_device_planned: lane order (and, with fold, alias
        folding) planned on the GPU inside the call's launches."""
        self._check_device_args(off.numel(), out, arena=arena, off=off, length=length)
        self._check(self._lib.msha_digest_batch_device_planned(self._ctx, arena.data_ptr(), off.data_ptr(),
                                                               length.data_ptr(), off.numel(),
                                                               1 if fold else 0, out.data_ptr(),
                                                               self._stream_ptr(stream)))

    def digest_uniform_device(self, arena, stride: int, msg_len: int, n: int, out, stream=None) -> None:
        self._check_device_args(n, out, arena=arena)
        self._check(self._lib.msha_digest_uniform_device(self._ctx, arena.data_ptr(), stride, msg_len, n,
                                                         out.data_ptr(), self._stream_ptr(stream)))

    def digest_of_digests_device(self, table, idx, begin, out, stream=None) -> None:
        self._check_device_args(begin.numel() - 1, out, table=table, idx=idx, begin=begin)
        self._check(self._lib.msha_digest_of_digests_device(self._ctx, table.data_ptr(), idx.data_ptr(),
                                                            begin.data_ptr(), begin.numel() - 1,
                                                            out.data_ptr(), self._stream_ptr(stream)))

    def clock_probe(self, blocks_per_lane: int = 48) -> dict:
        """msha_clock_probe: the clock the first GPU holds under the hash
        kernels' instruction mix (in-kernel s_memtime / s_memrealtime)."""
        c = L.MshaClockInfo()
        self._check(self._lib.msha_clock_probe(self._ctx, int(blocks_per_lane), ctypes.byref(c)))
        return {name: getattr(c, name) for name, _ in L.MshaClockInfo._fields_}

    def device_status(self) -> None:
        self._check(self._lib.msha_device_status(self._ctx))


def pack_parts(actions: Sequence[Sequence[bytes]]):
    """Pack [][]byte parts into (arena, part_off, part_len, action_part_begin),
    the layout a cgo adapter hands to msha_hash_actions."""
    parts = [bytes(p) for a in actions for p in a]
    lens = np.fromiter((len(p) for p in parts), dtype=np.uint64, count=len(parts))
    offs = np.zeros(len(parts), dtype=np.uint64)
    if len(parts) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    arena = np.frombuffer(b"".join(parts), dtype=np.uint8)
    begin = np.zeros(len(actions) + 1, dtype=np.uint64)
    if actions:
        begin[1:] = np.cumsum([len(a) for a in actions])
    return arena, offs, lens, begin
