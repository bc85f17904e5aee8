"""CPU oracle for the MirBFT hash path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module. It is the parity checker, never the thing measured
or shipped: ``mirbft_amd`` does not import it and has no CPU fallback.

Two restatements of the same reference behaviour, checked against each other and
against the committed FIPS 180-4 known answers (tests/golden/kat.json):

* ``liboracle_sha256.so`` built from ``oracle/sha256_oracle.c`` (plain scalar C),
  restating ``processor.ProcessHashActions`` (/root/reference/pkg/processor/serial.go:180-198)
  over Go ``crypto/sha256`` (FIPS 180-4; Go stdlib, not in the reference tree).
* ``py_sha256`` below: a pure-Python FIPS 180-4 restatement, for small inputs.
* ``liboracle_openssl.so`` built from ``oracle/sha256_openssl.c``: the same loop
  over OpenSSL libcrypto (SHA-NI where the CPU has it), multi-threaded; a third
  cross-check and bench.py's strongest CPU baseline.

The reference itself (Go) cannot be built or run in this image (no ``go``), so
parity is pinned by the FIPS 180-4 known-answer vectors plus an independent
implementation (``hashlib`` = OpenSSL 3.0.2) on every golden fixture.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle_sha256.so")
_SSL_PATH = os.path.join(_HERE, "build", "liboracle_openssl.so")
_lib = None
_ssl = None


def build() -> str:
    """Compile the C oracle (gcc) into oracle/build/."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.oracle_sha256.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.oracle_digest_batch.argtypes = [u8p, u64p, u64p, ctypes.c_uint64, u8p]
        L.oracle_process_hash_actions.argtypes = [u8p, u64p, u64p, u64p, ctypes.c_uint64, u8p]
        L.oracle_digest_of_digests.argtypes = [u8p, u32p, u64p, ctypes.c_uint64, u8p]
        for f in (L.oracle_sha256, L.oracle_digest_batch, L.oracle_process_hash_actions,
                  L.oracle_digest_of_digests):
            f.restype = None
        _lib = L
    return _lib


def ssl_lib():
    global _ssl
    if _ssl is None:
        if not os.path.exists(_SSL_PATH):
            build()
        L = ctypes.CDLL(_SSL_PATH)
        L.openssl_digest_batch.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
                                           ctypes.POINTER(ctypes.c_uint8), ctypes.c_int]
        L.openssl_digest_batch.restype = ctypes.c_int
        _ssl = L
    return _ssl


def openssl_digest_batch(arena: np.ndarray, off: np.ndarray, length: np.ndarray, threads: int = 1) -> np.ndarray:
    """digest_batch via OpenSSL libcrypto over `threads` threads; uint8 [n, 32]."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    if arena.size == 0:
        arena = np.zeros(1, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint64)
    n = off.size
    out = np.zeros((n, 32), dtype=np.uint8)
    if n == 0:
        return out
    rc = ssl_lib().openssl_digest_batch(_p(arena, ctypes.c_uint8), _p(off, ctypes.c_uint64),
                                        _p(length, ctypes.c_uint64), n, _p(out, ctypes.c_uint8), threads)
    if rc != 0:
        raise RuntimeError("openssl_digest_batch failed")
    return out


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def sha256(data: bytes) -> bytes:
    buf = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    lib().oracle_sha256(_p(buf, ctypes.c_uint8), len(data), _p(out, ctypes.c_uint8))
    return out.tobytes()


def digest_batch(arena: np.ndarray, off: np.ndarray, length: np.ndarray) -> np.ndarray:
    """One digest per (off, len) message; returns uint8 [n, 32]."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    if arena.size == 0:
        arena = np.zeros(1, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint64)
    n = off.size
    out = np.zeros((n, 32), dtype=np.uint8)
    lib().oracle_digest_batch(_p(arena, ctypes.c_uint8), _p(off, ctypes.c_uint64),
                              _p(length, ctypes.c_uint64), n, _p(out, ctypes.c_uint8))
    return out


def process_hash_actions(actions: Sequence[Sequence[bytes]]) -> list[bytes]:
    """serial.go:180-198 over Python parts lists: one digest per action, in order."""
    parts = [bytes(p) for a in actions for p in a]
    arena = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8)
    lens = np.array([len(p) for p in parts], dtype=np.uint64)
    offs = np.zeros(len(parts), dtype=np.uint64)
    if len(parts) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    begin = np.zeros(len(actions) + 1, dtype=np.uint64)
    begin[1:] = np.cumsum([len(a) for a in actions])
    out = np.zeros((len(actions), 32), dtype=np.uint8)
    if lens.size == 0:
        offs = np.zeros(1, dtype=np.uint64)
        lens = np.zeros(1, dtype=np.uint64)
    lib().oracle_process_hash_actions(_p(arena, ctypes.c_uint8), _p(offs, ctypes.c_uint64),
                                      _p(lens, ctypes.c_uint64), _p(begin, ctypes.c_uint64),
                                      len(actions), _p(out, ctypes.c_uint8))
    return [bytes(r) for r in out]


def digest_of_digests(table: np.ndarray, idx: np.ndarray, begin: np.ndarray) -> np.ndarray:
    table = np.ascontiguousarray(table, dtype=np.uint8).reshape(-1)
    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    begin = np.ascontiguousarray(begin, dtype=np.uint64)
    n = begin.size - 1
    out = np.zeros((n, 32), dtype=np.uint8)
    if idx.size == 0:
        idx = np.zeros(1, dtype=np.uint32)
    if table.size == 0:
        table = np.zeros(32, dtype=np.uint8)
    lib().oracle_digest_of_digests(_p(table, ctypes.c_uint8), _p(idx, ctypes.c_uint32),
                                   _p(begin, ctypes.c_uint64), n, _p(out, ctypes.c_uint8))
    return out


# ---------------------------------------------------------------------------
# Pure-Python FIPS 180-4 restatement (small inputs only).
# ---------------------------------------------------------------------------
_K = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2,
]
_IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
_M = 0xFFFFFFFF


def _rotr(x: int, n: int) -> int:
    return ((x >> n) | (x << (32 - n))) & _M


def py_sha256(data: bytes) -> bytes:
    """FIPS 180-4 section 6.2 with section 5.1.1 padding, pure Python."""
    ml = len(data) * 8
    msg = bytes(data) + b"\x80" + b"\0" * ((55 - len(data)) % 64) + ml.to_bytes(8, "big")
    h = list(_IV)
    for blk in range(0, len(msg), 64):
        w = [int.from_bytes(msg[blk + 4 * t: blk + 4 * t + 4], "big") for t in range(16)]
        for t in range(16, 64):
            s0 = _rotr(w[t - 15], 7) ^ _rotr(w[t - 15], 18) ^ (w[t - 15] >> 3)
            s1 = _rotr(w[t - 2], 17) ^ _rotr(w[t - 2], 19) ^ (w[t - 2] >> 10)
            w.append((s1 + w[t - 7] + s0 + w[t - 16]) & _M)
        a, b, c, d, e, f, g, hh = h
        for t in range(64):
            S1 = _rotr(e, 6) ^ _rotr(e, 11) ^ _rotr(e, 25)
            ch = (e & f) ^ (~e & g)
            T1 = (hh + S1 + ch + _K[t] + w[t]) & _M
            S0 = _rotr(a, 2) ^ _rotr(a, 13) ^ _rotr(a, 22)
            maj = (a & b) ^ (a & c) ^ (b & c)
            hh, g, f, e, d, c, b, a = g, f, e, (d + T1) & _M, c, b, a, (T1 + S0 + maj) & _M
        h = [(x + y) & _M for x, y in zip(h, (a, b, c, d, e, f, g, hh))]
    return b"".join(x.to_bytes(4, "big") for x in h)
