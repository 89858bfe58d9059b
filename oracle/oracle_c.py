"""ctypes binding of oracle/liboracle.so (the scalar C restatement).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker.  Never used by the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", _HERE, "all"])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        u8p = C.POINTER(C.c_uint8)
        L.oracle_build_matrix.argtypes = [C.c_int, C.c_int, u8p]
        L.oracle_gf_invert.argtypes = [u8p, C.c_int, u8p]
        L.oracle_encode_data.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_int64, u8p]
        L.oracle_encode_data.restype = C.c_int64
        L.oracle_reconstruct.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_int64, u8p, C.c_int]
        L.oracle_hh256.argtypes = [u8p, u8p, C.c_size_t, u8p]
        L.oracle_hh64.argtypes = [u8p, u8p, C.c_size_t]
        L.oracle_hh64.restype = C.c_uint64
        L.oracle_hh256_batch.argtypes = [u8p, u8p, C.c_size_t, C.c_size_t, C.c_size_t, u8p]
        L.oracle_fill.argtypes = [C.c_uint64, C.c_uint64, u8p, C.c_size_t]
        L.oracle_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.oracle_gf_mul.restype = C.c_uint8
        L.oracle_ceil_frac.argtypes = [C.c_int64, C.c_int64]
        L.oracle_ceil_frac.restype = C.c_int64
        _LIB = L
    return _LIB


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _u8(b) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(b), dtype=np.uint8)) if not isinstance(b, np.ndarray) \
        else np.ascontiguousarray(b, dtype=np.uint8)


def build_matrix(k: int, m: int) -> np.ndarray:
    out = np.zeros((k + m) * k, dtype=np.uint8)
    rc = lib().oracle_build_matrix(k, m, _p(out))
    if rc:
        raise ValueError(f"oracle_build_matrix rc={rc}")
    return out.reshape(k + m, k)


def encode_data(k: int, m: int, data, matrix: np.ndarray | None = None) -> np.ndarray:
    """EncodeData on one block -> (k+m, per) array (cmd/erasure-coding.go:77)."""
    if matrix is None:
        matrix = build_matrix(k, m)
    d = _u8(data)
    n = len(d)
    if n == 0:
        return np.zeros((k + m, 0), dtype=np.uint8)
    per = -(-n // k)
    out = np.zeros((k + m) * per, dtype=np.uint8)
    mat = np.ascontiguousarray(matrix, dtype=np.uint8)
    r = lib().oracle_encode_data(_p(mat), k, m, _p(d) if n else None, n, _p(out))
    assert r == per
    return out.reshape(k + m, per)


def reconstruct(k: int, m: int, shards: np.ndarray, present, data_only: bool,
                matrix: np.ndarray | None = None) -> int:
    """In-place reconstruct of a (k+m, per) array; returns the error code."""
    if matrix is None:
        matrix = build_matrix(k, m)
    pres = np.array([1 if p else 0 for p in present], dtype=np.uint8)
    mat = np.ascontiguousarray(matrix, dtype=np.uint8)
    assert shards.flags.c_contiguous
    return lib().oracle_reconstruct(_p(mat), k, m, _p(shards), shards.shape[1], _p(pres), int(data_only))


def hh256(key: bytes, msg) -> bytes:
    k = _u8(key)
    d = _u8(msg)
    out = np.zeros(32, dtype=np.uint8)
    lib().oracle_hh256(_p(k), _p(d) if len(d) else _p(np.zeros(1, np.uint8)), len(d), _p(out))
    return out.tobytes()


def hh64(key: bytes, msg) -> int:
    k = _u8(key)
    d = _u8(msg)
    return int(lib().oracle_hh64(_p(k), _p(d) if len(d) else _p(np.zeros(1, np.uint8)), len(d)))


def hh256_rows(key: bytes, rows: np.ndarray) -> np.ndarray:
    """HH256 of each row of a 2-D uint8 array -> (rows, 32)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint8)
    n, ln = rows.shape
    out = np.zeros((n, 32), dtype=np.uint8)
    k = _u8(key)
    src = rows if rows.size else np.zeros(1, np.uint8)
    lib().oracle_hh256_batch(_p(k), _p(src), n, ln, ln, _p(out))
    return out


def fill(seed: int, obj: int, nbytes: int) -> np.ndarray:
    out = np.zeros(max(nbytes, 1), dtype=np.uint8)
    lib().oracle_fill(seed, obj, _p(out), nbytes)
    return out[:nbytes]
