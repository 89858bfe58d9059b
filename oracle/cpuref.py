"""ctypes binding of oracle/libcpuref.so — the SIMD + threaded C++ restatement of the
reference's CPU encode structure (klauspost/reedsolomon v1.11.8 + minio/highwayhash
v1.0.2, blocks sequential, encode split by byte range over T threads, then the k+m
HighwayHash-256 sums; oracle/cpu_ref.cpp).

TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it, and the full-size GPU
tests use it as the fast checker of whole batches; tests/test_cpuref_pin.py pins its
parity rows and sums byte for byte to the scalar oracle, oracle/zs3_oracle.c).  Never
used by the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libcpuref.so")
        if not os.path.exists(path):
            from . import oracle_c
            oracle_c.build()
        L = C.CDLL(path)
        L.cpuref_isa.restype = C.c_char_p
        L.cpuref_encode_hash.restype = C.c_int64
        L.cpuref_encode_hash.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                         C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int]
        L.cpuref_hh256.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
        _LIB = L
    return _LIB


def isa() -> str:
    return lib().cpuref_isa().decode()


def threads_available() -> int:
    """CPU threads this process may use: the affinity mask, capped by
    OMP_NUM_THREADS when the environment sets one (the GPU box's CPU share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def encode_hash(k: int, m: int, matrix: np.ndarray, data: np.ndarray, block_len: int, n_blocks: int,
                data_stride: int, parity: np.ndarray, parity_stride: int, sums: np.ndarray | None,
                key: bytes, threads: int) -> int:
    """Encode + HH256 n_blocks blocks (block b at data[b*data_stride:]); parity row r of
    block b at parity[b*parity_stride + r*S:], sums (k+m)*32 per block.  Returns S."""
    mat = np.ascontiguousarray(matrix, dtype=np.uint8)
    kb = C.create_string_buffer(key, 32)
    return int(lib().cpuref_encode_hash(k, m, mat.ctypes.data, data.ctypes.data, block_len, n_blocks, data_stride,
                                        parity.ctypes.data, parity_stride,
                                        sums.ctypes.data if sums is not None else None, kb, threads))
