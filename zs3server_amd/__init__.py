"""zs3server_amd — MI355X-native erasure-shard + bitrot-hash data path.

Python binding of the C ABI in include/zs3gpu.h (libzs3gpu.so, built for gfx950).
The Go server binds the same ABI through cgo; this module is the
test/bench host and mirrors the reference's Erasure API in `erasure.py` and the
streaming bitrot format in `bitrot.py`.

There is no CPU fallback: if libzs3gpu.so is missing or fails to load, import of
`lib()` raises.  Device buffers are torch tensors on a ROCm device (or raw
device pointers as ints).

Two builds of the same ABI: libzs3gpu.so (the product: tuned default kernels and the
generic fallbacks) and libzs3gpu_diag.so (the same plus experimental kernel variants
and the zs3_debug_* calls of include/zs3gpu_diag.h).  Everything here runs on the
product library unless a `diag()` context is active in this thread.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading

try:  # load torch's HIP runtime first so the library binds to the same one
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libzs3gpu.so")
DIAG_LIB_PATH = os.path.join(_HERE, "libzs3gpu_diag.so")

ZS3_OK = 0
ERRORS = {
    -1: "ErrInvShardNum", -2: "ErrMaxShardNum", -3: "ErrTooFewShards", -4: "ErrShardNoData",
    -5: "ErrShardSize", -6: "ErrShortData", -7: "errFileCorrupt", -8: "errInvalidArgument",
    -9: "device error", -10: "out of memory", -11: "matrix is singular",
}

# cmd/bitrot.go:37
MAGIC_HH256_KEY = bytes.fromhex("4be734fa8e238acd263e83e6bb968552040f935da39f441497e09d1322de36a0")

# Every symbol include/zs3gpu.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "zs3_strerror", "zs3_version", "zs3_device_count", "zs3_set_device", "zs3_dev_alloc",
    "zs3_dev_free", "zs3_host_alloc", "zs3_host_free", "zs3_memcpy_h2d", "zs3_memcpy_d2h",
    "zs3_stream_sync", "zs3_codec_new", "zs3_codec_free", "zs3_codec_matrix", "zs3_shard_size",
    "zs3_shard_file_size", "zs3_shard_file_offset", "zs3_bitrot_shard_file_size",
    "zs3_encode_batch", "zs3_reconstruct_batch", "zs3_verify_reconstruct_batch", "zs3_hh256_batch",
    "zs3_hh256_verify_batch",
    "zs3_fill_batch", "zs3_encode_data", "zs3_decode_data_blocks", "zs3_hh256", "zs3_selftest",
    "zs3_stream_encode", "zs3_md5_batch", "zs3_sha256_batch", "zs3_etag_multipart",
    "zs3_last_path", "zs3_reconstruct_batch_masks", "zs3_verify_reconstruct_batch_masks",
    "zs3_hh256_batch_ragged", "zs3_bitrot_verify_file_batch", "zs3_codec_params",
    "zs3_queue_new", "zs3_queue_free", "zs3_queue_submit_encode", "zs3_queue_submit_decode", "zs3_req_wait",
    "zs3_queue_flush", "zs3_queue_stats", "zs3_queue_zero_copy_blocks", "zs3_queue_encode_data", "zs3_queue_decode_data_blocks",
    "zs3_stream_encode_multi", "zs3_split_range", "zs3_md5_parts", "zs3_sha256_parts",
    "zs3_queue_device_stats", "zs3_stream_decode", "zs3_path_mask",
    "zs3_pool_limit",
]
# include/zs3gpu_diag.h: exported by the diagnostics build only
DIAG_EXPORTS = ["zs3_debug_set_variant", "zs3_debug_set_buffer", "zs3_debug_encode_layout_ok",
                "zs3_debug_queue_timers"]


class ZS3Error(Exception):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        self.name = ERRORS.get(code, f"error {code}")
        super().__init__(f"{what}: {self.name} ({code})" if what else f"{self.name} ({code})")


_L = None        # product library
_LD = None       # diagnostics library
_tls = threading.local()


def lib():
    """The library this thread uses: the product libzs3gpu.so, or the diagnostics
    build inside a `diag()` context.  Raises if absent: there is no fallback."""
    d = getattr(_tls, "diag", None)
    return d if d is not None else product_lib()


def product_lib():
    global _L
    if _L is None:
        _L = _load(LIB_PATH)
    return _L


def diag_lib():
    """libzs3gpu_diag.so: the product ABI plus the experimental kernel variants."""
    global _LD
    if _LD is None:
        _LD = _load(DIAG_LIB_PATH)
        _LD.zs3_debug_set_variant.argtypes = [C.c_int]
        _LD.zs3_debug_set_buffer.argtypes = [C.c_void_p]
        i64 = C.c_int64
        _LD.zs3_debug_encode_layout_ok.argtypes = [C.c_void_p, i64, i64, i64, C.c_void_p, i64, i64]
    return _LD


@contextlib.contextmanager
def diag(variant: int = 0):
    """Run this thread's calls on the diagnostics build with fused-kernel `variant`
    (thread-local in the library too: other threads are unaffected)."""
    prev = getattr(_tls, "diag", None)
    L = diag_lib()
    _tls.diag = L
    L.zs3_debug_set_variant(variant)
    try:
        yield L
    finally:
        L.zs3_debug_set_variant(0)
        _tls.diag = prev


def _load(path):
    if not os.path.exists(path):
        raise ImportError(f"{path} not built — run __graft_entry__.build()")
    L = C.CDLL(path)
    vp, i64, u8p = C.c_void_p, C.c_int64, C.POINTER(C.c_uint8)
    L.zs3_strerror.restype = C.c_char_p
    L.zs3_strerror.argtypes = [C.c_int]
    L.zs3_codec_new.argtypes = [C.c_int, C.c_int, i64, C.POINTER(vp)]
    L.zs3_codec_free.argtypes = [vp]
    L.zs3_codec_free.restype = None
    L.zs3_codec_matrix.argtypes = [vp, u8p]
    for f in ("zs3_shard_size",):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = i64
    L.zs3_shard_file_size.argtypes = [vp, i64]
    L.zs3_shard_file_size.restype = i64
    L.zs3_shard_file_offset.argtypes = [vp, i64, i64, i64]
    L.zs3_shard_file_offset.restype = i64
    L.zs3_bitrot_shard_file_size.argtypes = [i64, i64]
    L.zs3_bitrot_shard_file_size.restype = i64
    L.zs3_encode_batch.argtypes = [vp, vp, i64, i64, i64, vp, i64, vp, vp]
    L.zs3_reconstruct_batch.argtypes = [vp, vp, i64, i64, i64, u8p, C.c_int, vp]
    L.zs3_verify_reconstruct_batch.argtypes = [vp, vp, i64, i64, i64, u8p, C.c_int, vp, vp, vp, vp]
    L.zs3_hh256_batch.argtypes = [vp, vp, i64, i64, i64, vp, vp]
    L.zs3_hh256_verify_batch.argtypes = [vp, vp, i64, i64, i64, vp, vp, vp]
    L.zs3_fill_batch.argtypes = [vp, i64, i64, i64, C.c_uint64, C.c_uint64, vp]
    L.zs3_encode_data.argtypes = [vp, vp, i64, i64, vp]
    L.zs3_encode_data.restype = i64
    L.zs3_decode_data_blocks.argtypes = [vp, vp, i64, u8p, C.c_int]
    L.zs3_hh256.argtypes = [vp, vp, i64, vp]
    L.zs3_device_count.argtypes = [C.POINTER(C.c_int)]
    L.zs3_set_device.argtypes = [C.c_int]
    L.zs3_stream_encode.argtypes = [vp, vp, i64, vp, vp, i64]
    L.zs3_stream_encode.restype = i64
    L.zs3_md5_batch.argtypes = [vp, i64, i64, vp, i64, vp, vp]
    L.zs3_sha256_batch.argtypes = [vp, i64, i64, vp, i64, vp, vp]
    L.zs3_md5_parts.argtypes = [vp, vp, vp, i64, vp, vp]
    L.zs3_sha256_parts.argtypes = [vp, vp, vp, i64, vp, vp]
    L.zs3_etag_multipart.argtypes = [vp, vp, vp, i64, vp]
    L.zs3_host_alloc.argtypes = [C.POINTER(vp), C.c_size_t]
    L.zs3_host_free.argtypes = [vp]
    L.zs3_reconstruct_batch_masks.argtypes = [vp, vp, i64, i64, i64, vp, C.c_int, vp, vp]
    L.zs3_verify_reconstruct_batch_masks.argtypes = [vp, vp, i64, i64, i64, vp, C.c_int, vp, vp, vp, vp, vp]
    L.zs3_hh256_batch_ragged.argtypes = [vp, vp, vp, i64, vp, vp]
    L.zs3_bitrot_verify_file_batch.argtypes = [vp, vp, i64, i64, i64, i64, i64, vp, vp, C.POINTER(C.c_int64), vp]
    L.zs3_codec_params.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(i64)]
    L.zs3_queue_new.argtypes = [vp, C.POINTER(QueueOpts), C.POINTER(vp)]
    L.zs3_queue_free.argtypes = [vp]
    L.zs3_queue_free.restype = None
    L.zs3_queue_submit_encode.argtypes = [vp, vp, i64, i64, vp, C.POINTER(vp)]
    L.zs3_queue_submit_decode.argtypes = [vp, vp, i64, vp, C.c_int, vp, vp, vp, C.POINTER(vp)]
    L.zs3_req_wait.argtypes = [vp]
    L.zs3_req_wait.restype = i64
    L.zs3_queue_flush.argtypes = [vp]
    L.zs3_queue_stats.argtypes = [vp, C.POINTER(i64), C.POINTER(i64)]
    L.zs3_queue_zero_copy_blocks.argtypes = [vp]
    L.zs3_queue_zero_copy_blocks.restype = i64
    L.zs3_queue_device_stats.argtypes = [vp, C.c_int, C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(i64)]
    L.zs3_queue_encode_data.argtypes = [vp, vp, i64, i64, vp]
    L.zs3_queue_encode_data.restype = i64
    L.zs3_queue_decode_data_blocks.argtypes = [vp, vp, i64, vp, C.c_int, vp, vp]
    L.zs3_stream_encode_multi.argtypes = [vp, vp, C.c_int, vp, i64, vp, vp, i64]
    L.zs3_stream_encode_multi.restype = i64
    L.zs3_stream_decode.argtypes = [vp, vp, i64, vp, C.c_int, vp, vp, vp, vp, i64]
    L.zs3_path_mask.argtypes = [C.c_int]
    L.zs3_path_mask.restype = C.c_uint32
    L.zs3_pool_limit.argtypes = [C.c_uint64]
    L.zs3_pool_limit.restype = i64
    L.zs3_stream_decode.restype = i64
    L.zs3_split_range.argtypes = [i64, C.c_int, C.c_int, C.POINTER(i64), C.POINTER(i64)]
    L.zs3_split_range.restype = None
    return L


class QueueOpts(C.Structure):
    """zs3_queue_opts (include/zs3gpu.h)."""
    _fields_ = [("device", C.c_int), ("max_batch", C.c_int), ("max_wait_us", C.c_int), ("slots", C.c_int),
                ("devices", C.POINTER(C.c_int)), ("n_devices", C.c_int)]


def _check(rc: int, what: str = "") -> int:
    if rc < 0:
        raise ZS3Error(int(rc), what)
    return rc


def _ptr(x, offset: int = 0):
    """Device pointer of a torch tensor (or an int address) plus a byte offset."""
    if x is None:
        return None
    if isinstance(x, int):
        return x + offset
    return x.data_ptr() + offset


def _stream(stream):
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _u8buf(a):
    import numpy as np
    arr = a if isinstance(a, np.ndarray) else np.frombuffer(a, dtype=np.uint8)
    return arr


class Codec:
    """Handle for one (k, m) coding matrix: the Erasure value of
    cmd/erasure-coding.go:35-73 (NewErasure's checks raise ZS3Error)."""

    def __init__(self, k: int, m: int, block_size: int = 1 << 20):
        L = lib()
        h = C.c_void_p()
        _check(L.zs3_codec_new(k, m, block_size, C.byref(h)), "NewErasure")
        self._L = L  # a codec belongs to the library that made it
        self._h = h
        self.k, self.m, self.block_size = k, m, block_size

    def __del__(self):
        h = getattr(self, "_h", None)
        L = getattr(self, "_L", None)
        if h is not None and h.value and L is not None:
            L.zs3_codec_free(h)
            self._h = None

    # ---- size arithmetic (erasure-coding.go:122-150) ----
    def shard_size(self) -> int:
        return self._L.zs3_shard_size(self._h)

    def shard_file_size(self, total: int) -> int:
        return self._L.zs3_shard_file_size(self._h, total)

    def shard_file_offset(self, start: int, length: int, total: int) -> int:
        return self._L.zs3_shard_file_offset(self._h, start, length, total)

    def matrix(self):
        import numpy as np
        out = np.zeros((self.k + self.m) * self.k, dtype=np.uint8)
        _check(self._L.zs3_codec_matrix(self._h, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.reshape(self.k + self.m, self.k)

    # ---- device-resident batches ----
    def encode_batch(self, data, data_stride: int, block_len: int, n_blocks: int, parity,
                     parity_stride: int, sums=None, parity_offset: int = 0, data_offset: int = 0,
                     stream=None) -> None:
        _check(self._L.zs3_encode_batch(self._h, _ptr(data, data_offset), data_stride, block_len, n_blocks,
                                      _ptr(parity, parity_offset), parity_stride, _ptr(sums),
                                      _stream(stream)), "encode_batch")

    def reconstruct_batch(self, shards, block_stride: int, shard_len: int, n_blocks: int, present,
                          data_only: bool, stream=None, offset: int = 0) -> None:
        pres = (C.c_uint8 * (self.k + self.m))(*[1 if p else 0 for p in present])
        _check(self._L.zs3_reconstruct_batch(self._h, _ptr(shards, offset), block_stride, shard_len, n_blocks,
                                           pres, 1 if data_only else 0, _stream(stream)), "reconstruct_batch")

    def verify_reconstruct_batch(self, shards, block_stride: int, shard_len: int, n_blocks: int, present,
                                 data_only: bool, expect, bad, sums_out=None, stream=None,
                                 offset: int = 0) -> None:
        """GET / heal pass (zs3_verify_reconstruct_batch): verify the k survivors
        against `expect` ([n][k+m][32] device), flag failures in `bad` ([n][k+m]
        int32 device), rebuild the missing shards in place, optionally hash them
        into `sums_out`."""
        pres = (C.c_uint8 * (self.k + self.m))(*[1 if p else 0 for p in present])
        _check(self._L.zs3_verify_reconstruct_batch(self._h, _ptr(shards, offset), block_stride, shard_len,
                                                  n_blocks, pres, 1 if data_only else 0, _ptr(expect), _ptr(bad),
                                                  _ptr(sums_out), _stream(stream)), "verify_reconstruct_batch")

    def reconstruct_batch_masks(self, shards, block_stride: int, shard_len: int, n_blocks: int, present,
                                data_only: bool, status=None, stream=None, offset: int = 0) -> int:
        """Per-block erasure patterns (zs3_reconstruct_batch_masks): `present` is an
        (n_blocks, k+m) array of flags.  Returns ZS3_OK or the first block's error;
        `status` (numpy int32, n_blocks) receives every block's status."""
        import numpy as np
        pres = np.ascontiguousarray(np.asarray(present, dtype=bool).astype(np.uint8).reshape(n_blocks, self.k + self.m))
        st = status if status is not None else np.zeros(n_blocks, np.int32)
        return int(self._L.zs3_reconstruct_batch_masks(self._h, _ptr(shards, offset), block_stride, shard_len,
                                                        n_blocks, pres.ctypes.data, 1 if data_only else 0,
                                                        st.ctypes.data, _stream(stream)))

    def verify_reconstruct_batch_masks(self, shards, block_stride: int, shard_len: int, n_blocks: int, present,
                                       data_only: bool, expect, bad, sums_out=None, status=None, stream=None,
                                       offset: int = 0) -> int:
        """GET / heal pass with per-block erasure patterns
        (zs3_verify_reconstruct_batch_masks); returns ZS3_OK or the first block error."""
        import numpy as np
        pres = np.ascontiguousarray(np.asarray(present, dtype=bool).astype(np.uint8).reshape(n_blocks, self.k + self.m))
        st = status if status is not None else np.zeros(n_blocks, np.int32)
        return int(self._L.zs3_verify_reconstruct_batch_masks(
            self._h, _ptr(shards, offset), block_stride, shard_len, n_blocks, pres.ctypes.data,
            1 if data_only else 0, _ptr(expect), _ptr(bad), _ptr(sums_out), st.ctypes.data, _stream(stream)))

    # ---- host-pointer calls ----
    def encode_data(self, buf, length: int, sums: bool = False):
        """EncodeData in place on a writable host buffer (numpy uint8 / bytearray)
        with capacity >= (k+m)*S.  Returns (S, sums_bytes_or_None)."""
        import numpy as np
        arr = _u8buf(buf)
        out = np.zeros((self.k + self.m) * 32, dtype=np.uint8) if sums else None
        S = self._L.zs3_encode_data(self._h, arr.ctypes.data, length, arr.nbytes,
                                  out.ctypes.data if sums else None)
        _check(S, "EncodeData")
        return S, (out.reshape(self.k + self.m, 32) if sums else None)

    def _stream_encode_args(self, name, src, total_len, parity, sums, batch_blocks):
        """Addresses of the encode stream's host buffers after checking their sizes: the
        library reads total_len bytes of src and writes nblocks*m*S parity bytes and
        nblocks*(k+m)*32 sum bytes through raw pointers (a short buffer would be overrun)."""
        import numpy as np

        if total_len < 0 or batch_blocks <= 0:
            raise ValueError(f"{name}: total_len >= 0 and batch_blocks > 0")
        B, k, m = self.block_size, self.k, self.m
        S = -(-B // k)
        nblocks = -(-total_len // B)
        out = []
        for x, what, need in ((src, "src", total_len), (parity, "parity", nblocks * m * S),
                              (sums, "sums", nblocks * (k + m) * 32)):
            if isinstance(x, HostBuffer):
                if not x.ptr or x.nbytes < need:
                    raise ValueError(f"{name}: {what} holds {x.nbytes} bytes, {nblocks} blocks need {need}")
                out.append(x.ptr)
            else:
                if not isinstance(x, np.ndarray) or not x.flags.c_contiguous or x.nbytes < need:
                    raise ValueError(f"{name}: {what} must be a C-contiguous numpy array of >= {need} bytes")
                out.append(x.ctypes.data)
        return out

    def stream_encode(self, src, total_len: int, parity, sums, batch_blocks: int = 256) -> int:
        """End-to-end host stream: returns the number of blocks (zs3_stream_encode).
        src/parity/sums are host buffers (numpy arrays or pinned HostBuffer)."""
        a, p, q = self._stream_encode_args("stream_encode", src, total_len, parity, sums, batch_blocks)
        n = self._L.zs3_stream_encode(self._h, a, total_len, p, q, batch_blocks)
        return _check(n, "stream_encode")

    def stream_encode_multi(self, devices, src, total_len: int, parity, sums, batch_blocks: int = 256) -> int:
        """zs3_stream_encode_multi: the stream split over `devices` (one host thread,
        stream set and pinned slots per device)."""
        a, p, q = self._stream_encode_args("stream_encode_multi", src, total_len, parity, sums, batch_blocks)
        devs = (C.c_int * len(devices))(*devices)
        n = self._L.zs3_stream_encode_multi(self._h, devs, len(devices), a, total_len, p, q, batch_blocks)
        return _check(n, "stream_encode_multi")

    def stream_decode(self, stripes, total_len: int, present, data_only: bool, expect=None, bad=None,
                      sums_out=None, status=None, batch_blocks: int = 128) -> int:
        """zs3_stream_decode: GET (data_only) / heal of a whole object's stripes in host
        memory (numpy uint8 or HostBuffer), pipelined through the device.  `present` is an
        (n_blocks, k+m) array; expect (n_blocks, k+m, 32) uint8, bad (n_blocks, k+m) int32,
        sums_out (n_blocks, k+m, 32) uint8 and status (n_blocks,) int32 are optional numpy
        arrays.  Returns the number of blocks or the first block's status (< 0)."""
        import numpy as np

        # the library reads and writes these buffers through raw pointers: check every size,
        # dtype and layout here (a short or strided array would be overrun in host memory)
        if total_len < 0 or batch_blocks <= 0:
            raise ValueError("stream_decode: total_len >= 0 and batch_blocks > 0")
        R = self.k + self.m
        B = self.block_size
        S = -(-B // self.k)
        nblocks = -(-total_len // B)
        need = nblocks * R * S

        def check(x, name, dtype, shape):
            if x is None:
                return None
            if not isinstance(x, np.ndarray) or x.dtype != np.dtype(dtype) or not x.flags.c_contiguous:
                raise ValueError(f"stream_decode: {name} must be a C-contiguous numpy {np.dtype(dtype)} array")
            if x.size != int(np.prod(shape)):
                raise ValueError(f"stream_decode: {name} has {x.size} elements, the object needs {shape}")
            return x.ctypes.data

        if isinstance(stripes, HostBuffer):
            if not stripes.ptr or stripes.nbytes < need:
                raise ValueError(f"stream_decode: stripes hold {stripes.nbytes} bytes, {nblocks} blocks need {need}")
            sp = stripes.ptr
        else:
            if (not isinstance(stripes, np.ndarray) or stripes.dtype != np.uint8 or not stripes.flags.c_contiguous
                    or stripes.nbytes < need):
                raise ValueError(f"stream_decode: stripes must be a C-contiguous uint8 array of >= {need} bytes")
            sp = stripes.ctypes.data
        pres = np.ascontiguousarray(np.asarray(present, dtype=bool).astype(np.uint8))
        if pres.size != nblocks * R:
            raise ValueError(f"stream_decode: present has {pres.size} entries, {nblocks} blocks of {R} shards need "
                             f"{nblocks * R}")
        e_p = check(expect, "expect", np.uint8, (nblocks, R, 32))
        b_p = check(bad, "bad", np.int32, (nblocks, R))
        o_p = check(sums_out, "sums_out", np.uint8, (nblocks, R, 32))
        s_p = check(status, "status", np.int32, (nblocks,))
        return int(self._L.zs3_stream_decode(self._h, sp, total_len, pres.ctypes.data, 1 if data_only else 0,
                                             e_p, b_p, o_p, s_p, batch_blocks))

    def decode_data_blocks(self, shards, present, data_only: bool) -> None:
        """Reconstruct in place on a (k+m, S) C-contiguous numpy uint8 array."""
        pres = (C.c_uint8 * (self.k + self.m))(*[1 if p else 0 for p in present])
        _check(self._L.zs3_decode_data_blocks(self._h, shards.ctypes.data, shards.shape[1], pres,
                                            1 if data_only else 0), "DecodeDataBlocks")


class Queue:
    """Cross-request batching queue (zs3_queue_*): concurrent callers' blocks are
    gathered into device batches.  Each call below blocks the calling thread only
    (ctypes releases the GIL), so N Python threads behave like N goroutines in cgo."""

    def __init__(self, codec: Codec, device: int = -1, max_batch: int = 0, max_wait_us: int = 0, slots: int = 0,
                 devices=None):
        self._L = codec._L
        self.codec = codec
        self.k, self.m = codec.k, codec.m
        devs = list(devices) if devices else []
        self._devs = (C.c_int * max(1, len(devs)))(*devs)
        opts = QueueOpts(device, max_batch, max_wait_us, slots, self._devs if devs else None, len(devs))
        h = C.c_void_p()
        _check(self._L.zs3_queue_new(codec._h, C.byref(opts), C.byref(h)), "queue_new")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.zs3_queue_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def encode_data(self, buf, length: int, sums: bool = True):
        """EncodeData in place on a host buffer through the queue; returns (S, sums)."""
        import numpy as np
        arr = _u8buf(buf)
        out = np.zeros((self.k + self.m) * 32, dtype=np.uint8) if sums else None
        S = self._L.zs3_queue_encode_data(self._h, arr.ctypes.data, length, arr.nbytes,
                                          out.ctypes.data if sums else None)
        _check(S, "queue EncodeData")
        return S, (out.reshape(self.k + self.m, 32) if sums else None)

    def submit_encode(self, buf, length: int, sums=None):
        """Asynchronous form: returns a request handle for wait()."""
        arr = _u8buf(buf)
        r = C.c_void_p()
        _check(self._L.zs3_queue_submit_encode(self._h, arr.ctypes.data, length, arr.nbytes,
                                               sums.ctypes.data if sums is not None else None, C.byref(r)),
               "queue submit")
        return r

    def wait(self, req) -> int:
        return int(self._L.zs3_req_wait(req))

    def decode(self, shards, present, data_only: bool, expect=None, bad=None, sums_out=None) -> int:
        """DecodeDataBlocks (data_only) / heal Reconstruct on one (k+m, S) host stripe
        (numpy uint8, C-contiguous), survivors verified against `expect` ((k+m, 32))
        when given.  Returns the status: 0, errFileCorrupt (-7, see `bad`), or the
        reedsolomon error of the pattern."""
        import numpy as np
        pres = np.asarray([1 if p else 0 for p in present], dtype=np.uint8)
        r = C.c_void_p()
        rc = self._L.zs3_queue_submit_decode(self._h, shards.ctypes.data, shards.shape[1], pres.ctypes.data,
                                             1 if data_only else 0,
                                             expect.ctypes.data if expect is not None else None,
                                             bad.ctypes.data if bad is not None else None,
                                             sums_out.ctypes.data if sums_out is not None else None, C.byref(r))
        if rc:
            return int(rc)
        return int(self._L.zs3_req_wait(r))

    def flush(self) -> None:
        _check(self._L.zs3_queue_flush(self._h))

    def stats(self) -> tuple[int, int]:
        b, n = C.c_int64(0), C.c_int64(0)
        _check(self._L.zs3_queue_stats(self._h, C.byref(b), C.byref(n)))
        return b.value, n.value

    def device_stats(self, index: int) -> tuple[int, int, int]:
        """(device, batches, blocks) of the index-th listed device."""
        d, b, n = C.c_int(0), C.c_int64(0), C.c_int64(0)
        _check(self._L.zs3_queue_device_stats(self._h, index, C.byref(d), C.byref(b), C.byref(n)))
        return d.value, b.value, n.value

    def zero_copy_blocks(self) -> int:
        """Blocks whose bytes were DMA'd straight from / to a pinned caller buffer."""
        return int(self._L.zs3_queue_zero_copy_blocks(self._h))


class HostBuffer:
    """Pinned host memory from zs3_host_alloc (the pinned-bpool backing, §8f.2)."""

    def __init__(self, nbytes: int):
        import numpy as np
        p = C.c_void_p()
        self._L = lib()  # the library whose queues see this buffer as pinned
        _check(self._L.zs3_host_alloc(C.byref(p), nbytes), "host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self._L.zs3_host_free(self.ptr)
            self.ptr = None


def split_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """zs3_split_range: the library's own multi-GPU split (pure host arithmetic)."""
    lo, hi = C.c_int64(0), C.c_int64(0)
    lib().zs3_split_range(total, world, rank, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


def bitrot_shard_file_size(size: int, shard_size: int) -> int:
    return lib().zs3_bitrot_shard_file_size(size, shard_size)


def hh256_batch(msgs, msg_stride: int, msg_len: int, n_msgs: int, sums, key: bytes | None = None,
                stream=None, offset: int = 0) -> None:
    kb = C.create_string_buffer(key, 32) if key else None
    _check(lib().zs3_hh256_batch(kb, _ptr(msgs, offset), msg_stride, msg_len, n_msgs, _ptr(sums),
                                 _stream(stream)), "hh256_batch")


def hh256_verify_batch(msgs, msg_stride: int, msg_len: int, n_msgs: int, want, bad,
                       key: bytes | None = None, stream=None, offset: int = 0) -> None:
    kb = C.create_string_buffer(key, 32) if key else None
    _check(lib().zs3_hh256_verify_batch(kb, _ptr(msgs, offset), msg_stride, msg_len, n_msgs, _ptr(want),
                                        _ptr(bad), _stream(stream)), "hh256_verify_batch")


def md5_batch(msgs, msg_stride: int, msg_len: int, n_msgs: int, out, lens=None, offset: int = 0,
              stream=None) -> None:
    """S3 ETag (MD5) of n device messages (zs3_md5_batch); `lens` = optional device int64
    per-message lengths; digest i at out[16*i : 16*i+16]."""
    _check(lib().zs3_md5_batch(_ptr(msgs, offset), msg_stride, msg_len, _ptr(lens), n_msgs, _ptr(out),
                               _stream(stream)), "md5_batch")


def sha256_batch(msgs, msg_stride: int, msg_len: int, n_msgs: int, out, lens=None, offset: int = 0,
                 stream=None) -> None:
    """Content SHA-256 of n device messages (zs3_sha256_batch); digest i at out[32*i:]."""
    _check(lib().zs3_sha256_batch(_ptr(msgs, offset), msg_stride, msg_len, _ptr(lens), n_msgs, _ptr(out),
                                  _stream(stream)), "sha256_batch")


def md5_parts(base, offsets, lens, n_msgs: int, out, stream=None) -> None:
    """MD5 of n independent device messages (multipart parts) in one launch
    (zs3_md5_parts): message i at base + offsets[i] (device int64), length lens[i]."""
    _check(lib().zs3_md5_parts(_ptr(base), _ptr(offsets), _ptr(lens), n_msgs, _ptr(out), _stream(stream)),
           "md5_parts")


def sha256_parts(base, offsets, lens, n_msgs: int, out, stream=None) -> None:
    """SHA-256 of n independent device messages in one launch (zs3_sha256_parts)."""
    _check(lib().zs3_sha256_parts(_ptr(base), _ptr(offsets), _ptr(lens), n_msgs, _ptr(out), _stream(stream)),
           "sha256_parts")


def etag_multipart(etags) -> bytes:
    """etag.Multipart (internal/etag/etag.go:211-226) over a list of raw ETag byte
    strings; returns b"" (the nil ETag) for an empty list."""
    import numpy as np
    n = len(etags)
    if n == 0:
        return b""
    cat = np.frombuffer(b"".join(etags) or b"\0", dtype=np.uint8).copy()
    lens = np.array([len(e) for e in etags], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    out = np.zeros(48, dtype=np.uint8)
    r = _check(lib().zs3_etag_multipart(cat.ctypes.data, offs.ctypes.data, lens.ctypes.data, n, out.ctypes.data),
               "etag_multipart")
    return out[:r].tobytes()


def hh256_batch_ragged(ptrs, lens, n_msgs: int, sums, key: bytes | None = None, stream=None) -> None:
    """HighwayHash-256 of messages of different lengths (zs3_hh256_batch_ragged):
    `ptrs` / `lens` are device int64 tensors of message addresses / lengths."""
    kb = C.create_string_buffer(key, 32) if key else None
    _check(lib().zs3_hh256_batch_ragged(kb, _ptr(ptrs), _ptr(lens), n_msgs, _ptr(sums), _stream(stream)),
           "hh256_batch_ragged")


def bitrot_verify_file_batch(files, file_stride: int, n_files: int, want_size: int, part_size: int,
                             shard_size: int, bad, file_bad=None, key: bytes | None = None, stream=None) -> int:
    """Deep-scan bitrotVerify of n device-resident shard files in the on-disk
    [sum][chunk]* layout (zs3_bitrot_verify_file_batch).  Raises errFileCorrupt when
    want_size is not bitrotShardFileSize(part_size, shard_size); returns chunks per
    file.  `bad` (device int32, n_files*chunks) flags corrupt chunks, `file_bad`
    (optional, n_files) corrupt files."""
    kb = C.create_string_buffer(key, 32) if key else None
    chunks = C.c_int64(0)
    _check(lib().zs3_bitrot_verify_file_batch(kb, _ptr(files), file_stride, n_files, want_size, part_size,
                                               shard_size, _ptr(bad), _ptr(file_bad), C.byref(chunks),
                                               _stream(stream)), "bitrotVerify")
    return chunks.value


def fill_batch(out, stride: int, length: int, n_blocks: int, seed: int = 0, obj0: int = 0,
               stream=None, offset: int = 0) -> None:
    _check(lib().zs3_fill_batch(_ptr(out, offset), stride, length, n_blocks, seed, obj0, _stream(stream)),
           "fill_batch")


def hh256(msg: bytes, key: bytes | None = None) -> bytes:
    """HighwayHash-256 of one host message through the device path."""
    import numpy as np
    m = np.frombuffer(bytes(msg), dtype=np.uint8) if len(msg) else np.zeros(1, np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    kb = C.create_string_buffer(key, 32) if key else None
    _check(lib().zs3_hh256(kb, m.ctypes.data, len(msg), out.ctypes.data), "hh256")
    return out.tobytes()


def selftest() -> None:
    """erasureSelfTest + bitrotSelfTest (server-main.go:437-438) on the device."""
    _check(lib().zs3_selftest(), "selftest")


def last_path() -> int:
    return lib().zs3_last_path()


KERNEL_VR_QUAD = 1 << 16  # include/zs3gpu.h ZS3_KERNEL_VR_QUAD


def path_mask(reset: bool = False) -> int:
    """Every kernel family this thread's launches used since the last reset (zs3_path_mask):
    bit 1 << ZS3_PATH_* per family, plus KERNEL_VR_QUAD for the survivor-quad GET / heal
    kernel."""
    return int(lib().zs3_path_mask(1 if reset else 0))


def pool_limit(max_idle_bytes: int) -> int:
    """zs3_pool_limit: cap (and trim to) the stream drivers' idle staging; bytes freed."""
    return int(lib().zs3_pool_limit(max_idle_bytes))


def set_debug_buffer(t) -> None:
    """Diagnostics build only: per-wave stamp buffer for this thread (None = off)."""
    diag_lib().zs3_debug_set_buffer(_ptr(t))


def device_count() -> int:
    n = C.c_int(0)
    _check(lib().zs3_device_count(C.byref(n)))
    return n.value
