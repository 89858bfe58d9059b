"""zs3server_amd — MI355X-native erasure-shard + bitrot-hash data path.

Python binding of the C ABI in include/zs3gpu.h (libzs3gpu.so, built for gfx950).
The Go server binds the same ABI through cgo; this module is the
test/bench host and mirrors the reference's Erasure API in `erasure.py` and the
streaming bitrot format in `bitrot.py`.

There is no CPU fallback: if libzs3gpu.so is missing or fails to load, import of
`lib()` raises.  Device buffers are torch tensors on a ROCm device (or raw
device pointers as ints).
"""
from __future__ import annotations

import ctypes as C
import os

try:  # load torch's HIP runtime first so the library binds to the same one
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libzs3gpu.so")

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
    "zs3_last_path", "zs3_debug_set_variant", "zs3_debug_set_buffer",
]


class ZS3Error(Exception):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        self.name = ERRORS.get(code, f"error {code}")
        super().__init__(f"{what}: {self.name} ({code})" if what else f"{self.name} ({code})")


_L = None


def lib():
    """Load libzs3gpu.so (raises if absent: the product path has no fallback)."""
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built — run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
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
    L.zs3_etag_multipart.argtypes = [vp, vp, vp, i64, vp]
    L.zs3_host_alloc.argtypes = [C.POINTER(vp), C.c_size_t]
    L.zs3_host_free.argtypes = [vp]
    _L = L
    return L


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
        self._h = h
        self.k, self.m, self.block_size = k, m, block_size

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _L is not None:
            _L.zs3_codec_free(h)
            self._h = None

    # ---- size arithmetic (erasure-coding.go:122-150) ----
    def shard_size(self) -> int:
        return lib().zs3_shard_size(self._h)

    def shard_file_size(self, total: int) -> int:
        return lib().zs3_shard_file_size(self._h, total)

    def shard_file_offset(self, start: int, length: int, total: int) -> int:
        return lib().zs3_shard_file_offset(self._h, start, length, total)

    def matrix(self):
        import numpy as np
        out = np.zeros((self.k + self.m) * self.k, dtype=np.uint8)
        _check(lib().zs3_codec_matrix(self._h, out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out.reshape(self.k + self.m, self.k)

    # ---- device-resident batches ----
    def encode_batch(self, data, data_stride: int, block_len: int, n_blocks: int, parity,
                     parity_stride: int, sums=None, parity_offset: int = 0, data_offset: int = 0,
                     stream=None) -> None:
        _check(lib().zs3_encode_batch(self._h, _ptr(data, data_offset), data_stride, block_len, n_blocks,
                                      _ptr(parity, parity_offset), parity_stride, _ptr(sums),
                                      _stream(stream)), "encode_batch")

    def reconstruct_batch(self, shards, block_stride: int, shard_len: int, n_blocks: int, present,
                          data_only: bool, stream=None, offset: int = 0) -> None:
        pres = (C.c_uint8 * (self.k + self.m))(*[1 if p else 0 for p in present])
        _check(lib().zs3_reconstruct_batch(self._h, _ptr(shards, offset), block_stride, shard_len, n_blocks,
                                           pres, 1 if data_only else 0, _stream(stream)), "reconstruct_batch")

    def verify_reconstruct_batch(self, shards, block_stride: int, shard_len: int, n_blocks: int, present,
                                 data_only: bool, expect, bad, sums_out=None, stream=None,
                                 offset: int = 0) -> None:
        """GET / heal pass (zs3_verify_reconstruct_batch): verify the k survivors
        against `expect` ([n][k+m][32] device), flag failures in `bad` ([n][k+m]
        int32 device), rebuild the missing shards in place, optionally hash them
        into `sums_out`."""
        pres = (C.c_uint8 * (self.k + self.m))(*[1 if p else 0 for p in present])
        _check(lib().zs3_verify_reconstruct_batch(self._h, _ptr(shards, offset), block_stride, shard_len,
                                                  n_blocks, pres, 1 if data_only else 0, _ptr(expect), _ptr(bad),
                                                  _ptr(sums_out), _stream(stream)), "verify_reconstruct_batch")

    # ---- host-pointer calls ----
    def encode_data(self, buf, length: int, sums: bool = False):
        """EncodeData in place on a writable host buffer (numpy uint8 / bytearray)
        with capacity >= (k+m)*S.  Returns (S, sums_bytes_or_None)."""
        import numpy as np
        arr = _u8buf(buf)
        out = np.zeros((self.k + self.m) * 32, dtype=np.uint8) if sums else None
        S = lib().zs3_encode_data(self._h, arr.ctypes.data, length, arr.nbytes,
                                  out.ctypes.data if sums else None)
        _check(S, "EncodeData")
        return S, (out.reshape(self.k + self.m, 32) if sums else None)

    def stream_encode(self, src, total_len: int, parity, sums, batch_blocks: int = 256) -> int:
        """End-to-end host stream: returns the number of blocks (zs3_stream_encode).
        src/parity/sums are host buffers (numpy arrays or pinned HostBuffer)."""
        def addr(x):
            return x.ptr if isinstance(x, HostBuffer) else x.ctypes.data
        n = lib().zs3_stream_encode(self._h, addr(src), total_len, addr(parity), addr(sums), batch_blocks)
        return _check(n, "stream_encode")

    def decode_data_blocks(self, shards, present, data_only: bool) -> None:
        """Reconstruct in place on a (k+m, S) C-contiguous numpy uint8 array."""
        pres = (C.c_uint8 * (self.k + self.m))(*[1 if p else 0 for p in present])
        _check(lib().zs3_decode_data_blocks(self._h, shards.ctypes.data, shards.shape[1], pres,
                                            1 if data_only else 0), "DecodeDataBlocks")


class HostBuffer:
    """Pinned host memory from zs3_host_alloc (the pinned-bpool backing, §8f.2)."""

    def __init__(self, nbytes: int):
        import numpy as np
        p = C.c_void_p()
        _check(lib().zs3_host_alloc(C.byref(p), nbytes), "host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            lib().zs3_host_free(self.ptr)
            self.ptr = None


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


def set_variant(v: int) -> None:
    """Diagnostics: experimental fused-kernel variant (0 = tuned default)."""
    lib().zs3_debug_set_variant(v)


def set_debug_buffer(t) -> None:
    L = lib()
    L.zs3_debug_set_buffer.argtypes = [C.c_void_p]
    L.zs3_debug_set_buffer(_ptr(t))


def device_count() -> int:
    n = C.c_int(0)
    _check(lib().zs3_device_count(C.byref(n)))
    return n.value
