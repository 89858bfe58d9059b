"""Mirror of the streaming bitrot format (HighwayHash256S) over the zs3gpu C ABI.

cmd/bitrot-streaming.go: every Write(p) of one shard chunk emits
[32-byte HH256(p)][p]; ReadAt re-hashes each chunk and returns errFileCorrupt on
mismatch.  cmd/bitrot.go:150-210: bitrotShardFileSize and bitrotVerify.
Hashes are computed by the device kernel (zs3_hh256 / zs3_hh256_batch).
"""
from __future__ import annotations

import io

from . import MAGIC_HH256_KEY, ZS3Error, bitrot_shard_file_size, hh256

HASH_SIZE = 32
ERR_FILE_CORRUPT = -7
ERR_UNEXPECTED = -8


class DiskError(Exception):
    """A StorageAPI error value (cmd/storage-errors.go): errFaultyDisk, errDiskNotFound,
    errFileNotFound, ...; `name` carries the Go identifier."""

    def __init__(self, name: str):
        self.name = name
        super().__init__(name)


class StreamingBitrotWriter:
    """newStreamingBitrotWriterBuffer (bitrot-streaming.go:84) — in-memory sink.
    close_with_err() mirrors streamingBitrotWriter.closeWithErr (the CreateFile pipe
    closed with an error: every later Write fails with it)."""

    def __init__(self, shard_size: int, sink=None):
        self.shard_size = shard_size
        self.iow = sink if sink is not None else io.BytesIO()
        self.err = None

    def Write(self, p: bytes) -> int:
        # bitrot-streaming.go:43-65
        if len(p) == 0:
            return 0
        return self.WriteWithSum(p, hh256(bytes(p), MAGIC_HH256_KEY))

    def WriteWithSum(self, p, sum32: bytes) -> int:
        """Write with the sum the fused device encode already computed (the cgo shim's
        precomputed-sum path): same [sum][chunk] bytes as Write."""
        if len(p) == 0:
            return 0
        if self.err is not None:
            raise DiskError(self.err)
        self.iow.write(bytes(sum32))
        self.iow.write(bytes(p))
        return len(p)

    def close_with_err(self, err: str) -> None:
        self.err = err

    def Close(self) -> None:
        pass

    def getvalue(self) -> bytes:
        return self.iow.getvalue()


class StreamingBitrotReader:
    """newStreamingBitrotReader over an in-memory shard file (bitrot-streaming.go:192)."""

    def __init__(self, data: bytes, till_offset: int, shard_size: int):
        self.data = data
        self.shard_size = shard_size
        self.till_offset = -(-till_offset // shard_size) * HASH_SIZE + till_offset
        self.rc = None
        self.curr_offset = 0

    def ReadAt(self, n: int, offset: int) -> bytes:
        # bitrot-streaming.go:142-189
        want, buf = self.read_raw(n, offset)
        if hh256(buf, MAGIC_HH256_KEY) != want:
            raise ZS3Error(ERR_FILE_CORRUPT, "ReadAt: content hash does not match")
        return buf

    def read_raw(self, n: int, offset: int):
        """ReadAt's stream handling (offset checks, [sum][chunk] framing, short reads)
        without the hash: returns (stored sum, chunk) so a caller can verify many
        chunks in one device launch (ParallelReader)."""
        if offset % self.shard_size != 0:
            raise ZS3Error(ERR_UNEXPECTED, "ReadAt: unaligned offset")
        if self.rc is None:
            self.curr_offset = offset
            stream_offset = (offset // self.shard_size) * HASH_SIZE + offset
            self.rc = io.BytesIO(self.data[stream_offset:self.till_offset])
        if offset != self.curr_offset:
            raise ZS3Error(ERR_UNEXPECTED, "ReadAt: non-sequential offset")
        want = self.rc.read(HASH_SIZE)
        buf = self.rc.read(n)
        if len(want) != HASH_SIZE or len(buf) != n:
            raise ZS3Error(ERR_UNEXPECTED, "ReadAt: short read (io.ErrUnexpectedEOF)")
        self.curr_offset += n
        return want, buf


class BadDiskReader:
    """A bitrot reader over badDisk (erasure-decode_test.go:31, erasure-encode_test.go:30):
    ReadFileStream fails with errFaultyDisk."""

    def ReadAt(self, n: int, offset: int) -> bytes:
        raise DiskError("errFaultyDisk")

    def read_raw(self, n: int, offset: int):
        raise DiskError("errFaultyDisk")


def bitrot_verify(stream: bytes, want_size: int, part_size: int, shard_size: int) -> None:
    """bitrotVerify for HighwayHash256S (cmd/bitrot.go:158-210): raises errFileCorrupt.

    The whole shard file goes to the device once and every chunk is verified in one
    launch against the sum stored in front of it (zs3_bitrot_verify_file_batch)."""
    bitrot_verify_files([stream], want_size, part_size, shard_size, raise_first=True)


def bitrot_verify_files(files, want_size: int, part_size: int, shard_size: int, raise_first: bool = False):
    """Deep scan of several shard files of one part (xlStorage.VerifyFile,
    cmd/xl-storage.go:2386-2404) in one device launch.  Returns the list of file
    indices that fail (errFileCorrupt); with raise_first, raises for the first one.
    A file shorter than want_size fails like the reference's short read."""
    import numpy as np
    import torch

    from . import bitrot_verify_file_batch

    if want_size != bitrot_shard_file_size(part_size, shard_size):
        raise ZS3Error(ERR_FILE_CORRUPT, "bitrotVerify: size")
    short = [i for i, f in enumerate(files) if len(f) < want_size]
    n = len(files)
    stride = max(16, (want_size + 15) // 16 * 16)
    host = np.zeros(n * stride, dtype=np.uint8)
    for i, f in enumerate(files):
        b = np.frombuffer(bytes(f[:want_size]), dtype=np.uint8)
        host[i * stride: i * stride + len(b)] = b
    dev = torch.from_numpy(host).to("cuda")
    chunks = -(-part_size // shard_size) if part_size else 0
    bad = torch.zeros(max(1, n * chunks), dtype=torch.int32, device="cuda")
    file_bad = torch.zeros(max(1, n), dtype=torch.int32, device="cuda")
    bitrot_verify_file_batch(dev, stride, n, want_size, part_size, shard_size, bad, file_bad, key=MAGIC_HH256_KEY)
    torch.cuda.synchronize()
    failed = sorted(set(short) | {int(i) for i in np.nonzero(file_bad.cpu().numpy()[:n])[0]})
    if raise_first and failed:
        raise ZS3Error(ERR_FILE_CORRUPT, f"bitrotVerify: file {failed[0]} hash mismatch")
    return failed
