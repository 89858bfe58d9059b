"""Mirror of the reference's Erasure API over the zs3gpu C ABI.

Same names, argument meaning and error behaviour as cmd/erasure-coding.go and
cmd/erasure-utils.go, so tests read like the reference's own (erasure_test.go).
Shards are Python lists of numpy uint8 views (None = missing, the Go nil/len 0).
All arithmetic runs in the HIP kernels (host-staged through pinned memory).
"""
from __future__ import annotations

import io
import os
import threading

import numpy as np

from . import Codec, ZS3Error

BLOCK_SIZE_V1 = 10 << 20  # cmd/object-api-common.go:37
BLOCK_SIZE_V2 = 1 << 20   # cmd/object-api-common.go:40

ERR_INV_SHARD_NUM, ERR_MAX_SHARD_NUM, ERR_TOO_FEW_SHARDS = -1, -2, -3
ERR_SHARD_NO_DATA, ERR_SHARD_SIZE, ERR_SHORT_DATA = -4, -5, -6
ERR_FILE_CORRUPT, ERR_INVALID_ARGUMENT = -7, -8


class ErasureReadQuorum(Exception):
    """errErasureReadQuorum (cmd/erasure-errors.go): fewer than k readable shards."""


class ErasureWriteQuorum(Exception):
    """errErasureWriteQuorum (cmd/erasure-errors.go): fewer than writeQuorum writers ok."""


# erasure-decode.go: the two read errors Decode / Heal pass upstream (heal triggers)
ERR_FILE_NOT_FOUND = "errFileNotFound"
ERR_FILE_CORRUPT_NAME = "errFileCorrupt"


# objectOpIgnoredErrs (cmd/erasure-object.go:48 = baseIgnoredErrs, storage-errors.go:127-133,
# + errDiskAccessDenied, errUnformattedDisk): not counted by reduceWriteQuorumErrs
OBJECT_OP_IGNORED_ERRS = frozenset({"errDiskNotFound", "errFaultyDisk", "errFaultyRemoteDisk",
                                    "errDiskAccessDenied", "errUnformattedDisk"})


def _err_name(e: BaseException) -> str:
    """The Go identifier of a writer / reader error (DiskError.name, a ZS3Error's
    reedsolomon sentinel), else the exception's own text."""
    name = getattr(e, "name", None)
    if name:
        return name
    if isinstance(e, ZS3Error) and e.code == ERR_FILE_CORRUPT:
        return "errFileCorrupt"
    return str(e) or type(e).__name__


def reduce_write_quorum_errs(errs: list, write_quorum: int):
    """reduceWriteQuorumErrs (cmd/erasure-metadata-utils.go:36-87): the most frequent
    non-ignored error value (None counts as a value, and wins ties) if it occurs at
    least write_quorum times, else errErasureWriteQuorum.  Returns None or raises."""
    counts: dict = {}
    for e in errs:
        if e in OBJECT_OP_IGNORED_ERRS:
            continue
        counts[e] = counts.get(e, 0) + 1
    max_count, max_err = 0, None
    for e, c in counts.items():
        if c > max_count:
            max_count, max_err = c, e
        elif c == max_count and e is None:
            max_err = None
    if max_count >= write_quorum:
        if max_err is None:
            return None
        from .bitrot import DiskError
        raise DiskError(max_err)
    raise ErasureWriteQuorum(f"{sum(e is None for e in errs)} writers ok < quorum {write_quorum}")


class ParallelWriter:
    """parallelWriter (cmd/erasure-encode.go:29-73): one Write per shard writer; a writer
    that fails in any way is dropped (its slot in the caller's list set to None, as the
    Go slice is shared) with its error recorded; below write quorum the per-writer errors
    are reduced as reduceWriteQuorumErrs does.  The fused device encode hands each writer
    its precomputed HighwayHash sum (WriteWithSum)."""

    def __init__(self, writers: list, write_quorum: int):
        self.writers = writers  # shared with the caller, like the Go slice
        self.write_quorum = write_quorum
        self.errs = [None] * len(writers)

    def Write(self, blocks: list, sums=None) -> None:
        for i, w in enumerate(self.writers):
            if w is None:
                self.errs[i] = "errDiskNotFound"
                continue
            if self.errs[i] is not None:
                continue
            try:
                if sums is not None and hasattr(w, "WriteWithSum"):
                    n = w.WriteWithSum(blocks[i], sums[i])
                else:
                    n = w.Write(blocks[i])
                if n != len(blocks[i]):
                    self.errs[i] = "io.ErrShortWrite"
                    self.writers[i] = None
            except Exception as e:  # noqa: BLE001 - every write error drops that writer (:51-58)
                self.errs[i] = _err_name(e)
                self.writers[i] = None
        # HealFile uses writeQuorum 1 (erasure-encode.go:63-69)
        if sum(e is None for e in self.errs) >= self.write_quorum:
            return
        reduce_write_quorum_errs(self.errs, self.write_quorum)


class ParallelReader:
    """parallelReader (cmd/erasure-decode.go:31-203).  Reads shard chunks reader by
    reader until k chunks verified: each round reads the next candidates' [sum][chunk]
    without hashing, then verifies all of them in ONE device launch
    (zs3_hh256_verify_batch, per-chunk errFileCorrupt flags); a failed or corrupt reader
    is dropped from both reader lists (shared with the caller, as in Go) and the next
    one is tried.  Same shards decode as the goroutine version: the data are unique."""

    def __init__(self, readers: list, e: "Erasure", offset: int, total_length: int):
        self.readers = readers
        self.org_readers = readers
        self.data_blocks = e.dataBlocks
        self.offset = (offset // e.blockSize) * e.ShardSize()
        self.shard_size = e.ShardSize()
        self.shard_file_size = e.ShardFileSize(total_length)
        self.reader_to_buf = list(range(len(readers)))

    def prefer_readers(self, prefer: list) -> None:
        # erasure-decode.go:65-90
        if len(prefer) != len(self.org_readers):
            return
        self.readers = list(self.org_readers)
        nxt = 0
        for i, ok in enumerate(prefer):
            if not ok or self.readers[i] is None:
                continue
            if i == nxt:
                nxt += 1
                continue
            self.readers[nxt], self.readers[i] = self.readers[i], self.readers[nxt]
            self.reader_to_buf[nxt] = i
            self.reader_to_buf[i] = nxt
            nxt += 1

    def Read(self):
        """Returns (bufs, err): bufs = k+m chunks (None = not read), err =
        errFileNotFound / errFileCorrupt when a reader failed that way but k chunks were
        still read; raises ErasureReadQuorum when fewer than k chunks could be read."""
        from .bitrot import DiskError
        n = len(self.readers)
        new_buf = [None] * n
        if self.offset + self.shard_size > self.shard_file_size:
            self.shard_size = self.shard_file_size - self.offset
        if self.shard_size == 0:
            return [np.zeros(0, np.uint8)] * n, None
        bitrot_heal = missing_heal = False
        ri = 0
        while sum(b is not None for b in new_buf) < self.data_blocks and ri < n:
            need = self.data_blocks - sum(b is not None for b in new_buf)
            cand = []  # (reader index, buf index, sum, chunk)
            while len(cand) < need and ri < n:
                i = ri
                ri += 1
                rr = self.readers[i]
                if rr is None:
                    continue
                bi = self.reader_to_buf[i]
                try:
                    want, chunk = rr.read_raw(self.shard_size, self.offset)
                    cand.append((i, bi, want, chunk))
                except (DiskError, ZS3Error) as err:
                    # erasure-decode.go:165-171: errFileNotFound -> missingPartsHeal,
                    # errFileCorrupt (a reader that detected the rot itself) -> bitrotHeal
                    name = _err_name(err)
                    if name == ERR_FILE_NOT_FOUND:
                        missing_heal = True
                    elif name == ERR_FILE_CORRUPT_NAME:
                        bitrot_heal = True
                    self.org_readers[bi] = None
                    self.readers[i] = None
            if not cand:
                continue
            bad = _verify_chunks([c[3] for c in cand], [c[2] for c in cand])
            for (i, bi, _, chunk), b in zip(cand, bad):
                if b:
                    bitrot_heal = True
                    self.org_readers[bi] = None
                    self.readers[i] = None
                else:
                    new_buf[bi] = np.frombuffer(bytes(chunk), dtype=np.uint8)
        if sum(b is not None for b in new_buf) >= self.data_blocks:
            self.offset += self.shard_size
            if missing_heal:
                return new_buf, ERR_FILE_NOT_FOUND
            if bitrot_heal:
                return new_buf, ERR_FILE_CORRUPT_NAME
            return new_buf, None
        raise ErasureReadQuorum(f"{sum(b is not None for b in new_buf)} shards read < {self.data_blocks}")


def _verify_chunks(chunks: list, wants: list) -> list:
    """HighwayHash-256 verify of equal-length chunks in one device launch: per-chunk
    errFileCorrupt flags (bitrot-streaming.go:182-185)."""
    import torch

    from . import MAGIC_HH256_KEY, hh256_verify_batch
    L = len(chunks[0])
    n = len(chunks)
    stride = max(16, -(-L // 16) * 16)
    host = np.zeros(n * stride, np.uint8)
    for i, c in enumerate(chunks):
        host[i * stride: i * stride + L] = np.frombuffer(bytes(c), np.uint8)
    want = np.frombuffer(b"".join(bytes(w) for w in wants), np.uint8).copy()
    d = torch.from_numpy(host).to("cuda")
    w = torch.from_numpy(want).to("cuda")
    bad = torch.zeros(n, dtype=torch.int32, device="cuda")
    hh256_verify_batch(d, stride, L, n, w, bad, key=MAGIC_HH256_KEY)
    return [bool(x) for x in bad.cpu().numpy()]


class Erasure:
    """cmd/erasure-coding.go:35-39."""

    def __init__(self, data_blocks: int, parity_blocks: int, block_size: int):
        self._codec = Codec(data_blocks, parity_blocks, block_size)  # raises ErrInvShardNum/ErrMaxShardNum
        self.dataBlocks = data_blocks
        self.parityBlocks = parity_blocks
        self.blockSize = block_size

    # erasure-coding.go:77-91
    def EncodeData(self, buf, length: int | None = None) -> list:
        """EncodeData(ctx, data): `buf` is a writable buffer whose first `length`
        bytes are the data and whose capacity holds (k+m)*S (the bpool buffer,
        cap 2*blockSize).  Returns k+m shard views into `buf` (parity in place)."""
        k, m = self.dataBlocks, self.parityBlocks
        arr = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
        n = len(arr) if length is None else length
        if n == 0:
            return [np.zeros(0, dtype=np.uint8) for _ in range(k + m)]
        S = -(-n // k)
        if len(arr) < (k + m) * S:
            # reedsolomon.Split allocates the padding shards when cap(data) is short;
            # the shard values are identical, only their backing differs.
            big = np.zeros((k + m) * S, dtype=np.uint8)
            big[:n] = arr[:n]
            arr = big
        S, _ = self._codec.encode_data(arr, n)
        return [arr[i * S:(i + 1) * S] for i in range(k + m)]

    def EncodeDataWithSums(self, buf, length: int):
        """EncodeData fused with the k+m streaming-bitrot HH256 sums
        (bitrot-streaming.go:47-49) — the GPU codec's fused entry point."""
        k, m = self.dataBlocks, self.parityBlocks
        arr = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
        if length == 0:
            return [np.zeros(0, dtype=np.uint8) for _ in range(k + m)], None
        S = -(-length // k)
        if len(arr) < (k + m) * S:  # reedsolomon.Split allocates the padding shards
            big = np.zeros((k + m) * S, dtype=np.uint8)
            big[:length] = arr[:length]
            arr = big
        S, sums = self._codec.encode_data(arr, length, sums=True)
        return [arr[i * S:(i + 1) * S] for i in range(k + m)], sums

    def _reconstruct(self, data: list, data_only: bool) -> None:
        k, m = self.dataBlocks, self.parityBlocks
        if len(data) != k + m:
            raise ZS3Error(ERR_TOO_FEW_SHARDS, "reconstruct")
        sizes = [len(s) for s in data if s is not None and len(s)]
        if not sizes:
            raise ZS3Error(ERR_SHARD_NO_DATA, "reconstruct")
        S = sizes[0]
        if any(sz != S for sz in sizes):
            raise ZS3Error(ERR_SHARD_SIZE, "reconstruct")
        present = [s is not None and len(s) > 0 for s in data]
        stripe = np.zeros((k + m, S), dtype=np.uint8)
        for i, s in enumerate(data):
            if present[i]:
                stripe[i] = np.asarray(s, dtype=np.uint8)
        self._codec.decode_data_blocks(stripe, present, data_only)
        for i in range(k + m):
            if not present[i] and (i < k or not data_only):
                data[i] = stripe[i].copy()

    # erasure-coding.go:96-109
    def DecodeDataBlocks(self, data: list) -> None:
        is_zero = 0
        for b in data:
            if b is None or len(b) == 0:
                is_zero += 1
                break
        if is_zero == 0 or is_zero == len(data):
            return
        self._reconstruct(data, True)

    # erasure-coding.go:113-119
    def DecodeDataAndParityBlocks(self, data: list) -> None:
        self._reconstruct(data, False)

    # erasure-coding.go:122-150
    def decode_verified(self, shards, S: int, n_blocks: int, present, expect, data_only: bool = True,
                        sums_out=None, stream=None) -> set:
        """GET path over a device batch [n][k+m][S] (torch uint8 on the GPU): verify
        the survivors' bitrot sums and rebuild missing shards in one fused pass
        (zs3_verify_reconstruct_batch).  A block whose survivor fails verification is
        re-decoded without that shard, as parallelReader does (erasure-decode.go:165-179:
        the corrupt reader is dropped and the next shard read); fewer than k good
        shards -> ErasureReadQuorum (errErasureReadQuorum, :201).  Returns the set of
        (block, shard) found corrupt (the bitrotHeal signal)."""
        import torch

        k, m = self.dataBlocks, self.parityBlocks
        R = k + m
        bad = torch.zeros((n_blocks, R), dtype=torch.int32, device=shards.device)
        self._codec.verify_reconstruct_batch(shards, R * S, S, n_blocks, present, data_only, expect, bad,
                                             sums_out=sums_out, stream=stream)
        flags = bad.cpu().numpy()
        corrupt = set()
        base = [bool(p) for p in present]
        for b in map(int, np.nonzero(flags.any(axis=1))[0]):
            pres = list(base)
            row = flags[b]
            while row.any():
                for i in map(int, np.nonzero(row)[0]):
                    corrupt.add((b, i))
                    pres[i] = False
                if sum(pres) < k:
                    raise ErasureReadQuorum(f"block {b}: {sum(pres)} verified shards < {k}")
                one = torch.zeros(R, dtype=torch.int32, device=shards.device)
                so = None if sums_out is None else sums_out.view(-1)[b * R * 32:]
                self._codec.verify_reconstruct_batch(shards.view(-1)[b * R * S:], R * S, S, 1, pres, data_only,
                                                     expect.view(-1)[b * R * 32:], one, sums_out=so,
                                                     stream=stream)
                row = one.cpu().numpy()
        return corrupt

    # erasure-encode.go:75-113
    def Encode(self, src, writers: list, buf, quorum: int) -> int:
        """Erasure.Encode: read `src` (a file-like) in blockSize pieces into the bpool
        buffer `buf` (capacity >= 2*blockSize), encode + hash each block on the device
        (EncodeDataWithSums) and hand it to parallelWriter.  Returns the byte count;
        raises ErasureWriteQuorum like the reference."""
        arr = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
        w = ParallelWriter(writers, quorum)
        total = 0
        bs = self.blockSize
        while True:
            chunk = src.read(bs)
            n = len(chunk)
            eof = n < bs
            if n == 0 and total != 0:
                break
            arr[:n] = np.frombuffer(chunk, np.uint8)
            # n == 0 and total == 0: empty data and parity files
            blocks, sums = self.EncodeDataWithSums(arr, n)
            w.Write(blocks, None if sums is None else [sums[i].tobytes() for i in range(len(blocks))])
            total += n
            if eof:
                break
        return total

    # erasure-decode.go:206-282
    def Decode(self, writer, readers: list, offset: int, length: int, total_length: int, prefer=None):
        """Erasure.Decode: returns (written, derr) where derr is errFileNotFound /
        errFileCorrupt when a reader failed that way but the read still succeeded;
        raises ZS3Error(errInvalidArgument) / ErasureReadQuorum like the reference."""
        if offset < 0 or length < 0:
            raise ZS3Error(ERR_INVALID_ARGUMENT, "Decode")
        if offset + length > total_length:
            raise ZS3Error(ERR_INVALID_ARGUMENT, "Decode")
        if length == 0:
            return 0, None
        reader = ParallelReader(readers, self, offset, total_length)
        if prefer is not None and len(prefer) == len(readers):
            reader.prefer_readers(prefer)
        bs = self.blockSize
        start_block, end_block = offset // bs, (offset + length) // bs
        written, derr = 0, None
        for block in range(start_block, end_block + 1):
            if start_block == end_block:
                boff, blen = offset % bs, length
            elif block == start_block:
                boff = offset % bs
                blen = bs - boff
            elif block == end_block:
                boff, blen = 0, (offset + length) % bs
            else:
                boff, blen = 0, bs
            if blen == 0:
                break
            bufs, err = reader.Read()
            if err in (ERR_FILE_NOT_FOUND, ERR_FILE_CORRUPT_NAME) and derr is None:
                derr = err
            self.DecodeDataBlocks(bufs)
            written += write_data_blocks(bufs, self.dataBlocks, boff, blen, dst=writer)
        if written != length:
            raise ZS3Error(ERR_SHORT_DATA, "Decode: errLessData")
        return written, derr

    # erasure-decode.go:285-332
    def Heal(self, writers: list, readers: list, total_length: int):
        """Erasure.Heal: read + DecodeDataAndParityBlocks + parallelWriter with write
        quorum 1 per block; the rebuilt chunks' sums come from one device launch per
        block.  Returns derr (errFileNotFound / errFileCorrupt or None)."""
        from . import MAGIC_HH256_KEY, hh256_batch
        if len(writers) != self.parityBlocks + self.dataBlocks:
            raise ZS3Error(ERR_INVALID_ARGUMENT, "Heal")
        reader = ParallelReader(readers, self, 0, total_length)
        end_block = total_length // self.blockSize + (1 if total_length % self.blockSize else 0)
        derr = None
        for _ in range(end_block):
            bufs, err = reader.Read()
            if err in (ERR_FILE_NOT_FOUND, ERR_FILE_CORRUPT_NAME) and derr is None:
                derr = err
            self.DecodeDataAndParityBlocks(bufs)
            sums = _hash_chunks(bufs, MAGIC_HH256_KEY, hh256_batch)
            ParallelWriter(writers, 1).Write(bufs, sums)
        return derr

    def ShardSize(self) -> int:
        return self._codec.shard_size()

    def ShardFileSize(self, total_length: int) -> int:
        return self._codec.shard_file_size(total_length)

    def ShardFileOffset(self, start_offset: int, length: int, total_length: int) -> int:
        return self._codec.shard_file_offset(start_offset, length, total_length)


def _hash_chunks(bufs: list, key: bytes, hh256_batch) -> list:
    """HighwayHash-256 of k+m equal-length chunks in one device launch."""
    import torch
    L = len(bufs[0])
    if L == 0:
        return None
    n = len(bufs)
    stride = max(16, -(-L // 16) * 16)
    host = np.zeros(n * stride, np.uint8)
    for i, c in enumerate(bufs):
        host[i * stride: i * stride + L] = np.asarray(c, dtype=np.uint8)
    d = torch.from_numpy(host).to("cuda")
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    hh256_batch(d, stride, L, n, out, key=key)
    o = out.cpu().numpy().reshape(n, 32)
    return [o[i].tobytes() for i in range(n)]


# ---------------------------------------------------------------------------------------
# The rocm build's codec cache (getGPUCodec), mirrored so the tests can
# drive it.  NewErasure(k, m, blockSize) is called per request with the object's own block
# size (cmd/erasure-object.go:283 with fi.Erasure.BlockSize, erasure-healing.go:467-468):
# blockSizeV2 = 1 MiB for new objects, blockSizeV1 = 10 MiB for legacy ones
# (cmd/object-api-common.go:37-40).  A queue batches blocks of ONE shard size, and a full
# block is exactly its codec's block size, so the cache is keyed by (k, m, blockSize): a
# legacy object's full 10 MiB blocks batch together in their own queue, and a 1 MiB
# object's full blocks are never mistaken for short blocks of a 10 MiB queue (nor
# rejected by it).
QUEUE_BATCH_BYTES = 64 << 20  # input bytes per device batch (queue_policy.hpp kBatchInputBytes)
QUEUE_MIN_BATCH, QUEUE_MAX_BATCH = 8, 512


def queue_max_batch(k: int, m: int, block_size: int) -> int:
    """Blocks per queue batch for a block size: the library's own rule
    (zs3server_amd/csrc/queue_policy.hpp slot_blocks with max_batch 0): 64 MiB of input,
    at least 8 and at most 512 blocks (RS(8+4) at 1 MiB: 64; at blockSizeV1 = 10 MiB: 8).
    The staging slots are sized to it; the shim passes max_batch 0."""
    return max(QUEUE_MIN_BATCH, min(QUEUE_MAX_BATCH, QUEUE_BATCH_BYTES // block_size))


class GPUCodec:
    """gpuCodec: the (k, m, blockSize) coding matrix and its batching
    queue, shared by every request of that geometry and block size."""

    def __init__(self, k: int, m: int, block_size: int, queue_factory=None):
        from . import Queue
        self.key = (k, m, block_size)
        self.codec = Codec(k, m, block_size)  # ErrInvShardNum / ErrMaxShardNum as NewErasure
        devices = gpu_devices()
        factory = queue_factory or (lambda c, mb: Queue(c, max_batch=0, max_wait_us=200, slots=4, devices=devices))
        self.max_batch = queue_max_batch(k, m, block_size)
        self.queue = factory(self.codec, self.max_batch)

    def encode_data(self, buf, length: int, sums: bool = True):
        """encodeDataGPU: Split + Encode in place (+ the k+m bitrot sums) through the queue."""
        return self.queue.encode_data(buf, length, sums=sums)

    def decode(self, shards, present, data_only: bool, expect=None, bad=None, sums_out=None) -> int:
        """reconstructGPU: DecodeDataBlocks / DecodeDataAndParityBlocks (+ verify / heal sums)."""
        return self.queue.decode(shards, present, data_only, expect=expect, bad=bad, sums_out=sums_out)


def gpu_devices() -> list:
    """The GPUs a queue spreads its blocks over: the current device
    only (an empty list: the queue's `device` option, -1 = current) unless
    ZS3_QUEUE_DEVICES (a comma list of HIP ordinals, e.g. "0,1,2,3,4,5,6,7") opts in to
    several.  The multi-device queue has run on one GPU only ([0, 0]):
    until a node-level run checks its parity and scaling it is not the default (ADVICE r05;
    each listed device also takes its own pinned + HBM staging, §2's footprint)."""
    env = os.environ.get("ZS3_QUEUE_DEVICES")
    if env:
        return [int(x) for x in env.split(",") if x.strip()]
    return []


# ---- per-block routing: host or device -----------------------------
# The reference encodes / decodes every block on the calling goroutine's core
# (cmd/erasure-encode.go:83-111, cmd/erasure-decode.go:230-276, klauspost/reedsolomon +
# HighwayHash).  Through the queue a block costs a PCIe round trip plus batching, so the
# device only wins once enough requests are in flight.  Device side (tools/queue_bench,
# profiles/r06/queue_product.jsonl, queue_product2.jsonl: RS(8+4) 1 MiB encode + sums,
# synchronous submitters, split copy streams, seal point 33 %): a lone block takes
# QUEUE_LONE_S (p50 305-310 us pinned; GET / heal 527 us) and the queue
# approaches QUEUE_MAX_BPS per device; with T submitters Little's law gives
# T*B / (lone + (T-1)*B/max): 23.9 / 35.3 GiB/s at T = 16 / 64 against 22.3 / 40.3-42.9
# measured (256 submitters: modelled 40.1, measured 30-41: there the box's 16-core share
# runs 256 submitter threads and the device waits for the host).  The model undershoots
# the 64-submitter rate: it keeps a block on the host a little longer, never shorter.  Host side: one core runs one
# block at CPU_CORE_BPS (oracle/cpu_ref.cpp, the reference's AVX-512 GFNI + AVX2 structure,
# BENCH_r05 cpu_baseline.t1: 5.35 GiB/s encode + sums; heal 6.4, §13.4), so T requests on
# `host_cores` cores run at min(T, host_cores) x that.
QUEUE_LONE_S = {"encode": 306e-6, "get": 527e-6, "heal": 527e-6}   # 1 MiB RS(8+4) block
QUEUE_LONE_BYTES = 1 << 20
QUEUE_FIXED_S = 240e-6               # the part of a lone block that does not scale with its size
QUEUE_MAX_BPS = 42 * 2**30           # per device (one PCIe x16 link), profiles/r06/queue_product*.jsonl
CPU_CORE_BPS = {"encode": 5.35 * 2**30, "get": 6.4 * 2**30, "heal": 6.4 * 2**30}


def device_codec_Bps(op: str, live: int, block_bytes: int, devices: int = 1) -> float:
    """Modelled queue throughput (object bytes/s) with `live` synchronous submitters."""
    if live <= 0 or block_bytes <= 0:
        return 0.0
    lone = QUEUE_FIXED_S + (QUEUE_LONE_S[op] - QUEUE_FIXED_S) * block_bytes / QUEUE_LONE_BYTES
    cap = QUEUE_MAX_BPS * max(1, devices)
    return live * block_bytes / (lone + (live - 1) * block_bytes / cap)


def host_codec_Bps(op: str, live: int, host_cores: int, cpu_Bps: float | None = None) -> float:
    """The reference structure's throughput: one block per request per core."""
    r = CPU_CORE_BPS[op] if cpu_Bps is None else cpu_Bps
    return min(max(0, live), max(0, host_cores)) * r


def codec_on_device(op: str, live: int, block_bytes: int, host_cores: int, devices: int = 1,
                    cpu_Bps: float | None = None) -> bool:
    """Where the rocm build runs one per-block EncodeData (op "encode"), GET
    DecodeDataBlocks ("get") or heal DecodeDataAndParityBlocks ("heal") with `live`
    requests of that kind in flight (this one included): True = the batching queue,
    False = the reference's own klauspost/reedsolomon + HighwayHash path on the calling
    goroutine.  `host_cores` = cores the server lets erasure coding use.  A lone 1 MiB
    request stays on the host (306-527 us through the device against ~190 us on one core);
    the device takes over once the queue's modelled rate beats min(live, host_cores) cores
    — with a whole 16-core host budget that is never on one GPU (30-43 GiB/s against 86),
    with 2 cores from 5 encode submitters, with 4 from 13.  (Legacy 10 MiB blocks: the
    lone-block time is extrapolated from the 1 MiB measurement — fixed 240 us + the rest
    scaled by size — and puts even a lone 10 MiB block on the device.)  Monotone: more
    live requests never move a block back to the host, more host cores never move one to
    the device."""
    if live <= 0 or block_bytes <= 0:
        return False
    return device_codec_Bps(op, live, block_bytes, devices) > host_codec_Bps(op, live, host_cores, cpu_Bps)


def codec_device_threshold(op: str, block_bytes: int, host_cores: int, devices: int = 1, max_live: int = 1 << 16):
    """Smallest live-request count that codec_on_device sends to the device (None: never)."""
    for t in range(1, max_live + 1):
        if codec_on_device(op, t, block_bytes, host_cores, devices):
            return t
    return None


_GPU_CODECS: dict = {}
_GPU_CODECS_MU = threading.Lock()


def get_gpu_codec(k: int, m: int, block_size: int, queue_factory=None) -> GPUCodec:
    """getGPUCodec: the process-wide GPUCodec of (k, m, blockSize), created on first use
    (LoadOrStore: concurrent first callers get the same one)."""
    key = (k, m, block_size)
    c = _GPU_CODECS.get(key)
    if c is not None:
        return c
    with _GPU_CODECS_MU:
        c = _GPU_CODECS.get(key)
        if c is None:
            c = GPUCodec(k, m, block_size, queue_factory)
            _GPU_CODECS[key] = c
        return c


def drop_gpu_codecs() -> None:
    """Release every cached codec and queue (tests; process shutdown flushes them)."""
    with _GPU_CODECS_MU:
        for c in _GPU_CODECS.values():
            close = getattr(c.queue, "close", None)
            if close:
                close()
        _GPU_CODECS.clear()


def NewErasure(data_blocks: int, parity_blocks: int, block_size: int) -> Erasure:
    """cmd/erasure-coding.go:42."""
    return Erasure(data_blocks, parity_blocks, block_size)


def get_data_block_len(en_blocks: list, data_blocks: int) -> int:
    """erasure-utils.go:32."""
    return sum(len(b) for b in en_blocks[:data_blocks] if b is not None)


def write_data_blocks(en_blocks: list, data_blocks: int, offset: int, length: int, dst=None):
    """erasure-utils.go:43-119: concatenate data shards [offset, offset+length).
    Writes to `dst` (a file-like) if given and returns the byte count, else returns bytes."""
    if offset < 0 or length < 0:
        raise ZS3Error(ERR_INVALID_ARGUMENT, "writeDataBlocks")
    if len(en_blocks) < data_blocks:
        raise ZS3Error(ERR_TOO_FEW_SHARDS, "writeDataBlocks")
    if get_data_block_len(en_blocks, data_blocks) < length:
        raise ZS3Error(ERR_SHORT_DATA, "writeDataBlocks")
    out = io.BytesIO() if dst is None else dst
    write = length
    total = 0
    for block in en_blocks[:data_blocks]:
        block = bytes(block)
        if offset >= len(block):
            offset -= len(block)
            continue
        block = block[offset:]
        offset = 0
        if write < len(block):
            out.write(block[:write])
            total += write
            break
        out.write(block)
        write -= len(block)
        total += len(block)
    return out.getvalue() if dst is None else total
