"""Mirror of the reference's Erasure API over the zs3gpu C ABI.

Same names, argument meaning and error behaviour as cmd/erasure-coding.go and
cmd/erasure-utils.go, so tests read like the reference's own (erasure_test.go).
Shards are Python lists of numpy uint8 views (None = missing, the Go nil/len 0).
All arithmetic runs in the HIP kernels (host-staged through pinned memory).
"""
from __future__ import annotations

import io

import numpy as np

from . import Codec, ZS3Error

BLOCK_SIZE_V1 = 10 << 20  # cmd/object-api-common.go:37
BLOCK_SIZE_V2 = 1 << 20   # cmd/object-api-common.go:40

ERR_INV_SHARD_NUM, ERR_MAX_SHARD_NUM, ERR_TOO_FEW_SHARDS = -1, -2, -3
ERR_SHARD_NO_DATA, ERR_SHARD_SIZE, ERR_SHORT_DATA = -4, -5, -6
ERR_FILE_CORRUPT, ERR_INVALID_ARGUMENT = -7, -8


class ErasureReadQuorum(Exception):
    """errErasureReadQuorum (cmd/erasure-errors.go): fewer than k readable shards."""


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

    def ShardSize(self) -> int:
        return self._codec.shard_size()

    def ShardFileSize(self, total_length: int) -> int:
        return self._codec.shard_file_size(total_length)

    def ShardFileOffset(self, start_offset: int, length: int, total_length: int) -> int:
        return self._codec.shard_file_offset(start_offset, length, total_length)


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
