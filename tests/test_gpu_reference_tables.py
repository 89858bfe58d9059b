"""The reference's own Encode / Decode / Heal edge-case tables, run through the device
path (erasure.py Encode / Decode / Heal mirrors over the C ABI: fused encode + sums per
block, batched bitrot verify per read round, device reconstruct).

* cmd/erasure-encode_test.go:58-165 — TestErasureEncode's 20 cases: offline disks,
  writers closed with errFaultyDisk, write quorum k+1, empty objects.
* cmd/erasure-decode_test.go:35-200 — TestErasureDecode's 38 cases: offsets / lengths
  across blocks, invalid ranges, then the same read with the first offDisks readers on
  badDisk and reader 0 offline (read quorum).
* cmd/erasure-decode_test.go:205 — TestErasureDecodeRandomOffsetLength, RS(7+7) over
  5 MiB, 200 seeded ranges (the reference runs 10 000 unseeded ones).
* cmd/erasure-heal_test.go:29-161 — TestErasureHeal's 20 cases: offline (stale) disks,
  bad readers, bad stale writers; healed shard files must equal the originals byte for
  byte ([sum][chunk] framing: identical bitrot sums, :154).

Every case uses HighwayHash256S, the only algorithm new writes use
(xl-storage-format-v1.go:124-126); the tables' BLAKE2b512 / SHA256 entries exercise the
same erasure logic with the streaming format.  Data are seeded random bytes.
"""
import io

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402
from zs3server_amd import bitrot as zb  # noqa: E402
from zs3server_amd import erasure as ze  # noqa: E402

MiB = 1 << 20
BS2 = ze.BLOCK_SIZE_V2


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()


def rand_bytes(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def encode_object(er, data, n_disks, block_size):
    """Encode `data` onto n_disks in-memory shard files (bitrot writers); returns the
    files and the bytes written."""
    writers = [zb.StreamingBitrotWriter(er.ShardSize()) for _ in range(n_disks)]
    buf = np.zeros(2 * block_size, np.uint8)
    n = er.Encode(io.BytesIO(data), writers, buf, er.dataBlocks + 1)
    return [w.getvalue() for w in writers], n


def readers_for(er, files, offset, length, total):
    till = er.ShardFileOffset(offset, length, total)
    return [None if f is None else zb.StreamingBitrotReader(f, till, er.ShardSize()) for f in files]


# (dataBlocks, onDisks, offDisks, blocksize, data, offset, shouldFail, shouldFailQuorum)
ENCODE_TESTS = [
    (2, 4, 0, BS2, MiB, 0, False, False), (3, 6, 0, BS2, MiB, 1, False, False),
    (4, 8, 2, BS2, MiB, 2, False, False), (5, 10, 3, BS2, MiB, MiB, False, False),
    (6, 12, 4, BS2, MiB, MiB, False, False), (7, 14, 5, BS2, 0, 0, False, False),
    (8, 16, 7, BS2, 0, 0, False, False), (2, 4, 2, BS2, MiB, 0, False, True),
    (4, 8, 4, BS2, MiB, 0, False, True), (7, 14, 7, BS2, MiB, 0, False, True),
    (8, 16, 8, BS2, MiB, 0, False, True), (5, 10, 3, MiB, MiB, 0, False, False),
    (3, 6, 1, BS2, MiB, MiB // 2, False, False), (2, 4, 0, MiB // 2, MiB, MiB // 2 + 1, False, False),
    (4, 8, 0, MiB - 1, MiB, MiB - 1, False, False), (8, 12, 2, BS2, MiB, 2, False, False),
    (8, 10, 1, BS2, MiB, 0, False, False), (10, 14, 0, BS2, MiB, 17, False, False),
    (2, 6, 2, MiB, MiB, MiB // 2, False, False), (10, 16, 8, BS2, MiB, 0, False, True),
]


@pytest.mark.parametrize("i", range(len(ENCODE_TESTS)))
def test_erasure_encode_table(oracle, i):
    k, on, off, bs, size, offset, should_fail, should_fail_q = ENCODE_TESTS[i]
    er = ze.NewErasure(k, on - k, bs)
    data = rand_bytes(100 + i, size)[offset:]
    writers = [zb.StreamingBitrotWriter(er.ShardSize()) for _ in range(on)]
    buf = np.zeros(2 * bs, np.uint8)
    try:
        n = er.Encode(io.BytesIO(data), writers, buf, k + 1)
        err = None
    except ze.ErasureWriteQuorum as e:
        err = e
    assert (err is not None) == should_fail, f"case {i}: {err}"
    if err is not None:
        return
    assert n == len(data)
    files = [w.getvalue() for w in writers]
    assert all(len(f) == z.bitrot_shard_file_size(er.ShardFileSize(len(data)), er.ShardSize()) if len(data)
               else len(f) == 0 for f in files)
    # stronger than the reference: the shard files read back to the data
    if data:
        out = io.BytesIO()
        er.Decode(out, readers_for(er, files, 0, len(data), len(data)), 0, len(data), len(data))
        assert out.getvalue() == data, f"case {i}: round trip"
    # second pass: offDisks writers fail (closeWithErr(errFaultyDisk)), writer 0 offline
    writers = [zb.StreamingBitrotWriter(er.ShardSize()) for _ in range(on)]
    for j in range(off):
        writers[j].close_with_err("errFaultyDisk")
    if off > 0:
        writers[0] = None
    try:
        n = er.Encode(io.BytesIO(data), writers, buf, k + 1)
        err = None
    except ze.ErasureWriteQuorum as e:
        err = e
    assert (err is not None) == should_fail_q, f"case {i}: quorum {err}"
    if err is None:
        assert n == len(data)


# (dataBlocks, onDisks, offDisks, blocksize, data, offset, length, shouldFail, shouldFailQuorum)
DECODE_TESTS = [
    (2, 4, 0, BS2, MiB, 0, MiB, False, False), (3, 6, 0, BS2, MiB, 0, MiB, False, False),
    (4, 8, 0, BS2, MiB, 0, MiB, False, False), (5, 10, 0, BS2, MiB, 1, MiB - 1, False, False),
    (6, 12, 0, MiB, MiB, MiB, 0, False, False), (7, 14, 0, MiB, MiB, 3, 1024, False, False),
    (8, 16, 0, MiB, MiB, 4, 8 * 1024, False, False), (7, 14, 7, BS2, MiB, MiB, 1, True, False),
    (6, 12, 6, BS2, MiB, 0, MiB, False, False), (5, 10, 5, MiB, MiB, 0, MiB, False, False),
    (4, 8, 4, BS2, MiB, 0, MiB, False, False), (3, 6, 3, MiB, MiB, 0, MiB, False, False),
    (2, 4, 2, BS2, MiB, 0, MiB, False, False), (2, 4, 1, MiB, MiB, 0, MiB, False, False),
    (3, 6, 2, MiB, MiB, 0, MiB, False, False), (4, 8, 3, 2 * MiB, MiB, 0, MiB, False, False),
    (5, 10, 6, MiB, MiB, 0, MiB, False, True), (5, 10, 2, BS2, 2 * MiB, MiB, MiB, False, False),
    (5, 10, 1, BS2, MiB, 0, MiB, False, False), (6, 12, 3, BS2, MiB, 0, MiB, False, False),
    (6, 12, 7, BS2, MiB, 0, MiB, False, True), (8, 16, 8, BS2, MiB, 0, MiB, False, False),
    (8, 16, 9, MiB, MiB, 0, MiB, False, True), (8, 16, 7, BS2, MiB, 0, MiB, False, False),
    (2, 4, 1, BS2, MiB, 0, MiB, False, False), (2, 4, 0, BS2, MiB, 0, MiB, False, False),
    (2, 4, 0, BS2, BS2 + 1, 0, BS2 + 1, False, False), (2, 4, 0, BS2, 2 * BS2, 12, BS2 + 17, False, False),
    (3, 6, 0, BS2, 2 * BS2, 1023, BS2 + 1024, False, False), (4, 8, 0, BS2, 2 * BS2, 11, BS2 + 2 * 1024, False, False),
    (6, 12, 0, BS2, 2 * BS2, 512, BS2 + 8 * 1024, False, False), (8, 16, 0, BS2, 2 * BS2, BS2, BS2 - 1, False, False),
    (2, 4, 0, BS2, MiB, -1, 3, True, False), (2, 4, 0, BS2, MiB, 1024, -1, True, False),
    (4, 6, 0, BS2, BS2, 0, BS2, False, False), (4, 6, 1, BS2, 2 * BS2, 12, BS2 + 17, False, False),
    (4, 6, 3, BS2, 2 * BS2, 1023, BS2 + 1024, False, True), (8, 12, 4, BS2, 2 * BS2, 11, BS2 + 2 * 1024, False, False),
]


@pytest.mark.parametrize("i", range(len(DECODE_TESTS)))
def test_erasure_decode_table(oracle, i):
    k, on, off, bs, size, offset, length, should_fail, should_fail_q = DECODE_TESTS[i]
    er = ze.NewErasure(k, on - k, bs)
    data = rand_bytes(200 + i, size)
    files, n = encode_object(er, data, on, bs)
    assert n == size
    out = io.BytesIO()
    readers = readers_for(er, files, offset, length, size)
    try:
        er.Decode(out, readers, offset, length, size)
        err = None
    except (z.ZS3Error, ze.ErasureReadQuorum) as e:
        err = e
    assert (err is not None) == should_fail, f"case {i}: {err}"
    if err is not None:
        return
    assert out.getvalue() == data[offset:offset + length], f"case {i}: content"
    # same read with the first offDisks readers on badDisk and reader 0 offline
    readers = readers_for(er, files, offset, length, size)
    for j in range(off):
        readers[j] = zb.BadDiskReader()
    if off > 0:
        readers[0] = None
    out = io.BytesIO()
    try:
        er.Decode(out, readers, offset, length, size)
        err = None
    except (z.ZS3Error, ze.ErasureReadQuorum) as e:
        err = e
    assert (err is not None) == should_fail_q, f"case {i}: quorum {err}"
    if err is None:
        assert out.getvalue() == data[offset:offset + length], f"case {i}: content with bad disks"


def test_erasure_decode_random_offset_length(oracle):
    """TestErasureDecodeRandomOffsetLength: RS(7+7), 5 MiB object, 200 seeded ranges."""
    k, m, bs = 7, 7, MiB
    er = ze.NewErasure(k, m, bs)
    data = rand_bytes(7, 5 * MiB)
    files, n = encode_object(er, data, k + m, bs)
    assert n == len(data)
    rng = np.random.default_rng(2024)
    for _ in range(200):
        offset = int(rng.integers(0, len(data)))
        rlen = int(rng.integers(0, len(data) - offset))
        out = io.BytesIO()
        er.Decode(out, readers_for(er, files, offset, rlen, len(data)), offset, rlen, len(data))
        assert out.getvalue() == data[offset:offset + rlen], (offset, rlen)


def test_decode_reports_corrupt_shard_and_recovers(oracle):
    """A rotted chunk on one disk: Decode returns the data and errFileCorrupt (the heal
    trigger, erasure-decode.go:256-263), reading the next shard instead."""
    k, m, bs = 4, 2, MiB
    er = ze.NewErasure(k, m, bs)
    data = rand_bytes(9, 3 * MiB + 5)
    files, _ = encode_object(er, data, k + m, bs)
    bad = bytearray(files[1])
    bad[32 + 1000] ^= 1  # chunk 0 of shard 1
    files[1] = bytes(bad)
    out = io.BytesIO()
    readers = readers_for(er, files, 0, len(data), len(data))
    n, derr = er.Decode(out, readers, 0, len(data), len(data))
    assert n == len(data) and out.getvalue() == data
    assert derr == ze.ERR_FILE_CORRUPT_NAME
    assert readers[1] is None  # dropped upstream, as the Go slice is


# (dataBlocks, disks, offDisks, badDisks, badStaleDisks, blocksize, size, shouldFail)
HEAL_TESTS = [
    (2, 4, 1, 0, 0, BS2, MiB, False), (3, 6, 2, 0, 0, BS2, MiB, False), (4, 8, 2, 1, 0, BS2, MiB, False),
    (5, 10, 3, 1, 0, BS2, MiB, False), (6, 12, 2, 3, 0, BS2, MiB, False), (7, 14, 4, 1, 0, BS2, MiB, False),
    (8, 16, 6, 1, 1, BS2, MiB, False), (7, 14, 2, 3, 0, MiB // 2, MiB, False), (6, 12, 1, 0, 1, MiB - 1, MiB, True),
    (5, 10, 3, 0, 3, MiB // 2, MiB, True), (4, 8, 1, 1, 0, BS2, MiB, False), (2, 4, 1, 0, 1, BS2, MiB, True),
    (6, 12, 8, 3, 0, BS2, MiB, True), (7, 14, 3, 4, 0, BS2, MiB, False), (7, 14, 6, 1, 0, BS2, MiB, False),
    (8, 16, 4, 5, 0, BS2, MiB, True), (2, 4, 1, 0, 0, BS2, MiB, False), (12, 16, 2, 1, 0, BS2, MiB, False),
    (6, 8, 1, 0, 0, BS2, MiB, False), (2, 4, 1, 0, 0, BS2, 64 * MiB, False),
]


@pytest.mark.parametrize("i", range(len(HEAL_TESTS)))
def test_erasure_heal_table(oracle, i):
    k, nd, off, bad, bad_stale, bs, size, should_fail = HEAL_TESTS[i]
    assert off >= bad_stale
    er = ze.NewErasure(k, nd - k, bs)
    data = rand_bytes(300 + i, size)
    files, n = encode_object(er, data, nd, bs)
    assert n == size
    sfs = er.ShardFileSize(size)
    readers = [zb.StreamingBitrotReader(f, sfs, er.ShardSize()) for f in files]
    for j in range(off):
        readers[j] = None  # stale disks: nothing to read
    for j in range(bad):
        readers[off + j] = zb.BadDiskReader()
    stale = [zb.StreamingBitrotWriter(er.ShardSize()) if j < off else None for j in range(nd)]
    for j in range(bad_stale):
        stale[j].close_with_err("errFaultyDisk")  # CreateFile on badDisk
    try:
        er.Heal(stale, readers, size)
        err = None
    except (z.ZS3Error, ze.ErasureReadQuorum, ze.ErasureWriteQuorum) as e:
        err = e
    assert (err is not None) == should_fail, f"case {i}: {err}"
    if err is None:
        for j, w in enumerate(stale):
            if w is None:
                continue
            assert w.getvalue() == files[j], f"case {i}: healed shard file {j} differs (bitrot sums / chunks)"
