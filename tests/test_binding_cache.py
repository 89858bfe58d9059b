"""CPU tests of the rocm build's codec cache (INTEGRATION.md §2 getGPUCodec, mirrored by
zs3server_amd.erasure.get_gpu_codec): the cache key carries the object's block size, as
NewErasure(k, m, blockSize) does per request (cmd/erasure-object.go:283,
cmd/erasure-healing.go:467-468), so legacy blockSizeV1 = 10 MiB objects
(cmd/object-api-common.go:37) get their own codec and batching queue next to the 1 MiB
ones.  The queue factory is faked: no device call is made."""
import threading

import pytest

import zs3server_amd as z
from zs3server_amd import erasure as ze

MiB = 1 << 20


class FakeQueue:
    made = []

    def __init__(self, codec, max_batch):
        self.codec, self.max_batch = codec, max_batch
        self.closed = False
        FakeQueue.made.append(self)

    def close(self):
        self.closed = True


@pytest.fixture(autouse=True)
def fresh_cache():
    import __graft_entry__ as g
    g.build_lib()
    ze.drop_gpu_codecs()
    FakeQueue.made = []
    yield
    ze.drop_gpu_codecs()


def test_cache_key_includes_block_size():
    a = ze.get_gpu_codec(8, 4, ze.BLOCK_SIZE_V2, FakeQueue)
    b = ze.get_gpu_codec(8, 4, ze.BLOCK_SIZE_V1, FakeQueue)
    assert a is not b
    assert a.key == (8, 4, MiB) and b.key == (8, 4, 10 * MiB)
    assert a.codec.block_size == MiB and b.codec.block_size == 10 * MiB
    assert a.codec.shard_size() == MiB // 8 and b.codec.shard_size() == 10 * MiB // 8
    assert ze.get_gpu_codec(8, 4, MiB, FakeQueue) is a
    assert ze.get_gpu_codec(8, 4, 10 * MiB, FakeQueue) is b
    assert ze.get_gpu_codec(12, 4, MiB, FakeQueue) is not a
    assert len(FakeQueue.made) == 3


def test_concurrent_first_callers_share_one_codec():
    got = []
    barrier = threading.Barrier(16)

    def worker(bs):
        barrier.wait()
        got.append((bs, ze.get_gpu_codec(12, 4, bs, FakeQueue)))

    th = [threading.Thread(target=worker, args=(MiB if i % 2 else 10 * MiB,)) for i in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    by_bs = {}
    for bs, c in got:
        by_bs.setdefault(bs, set()).add(id(c))
    assert {bs: len(ids) for bs, ids in by_bs.items()} == {MiB: 1, 10 * MiB: 1}
    assert len(FakeQueue.made) == 2


@pytest.mark.parametrize("k,m,bs,want", [(8, 4, MiB, 64), (12, 4, MiB, 64), (4, 2, MiB, 64), (16, 4, MiB, 64),
                                         (8, 4, 10 * MiB, 8), (12, 4, 10 * MiB, 8), (2, 2, 64 * MiB, 8),
                                         (8, 4, 64 << 10, 512)])
def test_queue_batch_sized_by_bytes(k, m, bs, want):
    """Blocks per batch by input bytes, the library's rule (queue_policy.hpp slot_blocks):
    64 MiB of input, 8..512 blocks — RS(8+4) 1 MiB 64, legacy 10 MiB blocks 8."""
    c = ze.get_gpu_codec(k, m, bs, FakeQueue)
    assert c.max_batch == want == ze.queue_max_batch(k, m, bs)
    assert FakeQueue.made[-1].max_batch == want


def test_new_erasure_errors_surface_from_the_cache():
    with pytest.raises(z.ZS3Error) as ei:
        ze.get_gpu_codec(0, 4, MiB, FakeQueue)
    assert ei.value.code == ze.ERR_INV_SHARD_NUM
    assert not FakeQueue.made


def test_drop_closes_queues():
    ze.get_gpu_codec(8, 4, MiB, FakeQueue)
    ze.get_gpu_codec(8, 4, 10 * MiB, FakeQueue)
    ze.drop_gpu_codecs()
    assert all(q.closed for q in FakeQueue.made)


def test_write_quorum_reduction():
    """reduceWriteQuorumErrs (cmd/erasure-metadata-utils.go:36-87): ignored disk errors do
    not count; a non-ignored error reaching quorum is returned as itself."""
    from zs3server_amd.bitrot import DiskError
    assert ze.reduce_write_quorum_errs([None, None, "errFaultyDisk"], 2) is None
    with pytest.raises(ze.ErasureWriteQuorum):
        ze.reduce_write_quorum_errs([None, "errFaultyDisk", "errDiskNotFound", "errFaultyDisk"], 3)
    with pytest.raises(DiskError) as ei:
        ze.reduce_write_quorum_errs(["errDiskFull", "errDiskFull", "errDiskFull", None], 3)
    assert ei.value.name == "errDiskFull"


def test_parallel_writer_drops_any_failing_writer():
    """parallelWriter.Write (cmd/erasure-encode.go:48-60): any write error (not only disk
    errors) drops that writer and the loop still reaches the remaining writers."""
    import numpy as np

    class Boom:
        def Write(self, p):
            raise ValueError("errDiskFull")

    class Sink:
        def __init__(self):
            self.n = 0

        def Write(self, p):
            self.n += len(p)
            return len(p)

    ws = [Boom(), Sink(), Sink(), Boom()]
    blocks = [np.zeros(10, np.uint8)] * 4
    w = ze.ParallelWriter(ws, 2)
    w.Write(blocks)
    assert ws[0] is None and ws[3] is None and ws[1].n == 10 and ws[2].n == 10
    assert w.errs == ["errDiskFull", None, None, "errDiskFull"]


def test_parallel_reader_flags_bitrot_heal_on_reader_corruption(monkeypatch):
    """parallelReader.Read (cmd/erasure-decode.go:165-171): a reader that reports
    errFileCorrupt itself sets the bitrot-heal signal."""
    import numpy as np

    from zs3server_amd.bitrot import DiskError

    class E:
        dataBlocks, blockSize = 2, 64

        def ShardSize(self):
            return 32

        def ShardFileSize(self, total):
            return 32

    class Good:
        def read_raw(self, n, off):
            return b"\0" * 32, b"x" * n

    class Rot:
        def read_raw(self, n, off):
            raise DiskError("errFileCorrupt")

    monkeypatch.setattr(ze, "_verify_chunks", lambda chunks, wants: [False] * len(chunks))
    readers = [Rot(), Good(), Good()]
    r = ze.ParallelReader(readers, E(), 0, 64)
    bufs, err = r.Read()
    assert err == ze.ERR_FILE_CORRUPT_NAME
    assert bufs[0] is None and all(isinstance(b, np.ndarray) for b in bufs[1:])
