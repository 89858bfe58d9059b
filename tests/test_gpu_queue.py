"""GPU parity of the cross-request batching queue (zs3_queue_*, SURVEY.md §8b
Threading): concurrent submitter threads — the stand-in for goroutines calling
Erasure.EncodeData / DecodeDataBlocks per 1 MiB block inside cgo
(cmd/erasure-encode.go:83-111, cmd/erasure-decode.go:230-276) — get bit-exact results
while the queue gathers their blocks into shared device batches.

Every expected value comes from the scalar oracle (oracle/zs3_oracle.c).
"""
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402

KEY = z.MAGIC_HH256_KEY


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()


def run_threads(n, fn):
    errs = []

    def wrap(t):
        try:
            fn(t)
        except BaseException as e:  # noqa: BLE001 - re-raised in the main thread
            errs.append((t, e))

    th = [threading.Thread(target=wrap, args=(t,)) for t in range(n)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    if errs:
        raise errs[0][1]


@pytest.mark.parametrize("k,m,bs", [(8, 4, 1 << 20), (4, 2, 1 << 16), (16, 4, 1 << 16), (5, 3, 100000)])
def test_queue_encode_8_threads(oracle, k, m, bs):
    """8 threads each push an 'object' (full blocks + a ragged last block, as the
    Erasure.Encode block loop does) through the queue: parity in place in the caller's
    buffer, Split zero-fill, bitrot sums, all vs the oracle; the queue batched them."""
    codec = z.Codec(k, m, bs)
    q = z.Queue(codec, max_batch=16, max_wait_us=300)
    R = k + m
    mat = oracle.build_matrix(k, m)
    nblocks = 3 if bs >= 1 << 20 else 6
    tails = [0, 1, 17, bs // 3 + 5, bs - 1, 33, 1000, 7]

    def obj(t):
        lens = [bs] * nblocks + ([tails[t]] if tails[t] else [])
        for i, ln in enumerate(lens):
            data = oracle.fill(100 + t, i, ln)
            S = -(-ln // k)
            buf = np.full(R * S + 64, 0xEE, dtype=np.uint8)  # capacity > (k+m)*S, junk after len
            buf[:ln] = data
            got_S, sums = q.encode_data(buf, ln)
            assert got_S == S
            want = oracle.encode_data(k, m, data, mat)
            assert np.array_equal(buf[:R * S].reshape(R, S), want), (t, i)
            assert np.array_equal(sums, oracle.hh256_rows(KEY, want)), (t, i)

    run_threads(8, obj)
    batches, blocks = q.stats()
    assert blocks == sum(nblocks + (1 if tails[t] else 0) for t in range(8))
    q.close()


def test_queue_encode_empty_block():
    codec = z.Codec(8, 4, 1 << 16)
    q = z.Queue(codec)
    S, _ = q.encode_data(np.zeros(16, np.uint8), 0)
    assert S == 0  # EncodeData of 0 bytes: nothing to do
    q.close()


def _stripe(oracle, k, m, bs, seed, b, ln=None):
    ln = bs if ln is None else ln
    mat = oracle.build_matrix(k, m)
    sh = oracle.encode_data(k, m, oracle.fill(seed, b, ln), mat)
    return sh, oracle.hh256_rows(KEY, sh)


@pytest.mark.parametrize("k,m,bs", [(8, 4, 1 << 20), (4, 2, 1 << 16), (16, 4, 1 << 16), (5, 3, 100000)])
def test_queue_decode_mixed_patterns_8_threads(oracle, k, m, bs):
    """8 threads decode blocks with per-block erasure patterns (GET: DecodeDataBlocks
    with the survivors verified; HEAL: all missing rows + their sums), including a
    rotted survivor (errFileCorrupt + its flag), too few shards (ErrTooFewShards) and a
    short last block; every block vs the oracle."""
    codec = z.Codec(k, m, bs)
    q = z.Queue(codec, max_batch=8, max_wait_us=300)
    R = k + m
    rng_master = np.random.default_rng(k * 31 + m)
    seeds = rng_master.integers(0, 1 << 30, size=8)

    def worker(t):
        rng = np.random.default_rng(int(seeds[t]))
        for i in range(5):
            short = i == 4
            ln = (bs // 2 + 3) if short else bs
            sh, sums = _stripe(oracle, k, m, bs, 200 + t, i, ln)
            S = sh.shape[1]
            heal = bool(rng.integers(0, 2))
            e = int(rng.integers(0, m + 1))
            missing = rng.choice(R, size=e, replace=False)
            present = np.ones(R, bool)
            present[missing] = False
            work = sh.copy()
            work[~present] = 0x5A
            kind = int(rng.integers(0, 5))
            if kind == 0 and e < m:  # one survivor rotted on disk
                j = [x for x in range(R) if present[x]][0]
                work[j, S // 2] ^= 1
                bad = np.zeros(R, np.int32)
                rc = q.decode(work, present, not heal, expect=sums, bad=bad)
                assert rc == -7, (t, i, rc)
                want = np.zeros(R, np.int32)
                want[j] = 1
                assert np.array_equal(bad, want), (t, i)
                continue
            if kind == 1:  # more than m lost
                lost = rng.choice(R, size=m + 1, replace=False)
                present2 = np.ones(R, bool)
                present2[lost] = False
                assert q.decode(work.copy(), present2, True, expect=sums) == -3
                continue
            out = np.zeros((R, 32), np.uint8) if heal else None
            bad = np.full(R, 9, np.int32)
            rc = q.decode(work, present, not heal, expect=sums, bad=bad, sums_out=out)
            assert rc == 0, (t, i, rc)
            assert not bad.any()
            for r in range(R):
                if present[r] or r < k or heal:
                    assert np.array_equal(work[r], sh[r]), (t, i, r)
                else:
                    assert (work[r] == 0x5A).all(), "DecodeDataBlocks leaves missing parity alone"
            if heal:
                for r in np.nonzero(~present)[0]:
                    assert np.array_equal(out[r], sums[r]), (t, i, r)

    run_threads(8, worker)
    q.close()


def test_queue_mixed_encode_and_decode_concurrently(oracle):
    """Encoders and decoders share one queue (separate lanes, same device)."""
    k, m, bs = 8, 4, 1 << 16
    codec = z.Codec(k, m, bs)
    q = z.Queue(codec, max_batch=32)
    R = k + m
    mat = oracle.build_matrix(k, m)

    def worker(t):
        for i in range(12):
            if t % 2 == 0:
                data = oracle.fill(300 + t, i, bs)
                buf = np.zeros(R * (bs // k), np.uint8)
                buf[:bs] = data
                S, sums = q.encode_data(buf, bs)
                want = oracle.encode_data(k, m, data, mat)
                assert np.array_equal(buf.reshape(R, S), want)
                assert np.array_equal(sums, oracle.hh256_rows(KEY, want))
            else:
                sh, sums = _stripe(oracle, k, m, bs, 400 + t, i)
                present = np.ones(R, bool)
                present[[i % k, (i + 5) % R]] = False
                work = sh.copy()
                work[~present] = 0
                assert q.decode(work, present, True, expect=sums) == 0
                assert np.array_equal(work[:k], sh[:k])

    run_threads(8, worker)
    batches, blocks = q.stats()
    assert blocks == 8 * 12
    q.close()


@pytest.mark.parametrize("k,m,bs", [(8, 4, 1 << 16), (4, 4, 1 << 20), (2, 2, 1 << 20), (3, 3, 1 << 16)])
def test_queue_batches_concurrent_blocks(oracle, k, m, bs):
    """Under concurrency the queue forms multi-block batches (fewer launches than
    blocks): 16 threads x 8 blocks, async submits, then waits.  k == m (RS(2+2), RS(3+3),
    RS(4+4): the 4-, 6- and 8-drive defaults) gives the slot's data and parity regions
    equal strides, which the encode layout check once rejected for every batch of two or
    more full blocks."""
    codec = z.Codec(k, m, bs)
    q = z.Queue(codec, max_batch=64, max_wait_us=2000)
    R = k + m
    mat = oracle.build_matrix(k, m)
    S = -(-bs // k)

    def worker(t):
        bufs, reqs, sums = [], [], []
        for i in range(8):
            b = np.zeros(R * S, np.uint8)
            b[:bs] = oracle.fill(500 + t, i, bs)
            s = np.zeros(R * 32, np.uint8)
            bufs.append(b)
            sums.append(s)
            reqs.append(q.submit_encode(b, bs, s))
        for i, r in enumerate(reqs):
            assert q.wait(r) == S
            want = oracle.encode_data(k, m, oracle.fill(500 + t, i, bs), mat)
            assert np.array_equal(bufs[i].reshape(R, S), want)
            assert np.array_equal(sums[i].reshape(R, 32), oracle.hh256_rows(KEY, want))

    run_threads(16, worker)
    batches, blocks = q.stats()
    assert blocks == 128 and batches < blocks
    q.close()


@pytest.mark.parametrize("k,m,bs,zc_mode", [(8, 4, 1 << 20, 1), (5, 3, 100000, 1), (12, 4, 1 << 20, 1),
                                             (10, 4, 1 << 20, 1), (8, 4, 1 << 20, 2), (12, 4, 1 << 20, 2),
                                             (8, 4, 1 << 20, 3), (12, 4, 1 << 20, 3), (10, 4, 1 << 20, 3)])
def test_queue_zero_copy_pinned_callers(oracle, k, m, bs, zc_mode, monkeypatch):
    """Callers whose block buffers come from zs3_host_alloc (the pinned bpool) are
    served zero-copy (the DMA engine reads the data rows from, and writes the parity
    rows / rebuilt rows into, the caller's buffer), side by side in the same batches
    with pageable callers and with pinned callers' short last blocks (staged); every
    result vs the oracle, and the queue reports the zero-copy blocks.  RS(12+4) (the
    16-drive default, UA kernel) and RS(10+4) (any-geometry kernel) at 1 MiB have Split
    padding (k*S > blockSize): a zero-copy block DMAs only its `len` data bytes, so the
    slot's padding bytes hold whatever the slot's previous batch left there, and every
    encode kernel must read them as zero.  Pinned-caller modes (queue.hip,
    ZS3_QUEUE_ZC, diagnostics build only): 1 = zero-copy for a lone caller's block (first
    of its batch, no other batch of the lane in flight), the rest staged (the default and
    the product library's only mode); 2 = every full block by a DMA of its own; 3 =
    copy-list kernels over the mapped pinned pages."""
    # the ZS3_QUEUE_ZC switch is read by the diagnostics build only (the product library
    # always runs mode 1); a codec and its queue belong to the library that made them
    monkeypatch.setenv("ZS3_QUEUE_ZC", str(zc_mode))
    R = k + m
    S = -(-bs // k)
    mat = oracle.build_matrix(k, m)
    nthr, per = 8, 4
    with z.diag(0):
        codec = z.Codec(k, m, bs)
        q = z.Queue(codec, max_batch=16, max_wait_us=500)
        # pinned ranges are registered per library: allocate from the queue's library
        pins = [z.HostBuffer(R * S + 64) for _ in range(nthr)]
        pins_dec = [z.HostBuffer(R * S) for _ in range(nthr)]

    def worker(t):
        pinned = t % 2 == 0
        for i in range(per):
            short = i == per - 1 and t % 4 == 0
            ln = bs // 3 + 7 if short else bs
            data = oracle.fill(700 + t, i, ln)
            Sb = -(-ln // k)
            buf = pins[t].array[:R * Sb + 64] if pinned else np.zeros(R * Sb + 64, np.uint8)
            buf[:] = 0xEE
            buf[:ln] = data
            got_S, sums = q.encode_data(buf, ln)
            want = oracle.encode_data(k, m, data, mat)
            assert got_S == Sb
            assert np.array_equal(buf[:R * Sb].reshape(R, Sb), want), (t, i)
            assert np.array_equal(sums, oracle.hh256_rows(KEY, want)), (t, i)
            # GET / heal of a full stripe from the pinned (or pageable) caller buffer
            sh, ssum = _stripe(oracle, k, m, bs, 800 + t, i)
            work = pins_dec[t].array.reshape(R, S) if pinned else np.zeros((R, S), np.uint8)
            work[:] = sh
            present = np.ones(R, bool)
            present[[(i + t) % k, k + (t % m)]] = False
            work[~present] = 0x5A
            heal = i % 2 == 1
            out = np.zeros((R, 32), np.uint8) if heal else None
            bad = np.full(R, 9, np.int32)
            assert q.decode(work, present, not heal, expect=ssum, bad=bad, sums_out=out) == 0, (t, i)
            assert not bad.any()
            for r in range(R):
                if present[r] or r < k or heal:
                    assert np.array_equal(work[r], sh[r]), (t, i, r)
                else:
                    assert (work[r] == 0x5A).all(), "DecodeDataBlocks leaves missing parity alone"
            if heal:
                for r in np.nonzero(~present)[0]:
                    assert np.array_equal(out[r], ssum[r]), (t, i, r)

    run_threads(nthr, worker)
    batches, blocks = q.stats()
    assert blocks == nthr * per * 2
    zc = q.zero_copy_blocks()
    # pinned threads: every full encode block and every decode block (modes 2, 3); mode 1
    # only those that opened their batch with no other batch of the lane in flight
    n_short = sum(1 for t in range(0, nthr, 2) if t % 4 == 0)
    if zc_mode == 1:
        assert 0 <= zc <= (nthr // 2) * per * 2 - n_short, zc
    else:
        assert zc == (nthr // 2) * per * 2 - n_short, zc
    q.close()
    for p in pins + pins_dec:
        p.free()


@pytest.mark.parametrize("k,m", [(12, 4), (8, 4)])
def test_queue_lone_pinned_caller_zero_copy(oracle, k, m):
    """Default pinned-caller mode (ZS3_QUEUE_ZC=1): a lone synchronous caller (each block
    submitted and waited for before the next) takes the zero-copy path for every full
    block, encode and decode (queue.hip zc_mode); results vs the oracle.  RS(12+4) on
    1 MiB blocks has Split padding, which the zero-copy DMA does not write."""
    bs = 1 << 20
    codec = z.Codec(k, m, bs)
    q = z.Queue(codec, max_batch=16, max_wait_us=500)
    R = k + m
    S = -(-bs // k)
    mat = oracle.build_matrix(k, m)
    pin = z.HostBuffer(R * S + 64)
    try:
        n = 3
        for i in range(n):
            data = oracle.fill(900 + k, i, bs)
            buf = pin.array[:R * S + 64]
            buf[:] = 0xEE
            buf[:bs] = data
            got_S, sums = q.encode_data(buf, bs)
            want = oracle.encode_data(k, m, data, mat)
            assert got_S == S
            assert np.array_equal(buf[:R * S].reshape(R, S), want), i
            assert np.array_equal(sums, oracle.hh256_rows(KEY, want)), i
        sh, ssum = _stripe(oracle, k, m, bs, 950 + k, 0)
        work = pin.array[:R * S].reshape(R, S)
        work[:] = sh
        present = np.ones(R, bool)
        present[[1, k]] = False
        work[~present] = 0x5A
        bad = np.full(R, 9, np.int32)
        assert q.decode(work, present, True, expect=ssum, bad=bad) == 0
        assert not bad.any()
        assert np.array_equal(work[1], sh[1])
        assert q.zero_copy_blocks() == n + 1
    finally:
        q.close()
        pin.free()


@pytest.mark.parametrize("k,m,bs", [(8, 4, 1 << 20), (12, 4, 1 << 20), (4, 4, 1 << 16)])
def test_queue_multi_device_16_threads(oracle, k, m, bs):
    """A multi-device queue (zs3_queue_opts.devices; here both entries are device 0, the
    box has one GPU): 16 submitter threads encode and decode / heal through it, every
    result vs the oracle, and both device parts received blocks and launched batches of
    their own (the assignment policy itself is checked on the CPU, tests/test_queue_policy.py)."""
    codec = z.Codec(k, m, bs)
    q = z.Queue(codec, max_wait_us=300, devices=[0, 0])
    R = k + m
    S = -(-bs // k)
    mat = oracle.build_matrix(k, m)

    def worker(t):
        for i in range(6):
            data = oracle.fill(1100 + t, i, bs)
            buf = np.zeros(R * S + 32, np.uint8)
            buf[:bs] = data
            got_S, sums = q.encode_data(buf, bs)
            want = oracle.encode_data(k, m, data, mat)
            assert got_S == S
            assert np.array_equal(buf[:R * S].reshape(R, S), want), (t, i)
            assert np.array_equal(sums, oracle.hh256_rows(KEY, want)), (t, i)
            if i % 2:
                sh, ssum = want, oracle.hh256_rows(KEY, want)
                work = sh.copy()
                present = np.ones(R, bool)
                present[[(i + t) % k, k + (t % m)]] = False
                work[~present] = 0x5A
                heal = t % 2 == 1
                out = np.zeros((R, 32), np.uint8) if heal else None
                bad = np.full(R, 9, np.int32)
                assert q.decode(work, present, not heal, expect=ssum, bad=bad, sums_out=out) == 0, (t, i)
                assert not bad.any()
                for r in range(R):
                    if present[r] or r < k or heal:
                        assert np.array_equal(work[r], sh[r]), (t, i, r)
                if heal:
                    for r in np.nonzero(~present)[0]:
                        assert np.array_equal(out[r], ssum[r]), (t, i, r)

    run_threads(16, worker)
    batches, blocks = q.stats()
    assert blocks == 16 * 6 + 16 * 3
    per = [q.device_stats(i) for i in range(2)]
    assert [d for d, _, _ in per] == [0, 0]
    assert sum(n for _, _, n in per) == blocks and sum(b for _, b, _ in per) == batches
    assert all(n > 0 and b > 0 for _, b, n in per), per
    # the assignment keeps the two parts within a few blocks of each other
    assert abs(per[0][2] - per[1][2]) <= 16, per
    q.close()
