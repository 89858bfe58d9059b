"""GPU parity of the streamed GET / heal path (zs3_stream_decode):
one large object's Erasure.Decode / Erasure.Heal block loops (cmd/erasure-decode.go:230-276,
:287-332) handed to the device in pipelined batches instead of one device round trip per
block.  RS(12+4) (the 16-drive default) on 1 MiB blocks, 200 blocks plus a short last
block, with per-block erasure patterns (a reader dropping out mid-object), a rotted chunk
(flagged exactly: errFileCorrupt for that (block, shard)), pinned and pageable stripes.
Expected shards and sums: oracle/cpu_ref (pinned to the scalar oracle by
tests/test_cpuref_pin.py) and, for the short last block and a few sampled blocks, the
scalar oracle itself.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402

KEY = z.MAGIC_HH256_KEY
MiB = 1 << 20


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()


def make_object(oracle, k, m, nfull, tail, seed):
    """Stripes of an object (nfull full blocks + a tail block) in the zs3_stream_decode
    layout, with every shard and bitrot sum; returns (stripes, sums, S, tail S)."""
    from oracle import cpuref
    R = k + m
    S = -(-MiB // k)
    E = R * S
    nb = nfull + (1 if tail else 0)
    st = np.zeros(nb * E, np.uint8)
    for b in range(nfull):
        st[b * E: b * E + MiB] = oracle.fill(seed, b, MiB)
    sums = np.zeros((nb, R, 32), np.uint8)
    mat = oracle.build_matrix(k, m)
    par = st[k * S:]
    cpuref.encode_hash(k, m, mat, st, MiB, nfull, E, par, E, sums, KEY, cpuref.threads_available())
    St = 0
    if tail:
        data = oracle.fill(seed, nfull, tail)
        sh = oracle.encode_data(k, m, data, mat)
        St = sh.shape[1]
        st[nfull * E: nfull * E + R * St] = sh.reshape(-1)
        sums[nfull] = oracle.hh256_rows(KEY, sh)
    # spot-check cpu_ref against the scalar oracle on two full blocks
    for b in (0, nfull - 1):
        want = oracle.encode_data(k, m, oracle.fill(seed, b, MiB), mat)
        assert np.array_equal(st[b * E: (b + 1) * E].reshape(R, S), want)
        assert np.array_equal(sums[b], oracle.hh256_rows(KEY, want))
    return st, sums, S, St


def rows(st, b, E, Sb, R):
    return st[b * E: b * E + R * Sb].reshape(R, Sb)


@pytest.mark.parametrize("heal", [False, True], ids=["get", "heal"])
@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
@pytest.mark.parametrize("tail", [0, 123457])
def test_stream_decode_rs124(oracle, heal, pinned, tail):
    k, m, nfull = 12, 4, 200
    R = k + m
    ref, sums, S, St = make_object(oracle, k, m, nfull, tail, seed=4242)
    E = R * S
    nb = nfull + (1 if tail else 0)
    total = nfull * MiB + tail
    present = np.ones((nb, R), bool)
    present[:, [1, 12]] = False                  # a data and a parity disk offline
    present[50:100, 5] = False                   # a reader drops out mid-object
    present[150, [0, 2]] = False                 # one block at the limit (4 lost)
    rot_b, rot_row = 137, 3                      # a rotted chunk on a survivor
    work_h = z.HostBuffer(nb * E) if pinned else None
    work = work_h.array if pinned else np.empty(nb * E, np.uint8)
    work[:] = ref
    for b in range(nb):
        Sb = S if b < nfull else St
        r = rows(work, b, E, Sb, R)
        r[~present[b]] = 0x5A
    rows(work, rot_b, E, S, R)[rot_row, 777] ^= 0x10
    bad = np.full((nb, R), 9, np.int32)
    status = np.full(nb, 77, np.int32)
    out = np.zeros((nb, R, 32), np.uint8) if heal else None
    try:
        n = z.Codec(k, m, MiB).stream_decode(work_h if pinned else work, total, present, not heal, expect=sums, bad=bad,
                                             sums_out=out, status=status, batch_blocks=64)
        assert n == nb, n
        assert (status == 0).all()
        want_bad = np.zeros((nb, R), np.int32)
        want_bad[rot_b, rot_row] = 1
        assert np.array_equal(bad, want_bad), np.argwhere(bad != want_bad)[:5]
        for b in range(nb):
            if b == rot_b:
                continue  # its rebuilt rows are invalid (the shim re-reads it with shard 3 dropped)
            Sb = S if b < nfull else St
            got, exp = rows(work, b, E, Sb, R), rows(ref, b, E, Sb, R)
            for j in range(R):
                if present[b, j] or j < k or heal:
                    assert np.array_equal(got[j], exp[j]), (b, j)
                else:
                    assert (got[j] == 0x5A).all(), "DecodeDataBlocks leaves missing parity alone"
            if heal:
                for j in np.nonzero(~present[b])[0]:
                    assert np.array_equal(out[b, j], sums[b, j]), (b, j)
    finally:
        if work_h is not None:
            work_h.free()


def test_stream_decode_too_few_shards_reports_the_block(oracle):
    """A block with more than m shards missing returns ErrTooFewShards (its status), the
    other blocks are still served."""
    k, m, nfull = 8, 4, 20
    R = k + m
    ref, sums, S, _ = make_object(oracle, k, m, nfull, 0, seed=99)
    E = R * S
    present = np.ones((nfull, R), bool)
    present[:, 2] = False
    present[7, [0, 1, 3, 4, 5]] = False
    work = ref.copy()
    status = np.full(nfull, 77, np.int32)
    rc = z.Codec(k, m, MiB).stream_decode(work, nfull * MiB, present, True, expect=sums, status=status,
                                          batch_blocks=8)
    assert rc == -3
    assert status[7] == -3 and (np.delete(status, 7) == 0).all()
    for b in range(nfull):
        if b != 7:
            assert np.array_equal(rows(work, b, E, S, R)[:k], rows(ref, b, E, S, R)[:k]), b


def _rs164_case(oracle, heal, pinned, nfull, tail, bands, batch_blocks, want_quad):
    """RS(16+4) streamed GET / heal over per-block patterns `bands` = [(first, last, lost
    rows)], a rotted survivor chunk in block 23, every byte vs cpu_ref; want_quad: the
    survivor-quad kernel (vr_quad.hpp) must have served a batch (zs3_path_mask)."""
    k, m = 16, 4
    R = k + m
    ref, sums, S, St = make_object(oracle, k, m, nfull, tail, seed=1604)
    E = R * S
    nb = nfull + (1 if tail else 0)
    present = np.ones((nb, R), bool)
    for lo, hi, lost in bands:
        present[lo:hi, lost] = False
    rot_b, rot_row = 23, 11
    assert present[rot_b, rot_row]
    work_h = z.HostBuffer(nb * E) if pinned else None
    work = work_h.array if pinned else np.empty(nb * E, np.uint8)
    try:
        work[:] = ref
        for b in range(nb):
            Sb = S if b < nfull else St
            rows(work, b, E, Sb, R)[~present[b]] = 0x5A
        rows(work, rot_b, E, S, R)[rot_row, 4097] ^= 0x02
        bad = np.full((nb, R), 9, np.int32)
        status = np.full(nb, 77, np.int32)
        out = np.zeros((nb, R, 32), np.uint8) if heal else None
        z.path_mask(reset=True)
        n = z.Codec(k, m, MiB).stream_decode(work_h if pinned else work, nfull * MiB + tail, present, not heal,
                                             expect=sums, bad=bad, sums_out=out, status=status,
                                             batch_blocks=batch_blocks)
        mask = z.path_mask()
        assert n == nb and (status == 0).all()
        if want_quad:
            assert mask & z.KERNEL_VR_QUAD, f"four rebuilt rows ran on the survivor-quad kernel (mask {mask:#x})"
        want_bad = np.zeros((nb, R), np.int32)
        want_bad[rot_b, rot_row] = 1
        assert np.array_equal(bad, want_bad), np.argwhere(bad != want_bad)[:5]
        for b in range(nb):
            if b == rot_b:
                continue
            Sb = S if b < nfull else St
            got, exp = rows(work, b, E, Sb, R), rows(ref, b, E, Sb, R)
            for j in range(R):
                if present[b, j] or j < k or heal:
                    assert np.array_equal(got[j], exp[j]), (b, j)
                else:
                    assert (got[j] == 0x5A).all(), ("DecodeDataBlocks leaves missing parity alone", b, j)
            if heal:
                for j in np.nonzero(~present[b])[0]:
                    assert np.array_equal(out[b, j], sums[b, j]), (b, j)
    finally:
        if work_h is not None:
            work_h.free()


@pytest.mark.parametrize("heal", [False, True], ids=["get", "heal"])
@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
def test_stream_decode_rs164_four_lost(oracle, heal, pinned):
    """RS(16+4) with four shards to rebuild on most blocks, in one batch large enough for
    the survivor-quad kernel (vr_quad.hpp; pattern groups of up to 1 024 blocks take the
    small-batch latency path, kernels.hip small_get): blocks 0-1049 lose four DATA rows in
    GET (GET rebuilds data rows only, so that is what reaches k_vr_quad) and two data + two
    parity rows in heal, as one run of blocks (a group with a block-id list takes
    k_vr_ws); blocks 1050-1059 swap a reader (another four-row pattern); GET blocks
    1060-1064 lose three data rows and parity row 17, which must stay untouched; the short
    last block takes the k_vr_ws instances (its shard size is not a multiple of 256).
    RS(16+4) rows of 1 MiB blocks are 256-byte aligned, so pinned stripes take the per-row
    DMA path (only rows some block of the batch has go up), pageable ones the
    staging."""
    if heal:
        bands = [(0, 1050, [0, 7, 16, 19]), (1050, 1060, [0, 9, 16, 19]), (1060, 1066, [2, 16])]
    else:
        bands = [(0, 1050, [0, 7, 9, 12]), (1050, 1060, [0, 3, 9, 12]), (1060, 1065, [0, 7, 9, 17]),
                 (1065, 1066, [1, 4])]
    _rs164_case(oracle, heal, pinned, 1065, 70001, bands, batch_blocks=1066, want_quad=True)


@pytest.mark.parametrize("heal", [False, True], ids=["get", "heal"])
def test_stream_decode_rs164_small_batches(oracle, heal):
    """The same per-block patterns through 16-block batches: every pattern group is small
    and takes the latency path (reconstruct + one-chain-per-quad hash), groups launch on
    shifted batches and on block-id lists."""
    if heal:
        bands = [(0, 10, [0, 7, 16, 19]), (10, 20, [0, 9, 16, 19]), (20, 41, [0, 7, 16, 19])]
    else:
        bands = [(0, 25, [0, 7, 9, 12]), (25, 30, [0, 7, 9, 17]), (30, 41, [0, 7, 9, 12])]
    _rs164_case(oracle, heal, False, 40, 70001, bands, batch_blocks=16, want_quad=False)


@pytest.mark.parametrize("heal", [False, True], ids=["get", "heal"])
def test_stream_decode_rs84_pinned_rows_and_failed_block(oracle, heal):
    """RS(8+4) 1 MiB blocks from pinned stripes: S = 131 072 is 256-byte aligned, so rows
    move by per-row DMA across each batch, and only rows that some block of the batch has
    are uploaded.  Rows are present in some blocks and missing in others within one batch;
    one block has too few shards: it reports ErrTooFewShards, the others are served, and
    nothing comes back into the failed block's stripe (its rows that were never uploaded
    would otherwise carry whatever the pooled device slot last held)."""
    k, m, nfull = 8, 4, 48
    R = k + m
    ref, sums, S, _ = make_object(oracle, k, m, nfull, 0, seed=8484)
    E = R * S
    present = np.ones((nfull, R), bool)
    present[0:12, 2] = False                     # row 2 lost in the first 12 blocks only
    present[5:30, 9] = False                     # parity row 9 lost in blocks 5-29
    present[20:48:3, 6] = False                  # row 6 lost in every third block
    present[33, [0, 1, 3, 4, 5]] = False         # block 33: five lost, too few shards
    work_h = z.HostBuffer(nfull * E)
    try:
        work = work_h.array
        work[:] = ref
        for b in range(nfull):
            rows(work, b, E, S, R)[~present[b]] = 0x5A
        before33 = rows(work, 33, E, S, R).copy()
        bad = np.full((nfull, R), 9, np.int32)
        status = np.full(nfull, 77, np.int32)
        out = np.zeros((nfull, R, 32), np.uint8) if heal else None
        rc = z.Codec(k, m, MiB).stream_decode(work_h, nfull * MiB, present, not heal, expect=sums, bad=bad,
                                              sums_out=out, status=status, batch_blocks=16)
        assert rc == -3, rc
        assert status[33] == -3 and (np.delete(status, 33) == 0).all(), status
        assert not bad.any()
        assert np.array_equal(rows(work, 33, E, S, R), before33), "a failed block's stripe is left as it was"
        for b in range(nfull):
            if b == 33:
                continue
            got, exp = rows(work, b, E, S, R), rows(ref, b, E, S, R)
            for j in range(R):
                if present[b, j] or j < k or heal:
                    assert np.array_equal(got[j], exp[j]), (b, j)
                else:
                    assert (got[j] == 0x5A).all(), (b, j)
            if heal:
                for j in np.nonzero(~present[b])[0]:
                    assert np.array_equal(out[b, j], sums[b, j]), (b, j)
        if heal:
            assert not out[33].any(), "no sums for a block that was not healed"
    finally:
        work_h.free()


def test_stream_decode_argument_checks():
    """The Python binding checks every buffer's size, dtype and layout before the library
    touches it through raw pointers: nothing reaches the device."""
    k, m = 8, 4
    c = z.Codec(k, m, MiB)
    R, S = k + m, MiB // k
    st = np.zeros(2 * R * S, np.uint8)
    pres = np.ones((2, R), bool)
    with pytest.raises(ValueError):
        c.stream_decode(st[:-1], 2 * MiB, pres, True)             # stripes too short
    with pytest.raises(ValueError):
        c.stream_decode(st, 2 * MiB, pres[:1], True)              # present for one block
    with pytest.raises(ValueError):
        c.stream_decode(st, 2 * MiB, pres, True, bad=np.zeros((2, R), np.int64))
    with pytest.raises(ValueError):
        c.stream_decode(st, 2 * MiB, pres, True, expect=np.zeros((2, R, 31), np.uint8))
    with pytest.raises(ValueError):
        c.stream_decode(st, 2 * MiB, pres, True, status=np.zeros(4, np.int32)[::2])
    with pytest.raises(ValueError):
        c.stream_decode(st.reshape(2, -1)[:, ::2], 2 * MiB, pres, True)


def test_stream_encode_argument_checks():
    """The encode stream wrappers check their host buffers' sizes the same way: a source
    shorter than total_len, or parity / sums arrays shorter than the object's blocks need,
    are refused before the library reads or writes them."""
    k, m = 8, 4
    c = z.Codec(k, m, MiB)
    S = MiB // k
    src = np.zeros(2 * MiB, np.uint8)
    par = np.zeros(2 * m * S, np.uint8)
    sums = np.zeros(2 * (k + m) * 32, np.uint8)
    for call in (lambda *a: c.stream_encode(*a), lambda *a: c.stream_encode_multi([0], *a)):
        with pytest.raises(ValueError):
            call(src[:-1], 2 * MiB, par, sums)          # source shorter than the stream
        with pytest.raises(ValueError):
            call(src, 2 * MiB, par[:-1], sums)          # parity for fewer blocks
        with pytest.raises(ValueError):
            call(src, 2 * MiB, par, sums[:-32])         # sums for fewer shards
        with pytest.raises(ValueError):
            call(src.reshape(2, -1)[:, ::2], MiB // 2, par, sums)  # strided source
    assert c.stream_encode(src, 2 * MiB, par, sums) == 2


@pytest.mark.parametrize("pinned", [False, True], ids=["pageable", "pinned"])
def test_stream_decode_many_rebuilt_rows(oracle, pinned):
    """RS(30+6) on 1 MiB blocks (S = 34 953, rows not 256-byte aligned): the rebuilt rows go
    back by k_rows_copy while a batch's union of lost rows fits its 32-row list (blocks 0-7
    lose rows 0-5) and as whole stripes when it does not (blocks 8-23 each lose 6 rows of a
    rotating set: 36 distinct rows per batch).  Heal: every lost row rebuilt and hashed."""
    k, m, nfull = 30, 6, 24
    R = k + m
    ref, sums, S, _ = make_object(oracle, k, m, nfull, 0, seed=3006)
    E = R * S
    present = np.ones((nfull, R), bool)
    present[:8, 0:6] = False
    for b in range(8, nfull):
        present[b, [(b * 6 + i) % R for i in range(6)]] = False
    work_h = z.HostBuffer(nfull * E) if pinned else None
    work = work_h.array if pinned else np.empty(nfull * E, np.uint8)
    work[:] = ref
    for b in range(nfull):
        rows(work, b, E, S, R)[~present[b]] = 0x5A
    out = np.zeros((nfull, R, 32), np.uint8)
    bad = np.full((nfull, R), 9, np.int32)
    try:
        n = z.Codec(k, m, MiB).stream_decode(work_h if pinned else work, nfull * MiB, present, False, expect=sums,
                                             bad=bad, sums_out=out, batch_blocks=8)
        assert n == nfull
        assert not bad.any()
        assert np.array_equal(work, ref)
        for b in range(nfull):
            for j in np.nonzero(~present[b])[0]:
                assert np.array_equal(out[b, j], sums[b, j]), (b, j)
    finally:
        if work_h is not None:
            work_h.free()
