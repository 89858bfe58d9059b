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


@pytest.mark.parametrize("heal", [False, True], ids=["get", "heal"])
def test_stream_decode_rs164_four_lost(oracle, heal):
    """RS(16+4) with four shards lost on every block (the survivor-quad kernel's case,
    vr_quad.hpp) through the streamed path: pattern groups launch on shifted batches,
    a rotted survivor chunk is flagged at its (block, shard), a short last block takes
    the k_vr_ws instances (its shard size is not a multiple of 256)."""
    k, m, nfull, tail = 16, 4, 40, 70001
    R = k + m
    ref, sums, S, St = make_object(oracle, k, m, nfull, tail, seed=1604)
    E = R * S
    nb = nfull + 1
    present = np.ones((nb, R), bool)
    present[:, [0, 7, 16, 19]] = False
    present[10:20, 7] = True                     # a reader back for ten blocks (3 lost there)
    present[10:20, 9] = False                    # ... while another drops out (4 lost again)
    rot_b, rot_row = 23, 11
    work = ref.copy()
    for b in range(nb):
        Sb = S if b < nfull else St
        r = rows(work, b, E, Sb, R)
        r[~present[b]] = 0x5A
    rows(work, rot_b, E, S, R)[rot_row, 4097] ^= 0x02
    bad = np.full((nb, R), 9, np.int32)
    status = np.full(nb, 77, np.int32)
    out = np.zeros((nb, R, 32), np.uint8) if heal else None
    n = z.Codec(k, m, MiB).stream_decode(work, nfull * MiB + tail, present, not heal, expect=sums, bad=bad,
                                         sums_out=out, status=status, batch_blocks=16)
    assert n == nb and (status == 0).all()
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
        if heal:
            for j in np.nonzero(~present[b])[0]:
                assert np.array_equal(out[b, j], sums[b, j]), (b, j)
