"""GPU parity of every compiled fused-kernel variant (kernels.hip / fused_v2.hip),
forced with set_variant, against the CPU oracle: parity shards and HighwayHash-256
sums bit-exact.  Shard sizes hit every tile-loop edge of fused_v2 (no full tile, exactly
one tile, whole tiles only, ragged tails of 16/32/128 B) and batch sizes that leave
dead stripes in the last workgroup (16-stripe workgroups at n = 1, 17, 33).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402
from conftest import variant_ctx  # noqa: E402

KEY = z.MAGIC_HH256_KEY
DEV = "cuda:0"

# RS(8+4) fused_v2 tile = 384 B per shard row
SIZES_84 = [8 * 16, 8 * 384, 8 * 384 * 3, 8 * (384 * 2 + 32), 8 * (384 * 5 + 16), 1 << 20,
            8 * 1024 * 2, 8 * (1024 * 2 + 48), 8 * (1024 * 3 + 512)]
VARIANTS = [0, 49, 99, 313, 410, 411, 412, 413, 414]


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()
    yield


def run_case(oracle, k, m, blen, nb, variant, seed):
    with variant_ctx(variant):
        _run_case(oracle, k, m, blen, nb, variant, seed)


def _run_case(oracle, k, m, blen, nb, variant, seed):
    codec = z.Codec(k, m, 1 << 20)
    S = -(-blen // k)
    stride = (k + m) * S
    host = np.zeros(nb * stride, dtype=np.uint8)
    for b in range(nb):
        host[b * stride: b * stride + blen] = oracle.fill(seed, b, blen)
    d = torch.from_numpy(host).to(DEV)
    sums = torch.zeros(nb * (k + m) * 32, dtype=torch.uint8, device=DEV)
    codec.encode_batch(d, stride, blen, nb, parity=d, parity_offset=k * S, parity_stride=stride, sums=sums)
    torch.cuda.synchronize()
    out = d.cpu().numpy().reshape(nb, k + m, S)
    hs = sums.cpu().numpy().reshape(nb, k + m, 32)
    mat = oracle.build_matrix(k, m)
    for b in range(nb):
        want = oracle.encode_data(k, m, host[b * stride: b * stride + blen], mat)
        assert np.array_equal(out[b, k:], want[k:]), f"variant {variant}: parity block {b}"
        assert np.array_equal(hs[b], oracle.hh256_rows(KEY, want)), f"variant {variant}: sums block {b}"


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("blen", SIZES_84)
def test_rs84_variant_tile_edges(oracle, variant, blen):
    nb = 3 if blen == 1 << 20 else 5
    run_case(oracle, 8, 4, blen, nb, variant, seed=blen % 251)


@pytest.mark.parametrize("variant", [49, 99, 313, 410, 412, 414])
@pytest.mark.parametrize("nb", [1, 17, 33])
def test_rs84_variant_dead_stripes(oracle, variant, nb):
    run_case(oracle, 8, 4, 8 * (384 * 4 + 128), nb, variant, seed=nb)


@pytest.mark.parametrize("variant", [0, 49, 99, 400, 401, 402, 403, 415])
@pytest.mark.parametrize("k,m,blen", [(4, 2, 4 * 16), (4, 2, 4 * (384 * 3 + 48)), (4, 2, 1 << 20),
                                      (16, 4, 16 * 640 * 2), (16, 4, 1 << 20), (4, 4, 4 * (384 * 3 + 48)),
                                      (4, 4, 1 << 20)])
def test_other_shapes_variants(oracle, variant, k, m, blen):
    run_case(oracle, k, m, blen, 3, variant, seed=k + m)


# RS(12+4) on blocks whose shard rows are not 16-byte aligned (1 MiB: S = 87 382) runs
# k_ehx_ws in UA mode; diagnostics 416 = the product shape with the region-interleaved
# workgroup order (fused_v2_diag.hip)
@pytest.mark.parametrize("variant", [0, 416])
@pytest.mark.parametrize("blen,nb", [(1 << 20, 3), (1 << 20, 9), (12 * (512 * 3 + 100) - 6, 17)])
def test_rs124_ua_variants(oracle, variant, blen, nb):
    with variant_ctx(variant):
        _run_case(oracle, 12, 4, blen, nb, variant, seed=nb)
        assert z.last_path() == 2, z.last_path()  # the warp-specialised kernel, not a fallback


def test_variants_are_per_thread(oracle):
    """The diagnostics build's variant selection is thread-local (no process-wide tuning
    state): two threads encode concurrently with different variants — and a third on
    the product library — and every result matches the oracle."""
    import threading

    k, m, blen, nb = 8, 4, 8 * (384 * 5 + 16), 17
    S = -(-blen // k)
    R = k + m
    host = np.zeros(nb * R * S, dtype=np.uint8)
    for b in range(nb):
        host[b * R * S: b * R * S + blen] = oracle.fill(71, b, blen)
    mat = oracle.build_matrix(k, m)
    want = [oracle.encode_data(k, m, host[b * R * S: b * R * S + blen], mat) for b in range(nb)]
    want_sums = [oracle.hh256_rows(KEY, w) for w in want]
    errs = []

    def worker(variant, reps):
        try:
            with variant_ctx(variant):
                codec = z.Codec(k, m, 1 << 20)
                stream = torch.cuda.Stream()
                for _ in range(reps):
                    with torch.cuda.stream(stream):
                        d = torch.from_numpy(host).to(DEV)
                        sums = torch.zeros(nb * R * 32, dtype=torch.uint8, device=DEV)
                        codec.encode_batch(d, R * S, blen, nb, parity=d, parity_offset=k * S, parity_stride=R * S,
                                           sums=sums)
                    stream.synchronize()
                    out = d.cpu().numpy().reshape(nb, R, S)
                    hs = sums.cpu().numpy().reshape(nb, R, 32)
                    for b in range(nb):
                        assert np.array_equal(out[b], want[b]), (variant, b)
                        assert np.array_equal(hs[b], want_sums[b]), (variant, b)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(v, 20)) for v in (49, 412, 0)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
