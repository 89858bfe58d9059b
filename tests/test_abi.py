"""CPU-only checks of the C-ABI library: it loads, exports every symbol
include/zs3gpu.h declares, and the host-only entry points (NewErasure checks,
size arithmetic, coding matrix) match the reference.  No compute calls."""
import os
import re
import subprocess

import numpy as np
import pytest

import zs3server_amd as z

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "zs3gpu.h")


DIAG_HEADER = os.path.join(ROOT, "include", "zs3gpu_diag.h")


def header_functions(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zs3_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module", autouse=True)
def built():
    import __graft_entry__ as g
    g.build_lib()
    z.lib()


def test_header_matches_python_export_list():
    assert header_functions() == sorted(z.EXPORTS)


def _exports(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path]).decode()
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_library_exports_every_header_symbol():
    syms = _exports(z.LIB_PATH)
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing


def test_product_library_has_no_diagnostics():
    """The experimental variants and the zs3_debug_* calls live only in the
    diagnostics build; the product library exports exactly include/zs3gpu.h."""
    assert header_functions(DIAG_HEADER) == sorted(z.DIAG_EXPORTS)
    zs3 = {s for s in _exports(z.LIB_PATH) if s.startswith("zs3_")}
    assert zs3 == set(header_functions())
    dsyms = _exports(z.DIAG_LIB_PATH)
    assert set(header_functions()) | set(z.DIAG_EXPORTS) <= dsyms


def test_version_and_strerror():
    L = z.lib()
    assert L.zs3_version() == (0 << 16) | (1 << 8)
    assert L.zs3_strerror(-3) == b"too few shards given"
    assert L.zs3_strerror(-7) == b"file is corrupted"


@pytest.mark.parametrize("k,m,code", [(0, 2, -1), (2, 0, -1), (-1, 4, -1), (200, 57, -2), (255, 2, -2)])
def test_new_erasure_errors(k, m, code):
    # cmd/erasure-coding.go:44-50
    with pytest.raises(z.ZS3Error) as ei:
        z.Codec(k, m, 1 << 20)
    assert ei.value.code == code


def test_new_erasure_max_shards_ok():
    c = z.Codec(128, 128, 1 << 20)  # k+m == 256 is allowed
    assert c.shard_size() == 8192


def test_codec_matrix_matches_oracle(oracle):
    for k, m in [(4, 2), (8, 4), (16, 4), (5, 3), (12, 4), (1, 1), (20, 12)]:
        assert np.array_equal(z.Codec(k, m).matrix(), oracle.build_matrix(k, m))


def ceil_frac(a, b):
    # cmd/utils.go:691
    if b == 0:
        return 0
    c = a // b if a >= 0 else -((-a) // b)
    if a > 0 and a % b:
        c = a // b + 1
    return c


@pytest.mark.parametrize("k,m,bs", [(4, 2, 1 << 20), (8, 4, 1 << 20), (16, 4, 1 << 20), (5, 3, 1 << 20),
                                    (6, 2, 10 << 20), (12, 4, 1 << 20)])
def test_shard_size_arithmetic(k, m, bs):
    # Erasure.ShardSize / ShardFileSize / ShardFileOffset, cmd/erasure-coding.go:122-150
    c = z.Codec(k, m, bs)
    ss = ceil_frac(bs, k)
    assert c.shard_size() == ss
    assert c.shard_file_size(0) == 0
    assert c.shard_file_size(-1) == -1
    rng = np.random.default_rng(k * 100 + m)
    for total in [1, 17, bs - 1, bs, bs + 1, 3 * bs + 5, 64 * bs] + list(rng.integers(1, 10 * bs, 20)):
        total = int(total)
        want = (total // bs) * ss + ceil_frac(total % bs, k)
        assert c.shard_file_size(total) == want
        for start, length in [(0, total), (total // 3, total - total // 3), (0, 0), (total - 1, 1)]:
            till = ((start + length) // bs) * ss + ss
            assert c.shard_file_offset(start, length, total) == min(till, want)


def test_bitrot_shard_file_size():
    # cmd/bitrot.go:150-155 (HighwayHash256S: 32-byte sum per shard chunk)
    assert z.bitrot_shard_file_size(35, 10) == 4 * 32 + 35
    assert z.bitrot_shard_file_size(131072, 131072) == 131072 + 32
    assert z.bitrot_shard_file_size(0, 10) == 0
    assert z.bitrot_shard_file_size(4 * 131072 + 1, 131072) == 5 * 32 + 4 * 131072 + 1


# Batch layout validation: every case is rejected before any device
# call, so the fake device addresses below are never dereferenced.
BASE = 1 << 40


def _codec_handle(k, m):
    c = z.Codec(k, m, 1 << 20)
    return c, c._h


@pytest.mark.parametrize("case", ["neg_stride", "data_overlap", "parity_overlap", "parity_on_data",
                                  "parity_on_next_block", "parity_span_on_data"])
def test_encode_batch_rejects_bad_layouts(case):
    import ctypes as C
    k, m = 8, 4
    c, h = _codec_handle(k, m)
    L = z.lib()
    S = (1 << 20) // k
    B, R = 1 << 20, k + m
    args = {
        # (data, data_stride, n, parity, parity_stride)
        "neg_stride": (BASE, -R * S, 4, BASE + k * S, -R * S),
        "data_overlap": (BASE, B - 16, 4, BASE + 64 * R * S, m * S),
        "parity_overlap": (BASE, R * S, 4, BASE + 64 * R * S, m * S - 1),
        "parity_on_data": (BASE, R * S, 4, BASE + k * S - 16, R * S),  # parity row 0 on data row 7
        "parity_on_next_block": (BASE, R * S - 16, 1 + 3, BASE + k * S, R * S - 16),
        "parity_span_on_data": (BASE, R * S, 4, BASE + 2 * R * S, m * S),  # separate span inside the data
    }[case]
    d, ds, n, p, ps = args
    rc = L.zs3_encode_batch(h, C.c_void_p(d), ds, B, n, C.c_void_p(p), ps, None, None)
    assert rc == -8, (case, rc)


@pytest.mark.parametrize("k,m", [(2, 2), (3, 3), (4, 4), (8, 4), (8, 8), (12, 4)])
def test_encode_batch_layouts_accepted(k, m):
    """separate data / parity regions are accepted whatever the strides.
    The queue's encode slots put [n][k*S] data then [n][m*S] parity, so for k == m (RS(2+2),
    RS(3+3), RS(4+4): the 4-, 6- and 8-drive defaults) both strides are equal; the layout
    check runs on the host only (zs3_debug_encode_layout_ok, no device call)."""
    import ctypes as C
    L = z.diag_lib()
    B = 1 << 20
    S = -(-B // k)
    KS, MS = k * S, m * S
    ok = lambda d, ds, n, p, ps: L.zs3_debug_encode_layout_ok(C.c_void_p(d), ds, B, n, C.c_void_p(p), ps, MS)
    for n in (1, 2, 5, 256):
        cap = n
        # the queue slot: data region then parity region right after it
        assert ok(BASE, KS, n, BASE + cap * KS, MS) == 1, (k, m, n, "queue slot")
        # separately allocated regions with equal strides, either order, any address gap
        assert ok(BASE, KS, n, BASE + (1 << 34) + 17, KS) == 1, (k, m, n, "separate, equal strides")
        assert ok(BASE + (1 << 34), KS, n, BASE, KS) == 1, (k, m, n, "parity below data")
        # the reference's in-place Split layout
        assert ok(BASE, (k + m) * S, n, BASE + KS, (k + m) * S) == 1, (k, m, n, "in place")
    # equal strides whose spans interleave without landing in each block's gap: rejected
    assert ok(BASE, KS + MS, 4, BASE + KS - 16, KS + MS) == 0
    # separate spans that overlap with different strides: rejected
    assert ok(BASE, KS, 4, BASE + 2 * KS, MS) == 0


@pytest.mark.parametrize("fn", ["reconstruct", "verify", "reconstruct_masks", "verify_masks"])
@pytest.mark.parametrize("stride_delta", [-1, -(1 << 30)])
def test_stripe_batches_reject_short_strides(fn, stride_delta):
    import ctypes as C
    k, m = 8, 4
    R = k + m
    c, h = _codec_handle(k, m)
    L = z.lib()
    S = (1 << 20) // k
    n = 4
    stride = R * S + stride_delta
    pres = (C.c_uint8 * R)(*([0, 0] + [1] * (R - 2)))
    presn = (C.c_uint8 * (R * n))(*(([0, 0] + [1] * (R - 2)) * n))
    fake = C.c_void_p(BASE)
    if fn == "reconstruct":
        rc = L.zs3_reconstruct_batch(h, fake, stride, S, n, pres, 1, None)
    elif fn == "verify":
        rc = L.zs3_verify_reconstruct_batch(h, fake, stride, S, n, pres, 1, fake, fake, None, None)
    elif fn == "reconstruct_masks":
        rc = L.zs3_reconstruct_batch_masks(h, fake, stride, S, n, presn, 1, None, None)
    else:
        rc = L.zs3_verify_reconstruct_batch_masks(h, fake, stride, S, n, presn, 1, fake, fake, None, None, None)
    assert rc == -8, (fn, rc)


@pytest.mark.parametrize("fn", ["zs3_md5_parts", "zs3_sha256_parts"])
def test_parts_digests_reject_missing_arrays(fn):
    """zs3_md5_parts / zs3_sha256_parts need both the offsets and the lengths arrays
    (rejected before any device call); zero messages is a no-op."""
    import ctypes as C
    L = z.lib()
    fake = C.c_void_p(BASE)
    assert getattr(L, fn)(fake, None, fake, 3, fake, None) == -8
    assert getattr(L, fn)(fake, fake, None, 3, fake, None) == -8
    assert getattr(L, fn)(fake, fake, fake, -1, fake, None) == -8


def test_path_mask_and_pool_limit_are_host_only():
    """zs3_path_mask on a thread that launched nothing is empty; zs3_pool_limit with no
    idle staging frees nothing (neither call touches a GPU)."""
    import threading
    got = []
    t = threading.Thread(target=lambda: got.append(z.path_mask(reset=True)))
    t.start()
    t.join()
    assert got == [0]
    assert z.pool_limit(1 << 30) == 0
    assert z.pool_limit(6 << 30) == 0
