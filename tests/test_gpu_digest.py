"""GPU parity of the object digests: zs3_md5_batch (S3 ETag,
internal/etag/reader.go:106-144), zs3_sha256_batch (content SHA-256,
internal/hash/reader.go:123-153) and zs3_etag_multipart (internal/etag/etag.go:211-226)
against the oracle (hashlib, pinned by the reference's etag_test.go vectors) — every
padding branch (length mod 64 = 0..63, the 55/56 boundary), multi-block messages,
per-message lengths, 1 MiB objects."""
import hashlib
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import zs3server_amd as z  # noqa: E402
from oracle import etag_oracle as eo  # noqa: E402
from zs3server_amd import etag as ze  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
VEC = json.load(open(os.path.join(HERE, "golden", "etag_vectors.json")))


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    z.lib()


def run(fn, host, stride, lens, width):
    n = len(lens)
    d = torch.from_numpy(host).cuda()
    dl = torch.tensor(lens, dtype=torch.int64, device="cuda")
    out = torch.zeros(n * width, dtype=torch.uint8, device="cuda")
    fn(d, stride, 0, n, out, lens=dl)
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(n, width)


@pytest.mark.parametrize("algo", ["md5", "sha256"])
def test_all_lengths_0_to_300(algo):
    rng = np.random.default_rng(5)
    lens = list(range(301))
    stride = 320
    host = rng.integers(0, 256, len(lens) * stride, dtype=np.uint8)
    fn, width, ref = (z.md5_batch, 16, hashlib.md5) if algo == "md5" else (z.sha256_batch, 32, hashlib.sha256)
    got = run(fn, host, stride, lens, width)
    for i, n in enumerate(lens):
        assert got[i].tobytes() == ref(host[i * stride: i * stride + n].tobytes()).digest(), n


@pytest.mark.parametrize("algo", ["md5", "sha256"])
def test_one_mib_objects_fixed_length(algo):
    n, blen = 8, (1 << 20) + 13
    stride = blen + 3  # unaligned message starts
    host = np.concatenate([np.frombuffer(os.urandom(stride), dtype=np.uint8) for _ in range(n)])
    d = torch.from_numpy(host).cuda()
    width = 16 if algo == "md5" else 32
    out = torch.zeros(n * width, dtype=torch.uint8, device="cuda")
    (z.md5_batch if algo == "md5" else z.sha256_batch)(d, stride, blen, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(n, width)
    ref = eo.md5 if algo == "md5" else eo.sha256
    for i in range(n):
        assert got[i].tobytes() == ref(host[i * stride: i * stride + blen].tobytes())


def test_reference_reader_vectors_on_device():
    tags = ze.object_etags([r["content"].encode() for r in VEC["reader"]])
    assert [t.hex() for t in tags] == [r["etag"] for r in VEC["reader"]]


def test_reference_multipart_vectors_on_device():
    for t in VEC["multipart"]:
        parts = [bytes(ze.Parse(e)) for e in t["etags"]]
        want = bytes(ze.Parse(t["multipart"])) if t["multipart"] else b""
        assert bytes(ze.Multipart(*parts)) == want


def test_content_sha256_mirror():
    objs = [b"", b"abc", os.urandom(1000), os.urandom(65536 + 7)]
    assert ze.content_sha256(objs) == [eo.sha256(o) for o in objs]


@pytest.mark.parametrize("algo", ["md5", "sha256"])
def test_parts_at_offsets_one_launch(algo):
    """Independent messages of very different lengths at arbitrary (unaligned,
    overlapping) offsets of one buffer in one launch (zs3_md5_parts / zs3_sha256_parts:
    the parts of multipart uploads), including empty, 55/56/64-byte boundaries and
    multi-MiB parts next to 1-byte ones in the same wave."""
    rng = np.random.default_rng(11)
    total = 9 << 20
    host = rng.integers(0, 256, total, dtype=np.uint8)
    lens = [0, 1, 55, 56, 63, 64, 65, 119, 120, 4096, (5 << 20) + 3, 3 << 20, 777777, 1 << 20] + \
        [int(x) for x in rng.integers(0, 300000, 150)]
    offs = [int(rng.integers(0, total - n + 1)) for n in lens]
    d = torch.from_numpy(host).cuda()
    do = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dl = torch.tensor(lens, dtype=torch.int64, device="cuda")
    width = 16 if algo == "md5" else 32
    out = torch.zeros(len(lens) * width, dtype=torch.uint8, device="cuda")
    (z.md5_parts if algo == "md5" else z.sha256_parts)(d, do, dl, len(lens), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(len(lens), width)
    ref = hashlib.md5 if algo == "md5" else hashlib.sha256
    for i, (o, n) in enumerate(zip(offs, lens)):
        assert got[i].tobytes() == ref(host[o:o + n].tobytes()).digest(), (i, n)
