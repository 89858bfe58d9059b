"""The object-digest oracle (oracle/etag_oracle.py) against the reference's own vectors
(internal/etag/etag_test.go readerTests and multipartTests, tests/golden/etag_vectors.json),
and the ETag mirror's byte-string helpers (CPU only)."""
import json
import os

from oracle import etag_oracle as eo
from zs3server_amd import etag as ze

HERE = os.path.dirname(os.path.abspath(__file__))
VEC = json.load(open(os.path.join(HERE, "golden", "etag_vectors.json")))


def parse(s: str) -> bytes:
    return bytes(ze.Parse(s)) if s else b""


def test_reader_vectors():
    for r in VEC["reader"]:
        assert eo.md5(r["content"].encode()).hex() == r["etag"]


def test_multipart_vectors():
    for t in VEC["multipart"]:
        assert eo.multipart([parse(e) for e in t["etags"]]) == parse(t["multipart"])


def test_etag_helpers():
    mp = ze.Parse("ceb8853ddc5086cc4ab9e149f8f09c88-2")
    assert mp.IsMultipart() and not mp.IsEncrypted() and mp.Parts() == 2
    assert mp.String() == "ceb8853ddc5086cc4ab9e149f8f09c88-2"
    sp = ze.Parse('"3b83ef96387f14655fc854ddc3c6bd57"')
    assert not sp.IsMultipart() and sp.Parts() == 1 and sp.String() == "3b83ef96387f14655fc854ddc3c6bd57"
    enc = ze.ETag(bytes(48))
    assert enc.IsEncrypted() and not enc.IsMultipart()
