"""CPU restatement of the reference's object digests (TEST INFRASTRUCTURE ONLY: used
by tests/ as the checker, never by the product path).

- ETag of an object = crypto/md5 of its bytes (internal/etag/reader.go:106-144).
- etag.Multipart (internal/etag/etag.go:211-226): MD5 over the concatenated singlepart
  ETags (multipart "-N" and encrypted ETags skipped, etag.go:145-155) || "-" || count;
  nil for an empty list.
- Content SHA-256 (internal/hash/reader.go:123-153; sha256-simd = FIPS 180-4).
MD5 and SHA-256 are Python's hashlib (RFC 1321 / FIPS 180-4, the algorithms Go's
crypto/md5 and minio/sha256-simd implement).  Pinned by the reference's own vectors in
internal/etag/etag_test.go (readerTests :120-133, multipartTests :147-178), committed as
tests/golden/etag_vectors.json.
"""
import hashlib


def md5(data: bytes) -> bytes:
    return hashlib.md5(data).digest()


def sha256(data: bytes) -> bytes:
    return hashlib.sha256(data).digest()


def is_multipart(e: bytes) -> bool:
    return len(e) > 16 and b"-" in e


def is_encrypted(e: bytes) -> bool:
    return len(e) > 16 and b"-" not in e


def multipart(etags) -> bytes:
    if len(etags) == 0:
        return b""
    h = hashlib.md5()
    n = 0
    for e in etags:
        if not is_multipart(e) and not is_encrypted(e):
            h.update(e)
            n += 1
    return h.digest() + b"-" + str(n).encode()
