"""Mirror of the reference's S3 ETag helpers (internal/etag) over the zs3gpu C ABI.

Same names and semantics as internal/etag/etag.go and reader.go so the tests read like
etag_test.go: an ETag is raw bytes (16-byte MD5 for singlepart objects; MD5 || "-N"
for multipart; longer without '-' = encrypted).  The MD5 work runs on the device
(zs3_md5_batch / zs3_etag_multipart); only the byte-string bookkeeping is Python.
"""
from __future__ import annotations

import numpy as np

from . import etag_multipart, md5_batch, sha256_batch


class ETag(bytes):
    """internal/etag/etag.go:128-175."""

    def IsEncrypted(self) -> bool:  # etag.go:145-147
        return len(self) > 16 and b"-" not in self

    def IsMultipart(self) -> bool:  # etag.go:153-155
        return len(self) > 16 and b"-" in self

    def Parts(self) -> int:  # etag.go:163-174
        if not self.IsMultipart():
            return 1
        return int(self[self.index(b"-") + 1:])

    def String(self) -> str:  # etag.go:137-142
        if self.IsMultipart():
            return self[:16].hex() + self[16:].decode()
        return self.hex()


def Parse(s: str) -> ETag:
    """etag.Parse for the unquoted / quoted hex forms (etag.go:101-126)."""
    s = s.strip('"')
    if "-" in s:
        h, n = s.split("-", 1)
        return ETag(bytes.fromhex(h) + b"-" + n.encode())
    return ETag(bytes.fromhex(s))


def Multipart(*etags: bytes) -> ETag:
    """etag.Multipart (etag.go:211-226): MD5 over the singlepart ETags || "-N"."""
    return ETag(etag_multipart([bytes(e) for e in etags]))


def object_etags(objects: list[bytes]) -> list[ETag]:
    """etag.NewReader(...).ETag() of each object (reader.go:106-144), one device batch."""
    import torch
    n = len(objects)
    if n == 0:
        return []
    stride = max(1, max(len(o) for o in objects))
    host = np.zeros(n * stride, dtype=np.uint8)
    for i, o in enumerate(objects):
        host[i * stride: i * stride + len(o)] = np.frombuffer(o, dtype=np.uint8)
    d = torch.from_numpy(host).cuda()
    lens = torch.tensor([len(o) for o in objects], dtype=torch.int64, device="cuda")
    out = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    md5_batch(d, stride, 0, n, out, lens=lens)
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(n, 16)
    return [ETag(r.tobytes()) for r in o]


def content_sha256(objects: list[bytes]) -> list[bytes]:
    """hash.Reader's content SHA-256 (internal/hash/reader.go:123-153) of each object."""
    import torch
    n = len(objects)
    if n == 0:
        return []
    stride = max(1, max(len(o) for o in objects))
    host = np.zeros(n * stride, dtype=np.uint8)
    for i, o in enumerate(objects):
        host[i * stride: i * stride + len(o)] = np.frombuffer(o, dtype=np.uint8)
    d = torch.from_numpy(host).cuda()
    lens = torch.tensor([len(o) for o in objects], dtype=torch.int64, device="cuda")
    out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    sha256_batch(d, stride, 0, n, out, lens=lens)
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(n, 32)
    return [r.tobytes() for r in o]
