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


# ---- digest routing ------------------------------------------------
# One message's 64-byte blocks form a serial chain, so a device lane hashes one message at
# its chain roof (profiles/r04/bench_paths_enc_ua_digest.jsonl: one 5 MiB
# part MD5 0.555 us / SHA-256 1.696 us per 64-byte block), i.e. ~115 MB/s (MD5) and ~38 MB/s
# (SHA-256) per message, against ~0.6-1 GB/s for one host core.  The device wins only on
# many concurrent messages: it hashes up to GPU_DIGEST_LANES of them at once.
GPU_LANE_BPS = {"md5": 64 / 0.555e-6, "sha256": 64 / 1.696e-6}
GPU_DIGEST_LANES = 256 * 4 * 64 // 2      # one lane per message, two waves per 64 messages, 4 per SIMD
GPU_LAUNCH_S = 30e-6                      # launch + result copy of one zs3_*_parts call
PCIE_BPS = 50e9                           # one x16 Gen5 link, measured pinned H2D


def digest_on_device(algo: str, n_msgs: int, msg_bytes: int, cpu_threads: int, cpu_Bps: float,
                     resident: bool = False) -> bool:
    """Where the rocm build hashes n_msgs concurrent messages (parts) of about msg_bytes:
    True = zs3_md5_parts / zs3_sha256_parts, False = the host's crypto/md5 and sha256-simd
    (internal/etag/reader.go:114, internal/hash/reader.go:137 unchanged).  Device time =
    one chain per message, GPU_DIGEST_LANES at a time, plus the launch and, unless the
    messages are already in HBM, their PCIe transfer; host time = the messages spread over
    cpu_threads cores at cpu_Bps each.  A single part always stays on the host."""
    if n_msgs <= 1 or msg_bytes <= 0:
        return False
    rounds = -(-n_msgs // GPU_DIGEST_LANES)
    t_dev = rounds * msg_bytes / GPU_LANE_BPS[algo] + GPU_LAUNCH_S
    if not resident:
        t_dev += n_msgs * msg_bytes / PCIE_BPS
    t_cpu = -(-n_msgs // max(1, cpu_threads)) * msg_bytes / cpu_Bps
    return t_dev < t_cpu


def host_digest_Bps(algo: str, nbytes: int = 8 << 20) -> float:
    """One host core's MD5 / SHA-256 rate (the calibration the rule above takes)."""
    import hashlib
    import time
    buf = bytes(nbytes)
    h = hashlib.md5 if algo == "md5" else hashlib.sha256
    h(buf[: 1 << 20]).digest()
    t0 = time.perf_counter()
    h(buf).digest()
    return nbytes / (time.perf_counter() - t0)
