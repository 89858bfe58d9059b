"""Committed golden fixtures (tests/golden/golden.json, made by make_golden.py from
the KAT-pinned oracles): the oracle must reproduce them (CPU), and the device path
must reproduce them through the C ABI without the oracle (GPU)."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def test_oracle_reproduces_golden(oracle):
    key = bytes.fromhex(GOLD["key"])
    for rec in GOLD["encode"]:
        if rec["block_len"] > (1 << 20) + 1:
            continue
        a = oracle.encode_data(rec["k"], rec["m"], oracle.fill(rec["seed"], 0, rec["block_len"]))
        assert hashlib.sha256(a.tobytes()).hexdigest() == rec["shards_sha256"]
        assert [s.tobytes().hex() for s in oracle.hh256_rows(key, a)] == rec["sums"]
    msg = oracle.fill(99, 3, 96)
    for h in GOLD["hh256"]:
        assert oracle.hh256(key, msg[: h["len"]]).hex() == h["sum"]


@pytest.mark.gpu
def test_device_reproduces_golden():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import zs3server_amd as z
    for rec in GOLD["encode"]:
        k, m, n = rec["k"], rec["m"], rec["block_len"]
        S = rec["shard_size"]
        buf = torch.zeros((k + m) * S, dtype=torch.uint8, device="cuda")
        z.fill_batch(buf, (k + m) * S, n, 1, seed=rec["seed"], obj0=0)
        sums = torch.zeros((k + m) * 32, dtype=torch.uint8, device="cuda")
        z.Codec(k, m).encode_batch(buf, (k + m) * S, n, 1, parity=buf, parity_offset=k * S,
                                   parity_stride=(k + m) * S, sums=sums)
        torch.cuda.synchronize()
        host = buf.cpu().numpy()
        assert hashlib.sha256(host.tobytes()).hexdigest() == rec["shards_sha256"], rec
        got = sums.cpu().numpy().reshape(k + m, 32)
        assert [s.tobytes().hex() for s in got] == rec["sums"], rec
        if "parity_hex" in rec:
            assert host[k * S:].tobytes().hex() == rec["parity_hex"]
    msg = torch.zeros(128, dtype=torch.uint8, device="cuda")
    z.fill_batch(msg, 128, 96, 1, seed=99, obj0=3)
    out = torch.zeros(97 * 32, dtype=torch.uint8, device="cuda")
    for h in GOLD["hh256"]:
        z.hh256_batch(msg, 128, h["len"], 1, out, offset=0)
        torch.cuda.synchronize()
        assert out[:32].cpu().numpy().tobytes().hex() == h["sum"], h["len"]
