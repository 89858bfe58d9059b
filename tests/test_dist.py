"""world_size-2 gloo test of the multi-GPU partitioning (CPU only).

Each rank encodes + hashes its own contiguous object range with the CPU oracle
(standing in for its GPU), rank 0 gathers the digests and checks that the union
equals the single-process result over all objects, and the timing reduction is a
max over ranks.  No data-path collective exists in the product path.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zs3server_amd.dist import max_over_ranks, object_range, split_range

K, M, BLEN, PER_RANK = 4, 2, 4096, 3
KEY = bytes.fromhex("4be734fa8e238acd263e83e6bb968552040f935da39f441497e09d1322de36a0")


def _digest(oracle, obj):
    shards = oracle.encode_data(K, M, oracle.fill(77, obj, BLEN))
    return oracle.hh256_rows(KEY, shards).reshape(-1)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle_c as oc
    lo, hi = object_range(rank, PER_RANK)
    mine = torch.from_numpy(np.stack([_digest(oc, o) for o in range(lo, hi)]))
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    slow = max_over_ranks([float(rank + 1), 0.5], world)
    if rank == 0:
        q.put((torch.cat(gathered).numpy(), slow))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_split_range_covers_stream():
    for total in (65536, 10, 7, 1):
        for world in (1, 2, 4, 8):
            spans = [split_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_two_ranks_gloo_partition_matches_single_process(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, slow = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.stack([_digest(oracle, o) for o in range(world * PER_RANK)])
    assert np.array_equal(got, want)
    assert slow == [2.0, 0.5]
