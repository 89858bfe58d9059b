"""world_size-2 gloo tests of the multi-GPU partitioning (CPU only).

* The bench's object partition: each rank encodes + hashes its own contiguous object
  range with the CPU oracle (standing in for its GPU), rank 0 gathers the digests and
  checks that the union equals the single-process result over all objects, and the
  timing reduction is a max over ranks.
* The end-to-end stream split of zs3_stream_encode_multi (BASELINE config 5): each
  rank takes the block range the LIBRARY's own zs3_split_range gives it (the last rank
  also the partial last block), encodes it with oracle/cpu_ref into the stream's
  output layout (parity of block b at b*m*S, sums at b*(k+m)*32), and the gathered,
  reassembled outputs equal the single-process encode of the whole stream.
No data-path collective exists in the product path.
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


def test_library_split_matches_python_split():
    """zs3_split_range (the C driver's split) == dist.split_range (the bench's)."""
    import zs3server_amd as z
    for total in (65536, 10240, 1000, 7, 1, 0):
        for world in (1, 2, 3, 4, 7, 8):
            for r in range(world):
                assert z.split_range(total, world, r) == split_range(total, world, r)


SK, SM, SBS, SNFULL, STAIL = 8, 4, 1 << 14, 37, 5000


def _stream_input():
    from oracle import oracle_c as oc
    total = SNFULL * SBS + STAIL
    return np.concatenate([oc.fill(91, b, SBS) for b in range(SNFULL + 1)])[:total]


def _encode_range(data, lo, hi, with_tail):
    """Blocks [lo, hi) (+ the tail) of the stream into the full-size output layout."""
    from oracle import cpuref, oracle_c as oc
    R, S = SK + SM, SBS // SK
    nblk = SNFULL + 1
    par = np.zeros(nblk * SM * S, np.uint8)
    sums = np.zeros(nblk * R * 32, np.uint8)
    mat = oc.build_matrix(SK, SM)
    if hi > lo:
        cpuref.encode_hash(SK, SM, mat, data[lo * SBS:], SBS, hi - lo, SBS, par[lo * SM * S:], SM * S,
                           sums[lo * R * 32:], KEY, 1)
    if with_tail:
        sh = oc.encode_data(SK, SM, data[SNFULL * SBS:])
        St = sh.shape[1]
        par[SNFULL * SM * S: SNFULL * SM * S + SM * St] = sh[SK:].reshape(-1)
        sums[SNFULL * R * 32:] = oc.hh256_rows(KEY, sh).reshape(-1)
    return par, sums


def _stream_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import zs3server_amd as z
    data = _stream_input()
    lo, hi = z.split_range(SNFULL, world, rank)
    par, sums = _encode_range(data, lo, hi, rank == world - 1)
    mine = torch.from_numpy(np.concatenate([par, sums]).astype(np.int32))
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    if rank == 0:
        q.put(torch.stack(gathered).sum(dim=0).numpy().astype(np.uint8))  # disjoint ranges: sum = union
    dist.destroy_process_group()


def test_two_ranks_gloo_stream_split_reassembles():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    par, sums = _encode_range(_stream_input(), 0, SNFULL, True)
    assert np.array_equal(got, np.concatenate([par, sums]))


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
