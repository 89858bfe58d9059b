"""world_size-2 run of the bench's partition on the product library (GPU).

bench.py under torch.distributed.run gives rank r the objects dist.split_range(total, N, r)
(BASELINE config 4 split over N GPUs, no data-path collective) and encodes them with one
zs3_encode_batch launch.  Here two ranks (gloo; both on cuda:0, the one GPU of a test box)
run exactly that sequence — Codec, fill_batch(obj0 = first object of the range),
encode_batch in the in-place bpool layout — and rank 0 gathers every rank's parity rows
and bitrot sums.  The reassembled output must equal the oracle's encode of all objects,
and the timing reduction is the bench's max over ranks.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu

K, M, BLEN, TOTAL, SEED = 8, 4, 1 << 16, 13, 4321
S = BLEN // K
R = K + M


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import zs3server_amd as z
    from zs3server_amd.dist import max_over_ranks, split_range
    lo, hi = split_range(TOTAL, world, rank)
    n = hi - lo
    codec = z.Codec(K, M, 1 << 20)
    buf = torch.empty(n * R * S, dtype=torch.uint8, device="cuda:0")
    sums = torch.zeros(n * R * 32, dtype=torch.uint8, device="cuda:0")
    z.fill_batch(buf, R * S, BLEN, n, seed=SEED, obj0=lo)
    codec.encode_batch(buf, R * S, BLEN, n, parity=buf, parity_offset=K * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() != 0, "the product library ran a kernel"
    out = np.zeros((TOTAL, R * S + R * 32), np.uint8)  # this rank's objects, zeros elsewhere
    out[lo:hi, :R * S] = buf.cpu().numpy().reshape(n, R * S)
    out[lo:hi, R * S:] = sums.cpu().numpy().reshape(n, R * 32)
    mine = torch.from_numpy(out.astype(np.int32))
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    slow = max_over_ranks([float(rank + 1)], world)
    if rank == 0:
        q.put((torch.stack(gathered).sum(dim=0).numpy().astype(np.uint8), slow))  # disjoint ranges
    dist.destroy_process_group()


def test_two_ranks_bench_partition_on_gpu(oracle):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, slow = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert slow == [2.0]
    import zs3server_amd as z
    mat = oracle.build_matrix(K, M)
    for o in range(TOTAL):
        shards = oracle.encode_data(K, M, oracle.fill(SEED, o, BLEN), mat)
        assert np.array_equal(got[o, :R * S].reshape(R, S), shards), f"object {o}"
        assert np.array_equal(got[o, R * S:].reshape(R, 32), oracle.hh256_rows(z.MAGIC_HH256_KEY, shards)), f"sums {o}"
