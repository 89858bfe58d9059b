"""world_size-2 run of the bench's partition on the product library (GPU).

bench.py under torch.distributed.run gives rank r the objects dist.split_range(total, N, r)
(BASELINE config 4 split over N GPUs, no data-path collective) and encodes them with one
zs3_encode_batch launch.  Here two ranks (gloo; both on cuda:0, the one GPU of a test box)
run exactly that sequence — Codec, fill_batch(obj0 = first object of the range),
encode_batch in the in-place bpool layout — and rank 0 gathers every rank's parity rows
and bitrot sums.  The reassembled output must equal the oracle's encode of all objects,
and the timing reduction is the bench's max over ranks.  The ranks gather one SHA-256 per
object (its parity-filled stripe and its sums); 13 objects of 64 KiB check every object,
4 098 objects of 1 MiB (2 049 per rank: the bulk k_ehx_ws shape the bench runs on each
rank) check the objects at both ends of each rank's range and a seeded sample against the
oracle.
"""
import hashlib
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu

K, M, SEED = 8, 4, 4321
R = K + M


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, total, blen):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import zs3server_amd as z
    from zs3server_amd.dist import max_over_ranks, split_range
    S = blen // K
    lo, hi = split_range(total, world, rank)
    n = hi - lo
    codec = z.Codec(K, M, 1 << 20)
    buf = torch.empty(n * R * S, dtype=torch.uint8, device="cuda:0")
    sums = torch.zeros(n * R * 32, dtype=torch.uint8, device="cuda:0")
    z.fill_batch(buf, R * S, blen, n, seed=SEED, obj0=lo)
    codec.encode_batch(buf, R * S, blen, n, parity=buf, parity_offset=K * S, parity_stride=R * S, sums=sums)
    torch.cuda.synchronize()
    assert z.last_path() != 0, "the product library ran a kernel"
    hb = buf.cpu().numpy().reshape(n, R * S)
    hs = sums.cpu().numpy().reshape(n, R * 32)
    del buf, sums
    dig = np.zeros((total, 32), np.uint8)  # this rank's objects, zeros elsewhere
    for i in range(n):
        dig[lo + i] = np.frombuffer(hashlib.sha256(hb[i].tobytes() + hs[i].tobytes()).digest(), np.uint8)
    mine = torch.from_numpy(dig.astype(np.int32))
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    slow = max_over_ranks([float(rank + 1)], world)
    if rank == 0:
        q.put((torch.stack(gathered).sum(dim=0).numpy().astype(np.uint8), slow))  # disjoint ranges
    dist.destroy_process_group()


@pytest.mark.parametrize("total,blen", [(13, 1 << 16), (4098, 1 << 20)])
def test_two_ranks_bench_partition_on_gpu(oracle, total, blen):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, total, blen)) for r in range(world)]
    for p in procs:
        p.start()
    got, slow = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert slow == [2.0]
    import zs3server_amd as z
    from zs3server_amd.dist import split_range
    S = blen // K
    if total <= 64:
        check = range(total)
    else:
        ends = set()
        for r in range(world):
            lo, hi = split_range(total, world, r)
            ends |= {lo, lo + 1, hi - 2, hi - 1}
        check = sorted(ends | set(np.random.default_rng(SEED).choice(total, 24, replace=False).tolist()))
    mat = oracle.build_matrix(K, M)
    for o in check:
        shards = oracle.encode_data(K, M, oracle.fill(SEED, o, blen), mat)
        want = hashlib.sha256(shards.tobytes() + oracle.hh256_rows(z.MAGIC_HH256_KEY, shards).tobytes()).digest()
        assert got[o].tobytes() == want, f"object {o}"
