"""CPU tests of bench.py's N-GPU launcher.

`python bench.py --gpus N` with no WORLD_SIZE in the environment spawns the N ranks
itself (one process per GPU, gloo rendezvous on 127.0.0.1) and prints rank 0's one JSON
line; it refuses to run (non-zero exit) when fewer than N devices are visible or when
WORLD_SIZE (torch.distributed.run) disagrees with --gpus, so it can never report N GPUs
it did not use.  ZS3_BENCH_DRY_RUN=1 exercises exactly that launcher, the rendezvous, the
barriers and the max-over-ranks reduction without any GPU work.  No GPU is needed here.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "ZS3_BENCH_SAME_DEVICE", "ZS3_BENCH_DRY_RUN")}
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "2", "--warmup", "1"],
                       env=_env(ZS3_BENCH_DRY_RUN="1"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n and out["dry_run"] is True
    assert out["value"] is None
    # rank 0 is a child process, not the launcher (the parent never initialises a GPU)
    assert out["pid"] != os.getpid()
    # the reduction is a max over ranks: the slowest rank sleeps n * 10 ms
    assert out["ms_per_step"] >= 10 * n
    # the roofline says which scope each field has: per-GPU fraction
    # beside the whole-job rate of all ranks' bytes over the slowest rank's kernel time
    rl = out["roofline"]
    assert rl["scope"] == "per_gpu" and rl["n_gpus"] == n
    assert rl["frac_per_gpu"] == rl["frac"]
    assert rl["traffic_scope"] == "per_gpu_per_launch" and rl["kernel_ms_scope"] == "max_over_ranks"
    assert rl["aggregate_peak"] == n * rl["peak"]
    assert rl["aggregate_algo_bytes"] == 65536 * (1 << 20) * 3 // 2 + 65536 * 12 * 32
    # 65 536 objects over n ranks: the aggregate is the ranks' shares over the same time
    assert rl["aggregate_achieved"] == pytest.approx(rl["achieved"] * 65536 / (65536 // n), rel=1e-3)


def test_roofline_block_scopes():
    """One GPU's share and the whole job: frac_per_gpu stays the per-GPU fraction while
    aggregate_achieved sums the ranks' bytes (the --gpus 2 same-device rehearsal line of
    round 5 printed frac 0.343 beside 3 399 GiB/s with nothing saying which was which)."""
    sys.path.insert(0, ROOT)
    import bench
    a = bench.algo_bytes_per_block(8, 4, 1 << 20)
    for n in (1, 2, 4, 8):
        rl = bench.roofline_block(8, 4, 1 << 20, 65536 // n, 65536, n, 18.0 / n, None, None)
        assert rl["frac_per_gpu"] == pytest.approx((65536 // n) * a / 18e-3 * n / 8e12, rel=1e-3)
        assert rl["aggregate_achieved"] == pytest.approx(65536 * a / (18.0 / n) * 1e-6, rel=1e-4)
        assert rl["aggregate_frac"] == pytest.approx(rl["frac_per_gpu"], rel=1e-3)


def test_too_few_devices_fails_loudly():
    """No MI355X in this container: --gpus 2 must exit non-zero, never fall back to 1."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "visible devices" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_fails_loudly():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1", "--warmup", "0"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", ZS3_BENCH_DRY_RUN="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 4" in r.stderr


def test_headline_traffic_is_keyed_by_full_kernel_name():
    """bench.py attaches committed PMC traffic only to the exact kernel instance it runs
    (a stale instance's counters are never reused) and has an entry for every per-GPU
    share of BASELINE config 4 (65 536 objects over N = 1 / 2 / 4 / 8)."""
    sys.path.insert(0, ROOT)
    import bench
    from zs3server_amd.dist import split_range
    k, m, blen = 8, 4, 1 << 20
    for n in (1, 2, 4, 8):
        lo, hi = split_range(65536, n, 0)
        traffic, src = bench.committed_traffic(k, m, hi - lo, blen)
        assert traffic is not None, (n, hi - lo)
        algo = (hi - lo) * bench.algo_bytes_per_block(k, m, blen)
        assert 1.0 <= traffic / algo < 1.02, (n, traffic / algo, src)
    assert bench.committed_traffic(k, m, 1000, blen) == (None, None)  # another instance
